// Batch-1..8 decode GEMV for gfx950: out[M, N] = X[M, K] . W[N, K]^T (+ bias), M <= 8
// (decode-skinny shapes at the low end of the BenchmarkJob concurrency sweep).
//
// At one to four rows a projection has no operand reuse worth an MFMA tile: it is a pure
// HBM stream of the weight.  Each wave owns R consecutive weight rows and walks K with 16-byte
// loads (lane l covers k = 8 l + 512 i), the R row loads of several K steps in flight at once
// (unrolled; no LDS, no barriers, ~30 VGPRs so many waves per SIMD hide the HBM latency).  The
// activation rows (<= 8 x K bf16, read by every wave) are served by L1 / L2.  Each wave reduces
// its M x R fp32 partial dot products across the 64 lanes with xor shuffles and stores them.
#include "common.h"

namespace {

// 8-element bf16 dot product on four v_dot2c_f32_bf16 (fp32 accumulate, no unpacking)
__device__ __forceinline__ float dot8(bf16x8 a, bf16x8 b, float acc) {
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(a, a, 0, 1), __builtin_shufflevector(b, b, 0, 1), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(a, a, 2, 3), __builtin_shufflevector(b, b, 2, 3), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(a, a, 4, 5), __builtin_shufflevector(b, b, 4, 5), acc, false);
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(a, a, 6, 7), __builtin_shufflevector(b, b, 6, 7), acc, false);
}

// SwiGLU operand on the fly: X holds [gate | up] (2K wide); the dot product sees
// bf16(silu(g) * u), bit-identical to act_and_mul followed by the plain GEMV.
__device__ __forceinline__ bf16x8 silu_mul8(bf16x8 g, bf16x8 u) {
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float gf = (float)g[j];
    o[j] = (bf16)(gf / (1.f + __expf(-gf)) * (float)u[j]);
  }
  return o;
}

template <bool ACT>
__device__ __forceinline__ bf16x8 ldx8(const bf16* p, int K) {
  if constexpr (ACT) return silu_mul8(ld8(p), ld8(p + K));
  else return ld8(p);
}

template <int M, int R, int U, bool ACT = false>   // U: K steps in flight (fewer for more rows: VGPR budget)
__global__ __launch_bounds__(256) void gemv_kernel(const bf16* __restrict__ X, int64_t ldx, const bf16* __restrict__ W,
                                                   const bf16* __restrict__ bias, bf16* __restrict__ out, int64_t ldo,
                                                   int N, int K) {
  const int lane = threadIdx.x & 63;
  const int n0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * R;
  if (n0 >= N) return;
  const bf16* wr[R];
#pragma unroll
  for (int r = 0; r < R; ++r) wr[r] = W + (int64_t)min(n0 + r, N - 1) * K;   // clamp: rows past N are computed, not stored
  float acc[M][R];
#pragma unroll
  for (int m = 0; m < M; ++m)
#pragma unroll
    for (int r = 0; r < R; ++r) acc[m][r] = 0.f;

  int k = lane * 8;
  // main body: U K steps (U x R 16-B weight loads per lane) in flight
  for (; k + (U - 1) * 512 < K; k += U * 512) {
    bf16x8 w[U][R], x[U][M];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int r = 0; r < R; ++r) w[u][r] = ld8(wr[r] + k + 512 * u);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int m = 0; m < M; ++m) x[u][m] = ldx8<ACT>(X + m * ldx + k + 512 * u, K);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int m = 0; m < M; ++m)
#pragma unroll
        for (int r = 0; r < R; ++r) acc[m][r] = dot8(x[u][m], w[u][r], acc[m][r]);
  }
  for (; k < K; k += 512) {
    bf16x8 w[R], x[M];
#pragma unroll
    for (int r = 0; r < R; ++r) w[r] = ld8(wr[r] + k);
#pragma unroll
    for (int m = 0; m < M; ++m) x[m] = ldx8<ACT>(X + m * ldx + k, K);
#pragma unroll
    for (int m = 0; m < M; ++m)
#pragma unroll
      for (int r = 0; r < R; ++r) acc[m][r] = dot8(x[m], w[r], acc[m][r]);
  }
#pragma unroll
  for (int m = 0; m < M; ++m)
#pragma unroll
    for (int r = 0; r < R; ++r) acc[m][r] = wave_sum(acc[m][r]);
  // lane (m * R + r) stores element (m, n0 + r)
#pragma unroll
  for (int m = 0; m < M; ++m)
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (lane == m * R + r && n0 + r < N)
        out[(int64_t)m * ldo + n0 + r] = (bf16)(acc[m][r] + (bias ? (float)bias[n0 + r] : 0.f));
}

}  // namespace

// X [M, K] (row stride ldx, 16-byte aligned rows), W [N, K] contiguous, out [M, N] (row stride ldo);
// 1 <= M <= 8, K % 8 == 0.  act = 1: X is the fused gate/up projection [M, 2K] and the operand is
// SiLU(gate) * up (the down projection with the SwiGLU folded into its operand load).
template <bool ACT>
static int gemv_launch(const void* X, int64_t ldx, const void* W, const void* bias, void* out, int64_t ldo, int M,
                       int N, int K, hipStream_t stream) {
  // narrow weights: 2 rows per wave (twice the waves to spread over 256 CUs); long rows (K >= 8192,
  // the down projection) with <= 2 activation rows: 8 K steps in flight per wave
  const bool narrow = N <= 4096, deep = K >= 8192 && M <= 2;
#define GV_L(MV, RV, UV)                                                                                    \
  gemv_kernel<MV, RV, UV, ACT><<<dim3((N + 4 * RV - 1) / (4 * RV)), 256, 0, stream>>>(                     \
      (const bf16*)X, ldx, (const bf16*)W, (const bf16*)bias, (bf16*)out, ldo, N, K)
#define GV(MV)                                                                              \
  if (MV <= 2 && deep) { if (narrow) GV_L(MV, 2, 8); else GV_L(MV, 4, 8); }                \
  else if (narrow) GV_L(MV, 2, (MV <= 4 ? 4 : 2));                                          \
  else GV_L(MV, 4, (MV <= 4 ? 4 : 2))
  switch (M) {
    case 1: GV(1); break;
    case 2: GV(2); break;
    case 3: GV(3); break;
    case 4: GV(4); break;
    case 5: GV(5); break;
    case 6: GV(6); break;
    case 7: GV(7); break;
    default: GV(8); break;
  }
#undef GV_L
#undef GV
  OME_CHECK_LAUNCH();
  return 0;
}

OME_API int ome_gemv(const void* X, int64_t ldx, const void* W, const void* bias, void* out, int64_t ldo, int M, int N,
                     int K, hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (M > 8 || K % 8 || ldx % 8 || K <= 0) return -2;
  return gemv_launch<false>(X, ldx, W, bias, out, ldo, M, N, K, stream);
}

OME_API int ome_gemv_act(const void* X, int64_t ldx, const void* W, const void* bias, void* out, int64_t ldo, int M,
                         int N, int K, hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (M > 8 || K % 8 || ldx % 8 || K <= 0 || ldx < 2 * (int64_t)K) return -2;
  return gemv_launch<true>(X, ldx, W, bias, out, ldo, M, N, K, stream);
}
