// Mamba-2 (selective state space) kernels for hybrid models (NemotronH; reference catalog
// ``NemotronHForCausalLM`` runtimes), CDNA4 / gfx950.
//
//   ome_ssm_conv1d       : causal depthwise conv (kernel K <= 8) + SiLU over a varlen batch of
//                          sequences, continuing from / updating each sequence's conv state
//   ome_dyn_conv1d       : the same with per-row (input-generated) taps (Jet-Nemotron JetBlock)
//   ome_ssm_scan         : the selective scan  h <- exp(dt*A) h + dt * B x,  y = C.h + D x
//                          (dt = softplus(dt + dt_bias) clamped below), recurrent over the rows of
//                          each sequence, state in fp32 per (slot, head, p, n)
//   ome_gated_rmsnorm    : out = w * groupRMSNorm(y * silu(z))  (norm_first: w[:group] * groupRMSNorm(y) * silu(z))
//
// Sequences are described by cu[S+1] (row ranges), slot[S] (state row) and reset[S] (1 = start
// from zero state: a sequence's first prefill chunk).  Decode is the S = batch, one-row case, so
// the same launches are captured in the decode HIP graph.
//
// Scan layout: one 256-thread workgroup per (head, sequence); the head's P x N state is split so
// that TPP = 256 / P consecutive lanes own one p row, NPT = N / TPP states each, held in VGPRs for
// the whole sequence.  Per row every lane reads its NPT B and C values straight from global (the
// TPP lanes of a p row read disjoint slices; the 256/TPP rows of the block read the same lines, so
// each B/C line is fetched once per wave through the vector cache) -- no LDS and no barrier in the
// time loop; y = C.h is a TPP-lane shuffle reduction.
#include "common.h"

#include <cstdlib>

namespace {

typedef float f32v4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float softplus_f(float x) { return x > 20.f ? x : log1pf(__expf(x)); }
__device__ __forceinline__ float silu_f(float x) { return x / (1.f + __expf(-x)); }

template <int K>
__global__ __launch_bounds__(256) void ssm_conv1d_kernel(const bf16* __restrict__ x, int64_t x_stride,
                                                         const bf16* __restrict__ w, const bf16* __restrict__ bias,
                                                         bf16* __restrict__ out, int64_t out_stride,
                                                         bf16* __restrict__ state, const int* __restrict__ cu,
                                                         const int* __restrict__ slot, const int* __restrict__ reset,
                                                         int C) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  const int s = blockIdx.y;
  if (c >= C) return;
  const int r0 = cu[s], r1 = cu[s + 1];
  if (r1 <= r0) return;
  bf16* st = state + ((int64_t)slot[s] * C + c) * (K - 1);
  float win[K - 1];
  const bool fresh = reset[s] != 0;
#pragma unroll
  for (int j = 0; j < K - 1; ++j) win[j] = fresh ? 0.f : (float)st[j];
  float wt[K];
#pragma unroll
  for (int j = 0; j < K; ++j) wt[j] = (float)w[(int64_t)c * K + j];
  const float b = bias != nullptr ? (float)bias[c] : 0.f;
  for (int r = r0; r < r1; ++r) {
    const float v = (float)x[(int64_t)r * x_stride + c];
    float acc = b + wt[K - 1] * v;
#pragma unroll
    for (int j = 0; j < K - 1; ++j) acc += wt[j] * win[j];
#pragma unroll
    for (int j = 0; j < K - 2; ++j) win[j] = win[j + 1];
    win[K - 2] = v;
    out[(int64_t)r * out_stride + c] = (bf16)silu_f(acc);
  }
#pragma unroll
  for (int j = 0; j < K - 1; ++j) st[j] = (bf16)win[j];
}

// Dynamic (input-conditioned) causal depthwise conv + SiLU (Jet-Nemotron's JetBlock value path):
// every row r brings its own taps kern[r][(c / cpk) * K + j] (cpk channels share a kernel: 1 =
// per-channel, head_v_dim = per-head), tap K-1 on the current row.  Same varlen / state contract
// as ssm_conv1d_kernel.
template <int K>
__global__ __launch_bounds__(256) void dyn_conv1d_kernel(const bf16* __restrict__ x, int64_t x_stride,
                                                         const bf16* __restrict__ kern, int64_t k_stride, int cpk,
                                                         bf16* __restrict__ out, int64_t out_stride,
                                                         bf16* __restrict__ state, const int* __restrict__ cu,
                                                         const int* __restrict__ slot, const int* __restrict__ reset,
                                                         int C) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  const int s = blockIdx.y;
  if (c >= C) return;
  const int r0 = cu[s], r1 = cu[s + 1];
  if (r1 <= r0) return;
  bf16* st = state + ((int64_t)slot[s] * C + c) * (K - 1);
  float win[K - 1];
  const bool fresh = reset[s] != 0;
#pragma unroll
  for (int j = 0; j < K - 1; ++j) win[j] = fresh ? 0.f : (float)st[j];
  const int64_t kc = (int64_t)(c / cpk) * K;
  for (int r = r0; r < r1; ++r) {
    const float v = (float)x[(int64_t)r * x_stride + c];
    const bf16* kr = kern + (int64_t)r * k_stride + kc;
    float acc = (float)kr[K - 1] * v;
#pragma unroll
    for (int j = 0; j < K - 1; ++j) acc += (float)kr[j] * win[j];
#pragma unroll
    for (int j = 0; j < K - 2; ++j) win[j] = win[j + 1];
    win[K - 2] = v;
    out[(int64_t)r * out_stride + c] = (bf16)silu_f(acc);
  }
#pragma unroll
  for (int j = 0; j < K - 1; ++j) st[j] = (bf16)win[j];
}

template <int NPT, bool NT>
__global__ __launch_bounds__(256) void ssm_scan_kernel(
    const bf16* __restrict__ x, int64_t x_stride, const bf16* __restrict__ dt, int64_t dt_stride,
    const bf16* __restrict__ B, const bf16* __restrict__ Cm, int64_t bc_stride, const float* __restrict__ A,
    const float* __restrict__ D, const float* __restrict__ dt_bias, float dt_min, float* __restrict__ state,
    bf16* __restrict__ y, int64_t y_stride, const int* __restrict__ cu, const int* __restrict__ slot,
    const int* __restrict__ reset, int H, int P, int N, int G, int PB) {
  // a workgroup owns PB of the head's P rows (P / PB workgroups per head and sequence)
  const int split = P / PB;
  const int h = blockIdx.x / split, s = blockIdx.y;
  const int r0 = cu[s], r1 = cu[s + 1];
  if (r1 <= r0) return;
  const int TPP = 256 / PB;
  const int p = (blockIdx.x % split) * PB + threadIdx.x / TPP, q = threadIdx.x % TPP;
  const int n0 = q * NPT;
  const int g = h / (H / G);
  // state row: NPT contiguous fp32 per lane, a wave covers one contiguous 64*NPT*4-byte span:
  // moved with 16-B vector loads / stores (decode is bound by this state traffic)
  f32v4* st4 = reinterpret_cast<f32v4*>(state + (((int64_t)slot[s] * H + h) * P + p) * N + n0);
  float hs[NPT];
  if (reset[s] != 0) {
#pragma unroll
    for (int j = 0; j < NPT; ++j) hs[j] = 0.f;
  } else {
#pragma unroll
    for (int j = 0; j < NPT / 4; ++j) {
      const f32v4 v = NT ? __builtin_nontemporal_load(st4 + j) : st4[j];
      hs[4 * j] = v.x, hs[4 * j + 1] = v.y, hs[4 * j + 2] = v.z, hs[4 * j + 3] = v.w;
    }
  }
  const float a = A[h], d = D[h], db = dt_bias[h];
  const int64_t boff = (int64_t)g * N + n0;
  // software pipeline: the next row's dt / x / B / C are loaded while this row's FMAs run
  bf16x8 bn[NPT / 8], cn[NPT / 8];
  float dtn = 0.f, xn = 0.f;
  auto fetch = [&](int r) {
    dtn = (float)dt[(int64_t)r * dt_stride + h];
    xn = (float)x[(int64_t)r * x_stride + h * P + p];
#pragma unroll
    for (int j = 0; j < NPT / 8; ++j) {
      bn[j] = ld8(B + (int64_t)r * bc_stride + boff + 8 * j);
      cn[j] = ld8(Cm + (int64_t)r * bc_stride + boff + 8 * j);
    }
  };
  fetch(r0);
  for (int r = r0; r < r1; ++r) {
    bf16x8 bv[NPT / 8], cv[NPT / 8];
#pragma unroll
    for (int j = 0; j < NPT / 8; ++j) bv[j] = bn[j], cv[j] = cn[j];
    const float dtr = dtn, xv = xn;
    if (r + 1 < r1) fetch(r + 1);
    const float dtv = fmaxf(softplus_f(dtr + db), dt_min);
    const float dA = __expf(dtv * a);
    const float dx = dtv * xv;
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < NPT / 8; ++j)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        hs[8 * j + k] = hs[8 * j + k] * dA + dx * (float)bv[j][k];
        acc += (float)cv[j][k] * hs[8 * j + k];
      }
    for (int off = 1; off < TPP; off <<= 1) acc += __shfl_xor(acc, off);
    if (q == 0) y[(int64_t)r * y_stride + h * P + p] = (bf16)(acc + d * xv);
  }
#pragma unroll
  for (int j = 0; j < NPT / 4; ++j)
  {
    const f32v4 v{hs[4 * j], hs[4 * j + 1], hs[4 * j + 2], hs[4 * j + 3]};
    if constexpr (NT) {
      __builtin_nontemporal_store(v, st4 + j);
    } else {
      st4[j] = v;
    }
  }
}

__global__ __launch_bounds__(256) void gated_rmsnorm_kernel(const bf16* __restrict__ y, int64_t y_stride,
                                                            const bf16* __restrict__ z, int64_t z_stride,
                                                            const bf16* __restrict__ w, bf16* __restrict__ out,
                                                            int64_t out_stride, int group, float eps, int norm_first) {
  __shared__ float red[4];
  const int row = blockIdx.y, g0 = blockIdx.x * group;
  const bf16* yr = y + (int64_t)row * y_stride + g0;
  const bf16* zr = z + (int64_t)row * z_stride + g0;
  float ss = 0.f;
  for (int i = threadIdx.x; i < group; i += 256) {
    const float v = norm_first ? (float)yr[i] : (float)yr[i] * silu_f((float)zr[i]);
    ss += v * v;
  }
  const float tot = block_sum<256>(ss, red);
  const float rs = rsqrtf(tot / (float)group + eps);
  bf16* orow = out + (int64_t)row * out_stride + g0;
  for (int i = threadIdx.x; i < group; i += 256) {
    if (norm_first) {   // Qwen3-Next: w (per group channel) * norm(y), then * silu(z)
      const float t = (float)(bf16)((float)(bf16)((float)yr[i] * rs) * (float)w[i]);
      orow[i] = (bf16)(t * silu_f((float)zr[i]));
    } else {
      const float v = (float)yr[i] * silu_f((float)zr[i]) * rs;
      orow[i] = (bf16)((float)(bf16)v * (float)w[g0 + i]);  // HF: normalise, cast, then scale by w
    }
  }
}

}  // namespace

OME_API int ome_ssm_conv1d(const void* x, int64_t x_stride, const void* w, const void* bias, void* out,
                           int64_t out_stride, void* state, const int* cu, const int* slot, const int* reset, int S,
                           int C, int K, hipStream_t stream) {
  if (S <= 0 || C <= 0) return 0;
  dim3 grid((C + 255) / 256, S);
#define CONV_CASE(KK)                                                                                         \
  case KK:                                                                                                     \
    ssm_conv1d_kernel<KK><<<grid, 256, 0, stream>>>((const bf16*)x, x_stride, (const bf16*)w, (const bf16*)bias, \
                                                    (bf16*)out, out_stride, (bf16*)state, cu, slot, reset, C);  \
    break;
  switch (K) {
    CONV_CASE(2)
    CONV_CASE(3)
    CONV_CASE(4)
    CONV_CASE(5)
    CONV_CASE(6)
    default:
      return -2;
  }
#undef CONV_CASE
  OME_CHECK_LAUNCH();
  return 0;
}

OME_API int ome_dyn_conv1d(const void* x, int64_t x_stride, const void* kern, int64_t k_stride, int cpk, void* out,
                           int64_t out_stride, void* state, const int* cu, const int* slot, const int* reset, int S,
                           int C, int K, hipStream_t stream) {
  if (S <= 0 || C <= 0) return 0;
  if (cpk <= 0 || C % cpk) return -3;
  dim3 grid((C + 255) / 256, S);
#define DCONV_CASE(KK)                                                                                         \
  case KK:                                                                                                      \
    dyn_conv1d_kernel<KK><<<grid, 256, 0, stream>>>((const bf16*)x, x_stride, (const bf16*)kern, k_stride, cpk, \
                                                    (bf16*)out, out_stride, (bf16*)state, cu, slot, reset, C);   \
    break;
  switch (K) {
    DCONV_CASE(2)
    DCONV_CASE(3)
    DCONV_CASE(4)
    DCONV_CASE(5)
    DCONV_CASE(6)
    default:
      return -2;
  }
#undef DCONV_CASE
  OME_CHECK_LAUNCH();
  return 0;
}

OME_API int ome_ssm_scan(const void* x, int64_t x_stride, const void* dt, int64_t dt_stride, const void* B,
                         const void* Cm, int64_t bc_stride, const float* A, const float* D, const float* dt_bias,
                         float dt_min, float* state, void* y, int64_t y_stride, const int* cu, const int* slot,
                         const int* reset, int S, int H, int P, int N, int G, hipStream_t stream) {
  if (S <= 0) return 0;
  if (P <= 0 || 256 % P != 0 || H % G != 0) return -2;
  // rows per workgroup: the whole head (PB = P).  Splitting a head's rows over more workgroups
  // (PB = P/4, 8 states per lane) measured SLOWER for 2 x 512-row prefill on gfx950 (812 vs 550 us,
  // scripts/ssm_scan_bench.py): the row loop is latency-bound per step, not occupancy-bound.
  const char* pbe = getenv("OME_SSM_PB");
  const int PB = pbe != nullptr && atoi(pbe) > 0 && P % atoi(pbe) == 0 ? atoi(pbe) : P;
  const int tpp = 256 / PB;
  if (N % tpp != 0) return -2;
  const int npt = N / tpp;
  dim3 grid(H * (P / PB), S);
#define SCAN_CASE(NN)                                                                                          \
  case NN:                                                                                                      \
    if (nt)                                                                                                     \
      ssm_scan_kernel<NN, true><<<grid, 256, 0, stream>>>((const bf16*)x, x_stride, (const bf16*)dt, dt_stride,  \
                                                          (const bf16*)B, (const bf16*)Cm, bc_stride, A, D,      \
                                                          dt_bias, dt_min, state, (bf16*)y, y_stride, cu, slot,  \
                                                          reset, H, P, N, G, PB);                                \
    else                                                                                                        \
      ssm_scan_kernel<NN, false><<<grid, 256, 0, stream>>>((const bf16*)x, x_stride, (const bf16*)dt, dt_stride, \
                                                           (const bf16*)B, (const bf16*)Cm, bc_stride, A, D,     \
                                                           dt_bias, dt_min, state, (bf16*)y, y_stride, cu, slot, \
                                                           reset, H, P, N, G, PB);                               \
    break;
  const char* nte = getenv("OME_SSM_NT");  // state I/O: 1 = non-temporal, 0 = plain (default)
  const bool nt = nte != nullptr && atoi(nte) != 0;
  switch (npt) {
    SCAN_CASE(8)
    SCAN_CASE(16)
    SCAN_CASE(32)
    SCAN_CASE(64)
    default:
      return -3;
  }
#undef SCAN_CASE
  OME_CHECK_LAUNCH();
  return 0;
}

OME_API int ome_gated_rmsnorm(const void* y, int64_t y_stride, const void* z, int64_t z_stride, const void* w,
                              void* out, int64_t out_stride, int rows, int I, int group, float eps,
                              int norm_first, hipStream_t stream) {
  if (rows <= 0) return 0;
  if (group <= 0 || I % group != 0) return -2;
  dim3 grid(I / group, rows);
  gated_rmsnorm_kernel<<<grid, 256, 0, stream>>>((const bf16*)y, y_stride, (const bf16*)z, z_stride,
                                                 (const bf16*)w, (bf16*)out, out_stride, group, eps,
                                                 norm_first);
  OME_CHECK_LAUNCH();
  return 0;
}
