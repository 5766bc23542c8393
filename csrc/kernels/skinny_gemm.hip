// Decode-shaped ("skinny") bf16 GEMM for gfx950: out[M, N] = X[M, K] . W[N, K]^T (+ bias), M <= 256
// ("hand-tuned MFMA kernels for decode-skinny shapes").
//
// Why: with <= 256 rows the library GEMMs tile the OUTPUT (256 x 128 / 128 x 128 tiles), which
// for the QKV / O / down projections of an 8B model is 32-96 tiles -- a fraction of the 256 CUs --
// so they stream the weights at 1.5-2.5 TB/s.  Here one workgroup owns ALL rows x 64 weight rows
// and, when the weight has too few 64-row tiles to fill the chip, a 1/splits slice of K
// (split-K); every weight byte is read from HBM exactly once, the activations (<= 256 x K bf16,
// L2-resident) are re-read per tile.
//
// Workgroup = 4 waves, tile = Mp (64 / 128 / 256) rows x 64 weight rows, K consumed 64 at a time:
//   * global -> registers -> LDS (X: Mp x 64, W: 64 x 64 bf16, 16-byte chunks xor-swizzled by
//     row so the MFMA operand reads are conflict-free); the next K step's loads are issued
//     before the current step's MFMAs;
//   * wave w owns rows [w * Mp / 4, +Mp / 4) and all 64 weight rows: C^T blocks computed by
//     v_mfma_f32_16x16x32_bf16 with A = 16 weight rows and B = 16 activation rows, both plain
//     16-byte LDS reads (lane l: row l % 16, k-chunk l / 16);
//   * epilogue: splits == 1 -> (+ bias) -> bf16, 8-byte stores; splits > 1 -> fp32 partial tile to
//     the workspace, device-scope release fence, tile counter atomic; the LAST split of a tile sums
//     the partials in fixed split order (deterministic), adds the bias, stores bf16 and re-arms
//     the counter (so the launch is HIP-graph replayable).
#include "common.h"

namespace {

constexpr int NT = 64;   // weight rows per workgroup
constexpr int KB = 64;   // K per step (8 chunks of 8 bf16)

__device__ __forceinline__ int sw(int row, int chunk) { return row * 8 + (chunk ^ (row & 7)); }

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

template <int MB>   // 16-row activation blocks per wave: Mp = 64 * MB
__global__ __launch_bounds__(256) void skinny_gemm_kernel(const bf16* __restrict__ X, int64_t ldx,
                                                          const bf16* __restrict__ W, const bf16* __restrict__ bias,
                                                          bf16* __restrict__ out, int64_t ldo, int M, int N, int K,
                                                          int splits, float* __restrict__ ws, int* __restrict__ cnt) {
  constexpr int MP = 64 * MB, XL = MP * 8 / 256;   // 16-byte X chunks per thread per step
  __shared__ __attribute__((aligned(16))) bf16 sX[MP * KB];
  __shared__ __attribute__((aligned(16))) bf16 sW[NT * KB];
  __shared__ int s_last;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int tile = blockIdx.x / splits, split = blockIdx.x - tile * splits;
  const int n0 = tile * NT;
  const int steps = K / KB;
  const int s0 = (int)((int64_t)steps * split / splits), s1 = (int)((int64_t)steps * (split + 1) / splits);

  bf16x8 rx[XL], rw[2];
  auto load = [&](int s) {
    const int k0 = s * KB;
#pragma unroll
    for (int i = 0; i < XL; ++i) {
      const int c = tid + 256 * i, row = c >> 3, ch = c & 7;
      rx[i] = row < M ? ld8(X + (int64_t)row * ldx + k0 + 8 * ch) : bf16x8{};
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + 256 * i, row = c >> 3, ch = c & 7;
      rw[i] = ld8(W + (int64_t)(n0 + row) * K + k0 + 8 * ch);
    }
  };

  f32x4 acc[4][MB];
#pragma unroll
  for (int nb = 0; nb < 4; ++nb)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) acc[nb][mb] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int r0 = wave * 16 * MB, lr = lane & 15, lg = lane >> 4;
  if (s0 < s1) load(s0);
  for (int s = s0; s < s1; ++s) {
    __syncthreads();   // the previous step's LDS reads are done
#pragma unroll
    for (int i = 0; i < XL; ++i) {
      const int c = tid + 256 * i;
      *reinterpret_cast<bf16x8*>(&sX[sw(c >> 3, c & 7) * 8]) = rx[i];
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + 256 * i;
      *reinterpret_cast<bf16x8*>(&sW[sw(c >> 3, c & 7) * 8]) = rw[i];
    }
    __syncthreads();
    if (s + 1 < s1) load(s + 1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = 4 * kk + lg;
      bf16x8 a[4], b[MB];
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) a[nb] = *reinterpret_cast<const bf16x8*>(&sW[sw(nb * 16 + lr, ch) * 8]);
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) b[mb] = *reinterpret_cast<const bf16x8*>(&sX[sw(r0 + mb * 16 + lr, ch) * 8]);
#pragma unroll
      for (int nb = 0; nb < 4; ++nb)
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) acc[nb][mb] = mfma16(a[nb], b[mb], acc[nb][mb]);
    }
  }

  // acc[nb][mb][r] = C[m = r0 + 16 mb + lr][n = n0 + 16 nb + 4 lg + r]
  if (splits > 1) {
    float* part = ws + ((int64_t)tile * splits + split) * MP * NT;
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
        *reinterpret_cast<f32x4*>(part + (r0 + 16 * mb + lr) * NT + 16 * nb + 4 * lg) = acc[nb][mb];
    __threadfence();   // release the partial tile (device scope: other XCDs' L2s)
    __syncthreads();
    if (tid == 0) s_last = atomicAdd(&cnt[tile], 1) == splits - 1;
    __syncthreads();
    if (!s_last) return;
    __threadfence();   // acquire the other splits' partials
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) {
        f32x4 sum = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int p = 0; p < splits; ++p)   // fixed order: deterministic
          sum += *reinterpret_cast<const f32x4*>(ws + ((int64_t)tile * splits + p) * MP * NT +
                                                 (r0 + 16 * mb + lr) * NT + 16 * nb + 4 * lg);
        acc[nb][mb] = sum;
      }
    if (tid == 0) cnt[tile] = 0;   // re-arm for the next launch / graph replay
  }
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) {
    const int n = n0 + 16 * nb + 4 * lg;
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (bias) {
#pragma unroll
      for (int r = 0; r < 4; ++r) bv[r] = (float)bias[n + r];
    }
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const int m = r0 + 16 * mb + lr;
      if (m < M) {
        bf16x4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = (bf16)(acc[nb][mb][r] + bv[r]);
        *reinterpret_cast<bf16x4*>(out + (int64_t)m * ldo + n) = v;
      }
    }
  }
}

}  // namespace

// X [M, K] (row stride ldx, 16-byte aligned rows), W [N, K] contiguous, out [M, N] (row stride ldo);
// M <= 256, N % 64 == 0, K % 64 == 0.  splits > 1 needs ws (>= N / 64 * splits * Mp * 64 floats,
// Mp = 64 / 128 / 256 by M) and cnt (>= N / 64 ints, zero on first use; re-armed by the kernel).
OME_API int ome_skinny_gemm(const void* X, int64_t ldx, const void* W, const void* bias, void* out, int64_t ldo, int M,
                            int N, int K, int splits, float* ws, int* cnt, hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (M > 256 || N % NT || K % KB || ldx % 8 || ldo % 4 || splits < 1 || splits > K / KB) return -2;
  if (splits > 1 && (!ws || !cnt)) return -3;
  dim3 grid((N / NT) * splits);
#define SKINNY(MBV)                                                                                          \
  skinny_gemm_kernel<MBV><<<grid, 256, 0, stream>>>((const bf16*)X, ldx, (const bf16*)W, (const bf16*)bias, \
                                                    (bf16*)out, ldo, M, N, K, splits, ws, cnt)
  if (M <= 64) SKINNY(1);
  else if (M <= 128) SKINNY(2);
  else SKINNY(4);
#undef SKINNY
  OME_CHECK_LAUNCH();
  return 0;
}
