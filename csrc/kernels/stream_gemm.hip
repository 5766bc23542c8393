// Weight-streaming bf16 GEMM for decode-shaped batches on gfx950:
//   out[M, N] = X[M, K] . W[N, K]^T (+ bias),  M <= 256
// (hand-tuned MFMA kernels for decode-skinny shapes; second design after
// skinny_gemm.hip, whose LDS-staged weight tiles made it LDS-bound at M = 256).
//
// At M <= 256 every projection of a decode step is bound by streaming the weight from HBM once;
// the activations (<= 2 MB for K = 4096) stay L2-resident.  Design:
//   * one workgroup = 4 waves owns ALL M rows x (4 x 32 NF) weight rows x a K range (split-K
//     when N has too few tiles to fill 256 CUs; fp32 partials + a reduce kernel);
//   * the weight never touches LDS: each wave loads its 32 NF rows straight into the MFMA A
//     operand (v_mfma_f32_32x32x16_bf16, lane l -> weight row l % 32).  K is permuted inside
//     each 64-wide step so lane half h owns k in [32h, 32h + 32): 64 contiguous bytes per lane,
//     consumed as four 16-k MFMA sub-steps.  Two steps of weight are in flight in VGPRs;
//   * the activation step (Mp x 64 bf16) is shared by the 4 waves through a double-buffered LDS
//     image (16-B chunk c of row r at slot c ^ ((r >> 1) & 7): the 32x32x16 B-operand reads and
//     the row-contiguous stores are both conflict-free), one barrier per K step;
//   * per wave and step: 4 x MF x NF MFMAs against 4 x MF ds_read_b128, so LDS runs at <= 50 %
//     of the MFMA time for NF = 2.
#include "common.h"

namespace {

constexpr int KB = 64;   // K per step

__device__ __forceinline__ int xs(int row, int chunk) { return row * 64 + ((chunk ^ ((row >> 1) & 7)) << 3); }

template <int MF, int NF>   // MF: 32-row activation fragments (Mp = 32 MF); NF: 32-row weight fragments per wave
__global__ __launch_bounds__(256) void stream_gemm_kernel(const bf16* __restrict__ X, int64_t ldx,
                                                          const bf16* __restrict__ W, const bf16* __restrict__ bias,
                                                          bf16* __restrict__ out, int64_t ldo, int M, int N, int K,
                                                          int splits, float* __restrict__ ws, int* __restrict__ cnt) {
  constexpr int MP = 32 * MF;
  __shared__ __attribute__((aligned(16))) bf16 sX[2][MP * KB];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, lr = lane & 31, lh = lane >> 5;
  const int tile = blockIdx.x / splits, split = blockIdx.x - tile * splits;
  const int nw = tile * (128 * NF) + wave * (32 * NF);   // this wave's first weight row
  const int steps = K / KB;
  const int s0 = (int)((int64_t)steps * split / splits), s1 = (int)((int64_t)steps * (split + 1) / splits);

  const bf16* wp[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) wp[f] = W + (int64_t)(nw + 32 * f + lr) * K + 32 * lh;

  bf16x8 rx[MF];           // next activation step, staged in registers
  bf16x8 rw[2][NF][4];     // weight steps s (even / odd) in flight
  const bf16* xp[MF];
#pragma unroll
  for (int i = 0; i < MF; ++i) {
    const int c = tid + 256 * i, row = c >> 3;
    xp[i] = row < M ? X + (int64_t)row * ldx + 8 * (c & 7) : nullptr;
  }
  auto load_x = [&](int s) {
#pragma unroll
    for (int i = 0; i < MF; ++i) rx[i] = xp[i] ? ld8(xp[i] + s * KB) : bf16x8{};
  };
  auto store_x = [&](int buf) {
#pragma unroll
    for (int i = 0; i < MF; ++i) {
      const int c = tid + 256 * i;
      *reinterpret_cast<bf16x8*>(&sX[buf][xs(c >> 3, c & 7)]) = rx[i];
    }
  };
  auto load_w = [&](int s, bf16x8 (&r)[NF][4]) {
    const int k0 = s * KB;
#pragma unroll
    for (int f = 0; f < NF; ++f)
#pragma unroll
      for (int j = 0; j < 4; ++j) r[f][j] = ld8(wp[f] + k0 + 8 * j);
  };

  f32x16 acc[NF][MF];
#pragma unroll
  for (int f = 0; f < NF; ++f)
#pragma unroll
    for (int m = 0; m < MF; ++m)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[f][m][r] = 0.f;

  auto compute = [&](int buf, const bf16x8 (&r)[NF][4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bf16x8 b[MF];
#pragma unroll
      for (int m = 0; m < MF; ++m) b[m] = *reinterpret_cast<const bf16x8*>(&sX[buf][xs(32 * m + lr, 4 * lh + j)]);
#pragma unroll
      for (int m = 0; m < MF; ++m)
#pragma unroll
        for (int f = 0; f < NF; ++f) acc[f][m] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(r[f][j], b[m], acc[f][m], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);   // keep each sub-step's operand reads next to its MFMAs (VGPR budget)
    }
  };

  // steps alternate LDS buffer / weight registers; unrolled by two so register indices are static
  const int n = s1 - s0;
  if (n > 0) {
    load_x(s0);
    load_w(s0, rw[0]);
    store_x(0);
    if (n > 1) {
      load_x(s0 + 1);
      load_w(s0 + 1, rw[1]);
    }
    __syncthreads();
  }
  for (int i = 0; i + 1 < n; i += 2) {
    compute(0, rw[0]);
    store_x(1);
    if (i + 2 < n) {
      load_x(s0 + i + 2);
      load_w(s0 + i + 2, rw[0]);
    }
    __syncthreads();
    compute(1, rw[1]);
    if (i + 2 < n) store_x(0);
    if (i + 3 < n) {
      load_x(s0 + i + 3);
      load_w(s0 + i + 3, rw[1]);
    }
    __syncthreads();
  }
  if (n & 1) compute(0, rw[0]);

  // acc[f][m][r] = C[row = 32 m + lr][col = nw + 32 f + 8 (r / 4) + 4 lh + r % 4]
  if (splits > 1) {
    float* part = ws + (int64_t)split * M * N;
#pragma unroll
    for (int m = 0; m < MF; ++m) {
      const int row = 32 * m + lr;
      if (row < M) {
#pragma unroll
        for (int f = 0; f < NF; ++f)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int n = nw + 32 * f + 8 * q + 4 * lh;
            *reinterpret_cast<f32x4*>(part + (int64_t)row * N + n) =
                f32x4{acc[f][m][4 * q], acc[f][m][4 * q + 1], acc[f][m][4 * q + 2], acc[f][m][4 * q + 3]};
          }
      }
    }
    if (cnt == nullptr) return;   // two-launch form: stream_gemm_reduce_kernel sums the slabs
    // In-launch combine (one agent-scope release per writer, one acquire in the tile's last
    // arriver; correct for any placement of a tile's splits over XCDs): the last of the tile's
    // `splits` workgroups sums every slab in fixed split order and stores bf16.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();   // every wave has left the K loop: the LDS image is free for the flag
    int* flag = reinterpret_cast<int*>(&sX[0][0]);
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int t = __hip_atomic_fetch_add(&cnt[tile], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      flag[0] = t == splits - 1;
    }
    __syncthreads();
    if (!flag[0]) return;
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(&cnt[tile], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // re-arm (graph replay)
    }
    __syncthreads();
    constexpr int NWG = 128 * NF, V = NWG / 4;   // tile columns, float4 columns per row
    const int c0 = tile * NWG;
    for (int e = tid; e < M * V; e += 256) {
      const int row = e / V, n = c0 + 4 * (e - row * V);
      f32x4 sum = *reinterpret_cast<const f32x4*>(ws + (int64_t)row * N + n);
      for (int sp = 1; sp < splits; ++sp)
        sum += *reinterpret_cast<const f32x4*>(ws + ((int64_t)sp * M + row) * N + n);
      bf16x4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = (bf16)(sum[r] + (bias ? (float)bias[n + r] : 0.f));
      *reinterpret_cast<bf16x4*>(out + (int64_t)row * ldo + n) = v;
    }
    return;
  }
#pragma unroll
  for (int f = 0; f < NF; ++f)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n = nw + 32 * f + 8 * q + 4 * lh;
      float bv[4] = {0.f, 0.f, 0.f, 0.f};
      if (bias) {
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[r] = (float)bias[n + r];
      }
#pragma unroll
      for (int m = 0; m < MF; ++m) {
        const int row = 32 * m + lr;
        if (row < M) {
          bf16x4 v;
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = (bf16)(acc[f][m][4 * q + r] + bv[r]);
          *reinterpret_cast<bf16x4*>(out + (int64_t)row * ldo + n) = v;
        }
      }
    }
}

// out[m, n] = sum_s ws[s, m, n] (+ bias[n]), fixed split order (deterministic); 8 columns per thread
__global__ __launch_bounds__(256) void stream_gemm_reduce_kernel(const float* __restrict__ ws, const bf16* __restrict__ bias,
                                                                 bf16* __restrict__ out, int64_t ldo, int M, int N,
                                                                 int splits) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x, total = (int64_t)M * N / 8;
  if (i >= total) return;
  const int64_t e = i * 8;
  const int m = (int)(e / N), n = (int)(e - (int64_t)m * N);
  f32x4 a = *reinterpret_cast<const f32x4*>(ws + e), b = *reinterpret_cast<const f32x4*>(ws + e + 4);
  for (int s = 1; s < splits; ++s) {
    const float* p = ws + (int64_t)s * M * N + e;
    a += *reinterpret_cast<const f32x4*>(p);
    b += *reinterpret_cast<const f32x4*>(p + 4);
  }
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    o[j] = (bf16)(a[j] + (bias ? (float)bias[n + j] : 0.f));
    o[j + 4] = (bf16)(b[j] + (bias ? (float)bias[n + 4 + j] : 0.f));
  }
  st8(out + (int64_t)m * ldo + n, o);
}

}  // namespace

// X [M, K] (row stride ldx), W [N, K] contiguous, out [M, N] (row stride ldo); 1 <= M <= 256,
// nf in {1, 2} (2 only for M <= 128), N % (128 nf) == 0, K % 64 == 0, 1 <= splits <= K / 64.  splits > 1 needs ws with
// >= splits * M * N floats; with cnt (>= N / (128 nf) ints, zero before the first launch, re-armed by
// the kernel: HIP-graph replayable) the tile's last split combines the slabs in the same launch,
// without it a second kernel does.
OME_API int ome_stream_gemm(const void* X, int64_t ldx, const void* W, const void* bias, void* out, int64_t ldo, int M,
                            int N, int K, int nf, int splits, float* ws, int* cnt, hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (M > 256 || (nf != 1 && nf != 2) || N % (128 * nf) || K % KB || ldx % 8 || ldo % 8 || splits < 1 ||
      splits > K / KB)
    return -2;
  if (splits > 1 && !ws) return -3;
  if (nf == 2 && M > 128) return -2;   // 256 accumulators per lane at Mp = 256 would spill
  const dim3 grid((N / (128 * nf)) * splits);
  const int mf = (M + 31) / 32;
#define SG(MFV, NFV)                                                                                          \
  stream_gemm_kernel<MFV, NFV><<<grid, 256, 0, stream>>>((const bf16*)X, ldx, (const bf16*)W, (const bf16*)bias, \
                                                         (bf16*)out, ldo, M, N, K, splits, ws, cnt)
#define SG_NF(MFV) \
  if (nf == 1) SG(MFV, 1); else SG(MFV, 2)
  switch (mf) {
    case 1: SG_NF(1); break;
    case 2: SG_NF(2); break;
    case 3: SG_NF(3); break;
    case 4: SG_NF(4); break;
    case 5: SG(5, 1); break;
    case 6: SG(6, 1); break;
    case 7: SG(7, 1); break;
    default: SG(8, 1); break;
  }
#undef SG_NF
#undef SG
  OME_CHECK_LAUNCH();
  if (splits > 1 && cnt == nullptr) {
    const int64_t threads = (int64_t)M * N / 8;
    stream_gemm_reduce_kernel<<<(unsigned)((threads + 255) / 256), 256, 0, stream>>>(ws, (const bf16*)bias, (bf16*)out,
                                                                                     ldo, M, N, splits);
    OME_CHECK_LAUNCH();
  }
  return 0;
}
