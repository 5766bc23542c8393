// Mixture-of-Experts kernels (SURVEY.md §2.9 K10 routing + K11 grouped GEMM) for gfx950.
//
//   ome_moe_route   : gate logits [T, E] -> softmax (or sigmoid) -> top-k ids / weights,
//                     optional renormalisation; one wave per token, E <= 512, k <= 16.
//   ome_moe_align   : counting sort of the T*k assignments by expert -> expert_offsets [E+1],
//                     sorted_ids [T*k] (flat assignment index t*k+j) and its inverse, all on the
//                     device (graph-capturable: no host sync on the per-expert counts).
//   ome_moe_gemm    : grouped GEMM  out[p, :] = A[row(p), :] @ W[e(p)]^T  over the sorted
//                     assignments p; A rows are gathered through sorted_ids / k (gate_up) or
//                     read in sorted order (down).  64x64 MFMA tiles, tiles of an expert never
//                     straddle experts; each workgroup finds its (expert, m-tile) by scanning
//                     the offsets, so the grid is a static upper bound.
//   ome_moe_combine : out[t] = sum_j w[t, j] * Y[inv[t*k + j]]   (fp32 accumulate)
#include "common.h"

#include <cstdlib>

#ifndef OME_NEG_INF
#define OME_NEG_INF (-__builtin_inff())
#endif

// ------------------------------------------------------------------------------------------
// routing
// ------------------------------------------------------------------------------------------
// group_mode: 0 = plain top-k; 1 = DeepSeek-V2 "group_limited_greedy" (group score = max);
// 2 = DeepSeek-V3 "noaux_tc" (group score = sum of the group's top-2 biased scores).  Experts are
// chosen on score + bias (``e_score_correction_bias``) restricted to the best ``topk_group``
// groups (other experts score 0, as in the HF reference); weights are the unbiased scores.
template <typename T>
__global__ __launch_bounds__(256) void moe_route_kernel(const T* __restrict__ logits, int64_t stride, int n_tok,
                                                        int E, int k, int renorm, int scoring,
                                                        const float* __restrict__ bias, int n_group, int topk_group,
                                                        int group_mode, float* __restrict__ topk_w,
                                                        int* __restrict__ topk_ids) {
  __shared__ float s_key[4][512];
  __shared__ int s_gsel[4][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + wave;
  if (t >= n_tok) return;
  constexpr int MAXV = 8;  // E <= 512
  float v[MAXV], key[MAXV];
  const T* row = logits + (int64_t)t * stride;
  float mx = OME_NEG_INF;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int e = lane + 64 * i;
    v[i] = e < E ? (float)row[e] : OME_NEG_INF;
    mx = fmaxf(mx, v[i]);
  }
  mx = wave_max(mx);
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int e = lane + 64 * i;
    float p;
    if (scoring == 0) p = e < E ? __expf(v[i] - mx) : 0.f;        // softmax numerator
    else p = e < E ? 1.f / (1.f + __expf(-v[i])) : -1.f;           // sigmoid score
    v[i] = p;
    sum += (e < E && scoring == 0) ? p : 0.f;
  }
  if (scoring == 0) {
    sum = wave_sum(sum);
    const float inv = 1.f / sum;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) v[i] *= inv;
  }
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int e = lane + 64 * i;
    key[i] = e < E ? v[i] + (bias ? bias[e] : 0.f) : -3.f;
  }
  if (group_mode && n_group > 1) {
    const int gs = E / n_group;
#pragma unroll
    for (int i = 0; i < MAXV; ++i)
      if (lane + 64 * i < E) s_key[wave][lane + 64 * i] = key[i];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    float gscore = OME_NEG_INF;
    if (lane < n_group) {
      float b1 = OME_NEG_INF, b2 = OME_NEG_INF;
      for (int j = 0; j < gs; ++j) {
        const float x = s_key[wave][lane * gs + j];
        if (x > b1) {
          b2 = b1;
          b1 = x;
        } else if (x > b2) {
          b2 = x;
        }
      }
      gscore = group_mode == 1 ? b1 : b1 + (gs > 1 ? b2 : 0.f);
    }
    int chosen = 0;  // bit set on the lanes whose group is selected
    for (int j = 0; j < topk_group; ++j) {
      float best = gscore;
      int bi = lane < n_group ? lane : 1 << 30;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float ob = __shfl_xor(best, o);
        const int oi = __shfl_xor(bi, o);
        if (ob > best || (ob == best && oi < bi)) {
          best = ob;
          bi = oi;
        }
      }
      if (lane == bi) {
        chosen = 1;
        gscore = OME_NEG_INF;
      }
    }
    s_gsel[wave][lane] = chosen;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int e = lane + 64 * i;
      if (e < E && !s_gsel[wave][e / gs]) key[i] = 0.f;
    }
  }
  float picked_sum = 0.f;
  for (int j = 0; j < k; ++j) {
    // argmax over the wave on the selection key (ties -> lowest expert id)
    float best = -4.f, bw = 0.f;
    int bi = 1 << 30;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int e = lane + 64 * i;
      if (e < E && (key[i] > best || (key[i] == best && e < bi))) {
        best = key[i];
        bw = v[i];
        bi = e;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ob = __shfl_xor(best, o);
      const float ow = __shfl_xor(bw, o);
      const int oi = __shfl_xor(bi, o);
      if (ob > best || (ob == best && oi < bi)) {
        best = ob;
        bw = ow;
        bi = oi;
      }
    }
    if (bi >= E) {   // no key beat the floor (NaN logits): still emit a valid expert id
      bi = j < E ? j : E - 1;
      bw = 0.f;
    }
    if (lane == 0) {
      topk_w[(int64_t)t * k + j] = bw;
      topk_ids[(int64_t)t * k + j] = bi;
    }
    picked_sum += bw;
#pragma unroll
    for (int i = 0; i < MAXV; ++i)  // remove the winner (static register indexing)
      if (lane + 64 * i == bi) key[i] = -5.f;
  }
  if (renorm && lane == 0) {
    const float inv = 1.f / (picked_sum + 1e-20f);
    for (int j = 0; j < k; ++j) topk_w[(int64_t)t * k + j] *= inv;
  }
}

OME_API int ome_moe_route(const void* logits, int is_bf16, int64_t stride, int n_tok, int E, int k, int renorm,
                          int scoring, const float* bias, int n_group, int topk_group, int group_mode,
                          float* topk_w, int* topk_ids, hipStream_t stream) {
  if (n_tok <= 0) return 0;
  if (E > 512 || k > E || k <= 0) return -2;
  if (group_mode && n_group > 1 && (E % n_group || n_group > 64 || topk_group > n_group)) return -2;
  const int g = (n_tok + 3) / 4;
  if (is_bf16)
    moe_route_kernel<bf16><<<g, 256, 0, stream>>>((const bf16*)logits, stride, n_tok, E, k, renorm, scoring, bias,
                                                  n_group, topk_group, group_mode, topk_w, topk_ids);
  else
    moe_route_kernel<float><<<g, 256, 0, stream>>>((const float*)logits, stride, n_tok, E, k, renorm, scoring, bias,
                                                   n_group, topk_group, group_mode, topk_w, topk_ids);
  OME_CHECK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------------------------------------
// alignment (counting sort by expert), single workgroup
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void moe_align_kernel(const int* __restrict__ topk_ids, int n, int E,
                                                         int* __restrict__ offsets, int* __restrict__ sorted_ids,
                                                         int* __restrict__ inv) {
  extern __shared__ int sh[];  // [E] counts then [E] cursors
  int* cnt = sh;
  int* cur = sh + E;
  for (int e = threadIdx.x; e < E; e += blockDim.x) cnt[e] = 0;
  __syncthreads();
  // ids outside [0, E) (never produced by moe_route) are clamped rather than indexing LDS out of range
  for (int i = threadIdx.x; i < n; i += blockDim.x) atomicAdd(&cnt[min(max(topk_ids[i], 0), E - 1)], 1);
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int e = 0; e < E; ++e) {
      offsets[e] = acc;
      cur[e] = acc;
      acc += cnt[e];
    }
    offsets[E] = acc;
  }
  __syncthreads();
  // stable within an expert is not required (the combine uses the inverse map)
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int p = atomicAdd(&cur[min(max(topk_ids[i], 0), E - 1)], 1);
    sorted_ids[p] = i;
    inv[i] = p;
  }
}

OME_API int ome_moe_align(const int* topk_ids, int n, int E, int* offsets, int* sorted_ids, int* inv,
                          hipStream_t stream) {
  if (n <= 0) {
    return hipMemsetAsync(offsets, 0, (E + 1) * sizeof(int), stream);
  }
  moe_align_kernel<<<1, 1024, 2 * E * sizeof(int), stream>>>(topk_ids, n, E, offsets, sorted_ids, inv);
  OME_CHECK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------------------------------------
// grouped GEMM: 64x64 output tile per 256-thread workgroup, BK = 32, MFMA 16x16x32 bf16.
// Waves as 2(M) x 2(N), each 32x32 = 2x2 MFMA tiles.  LDS rows padded to 40 bf16 (80 B) so
// the 16 rows a ds_read_b128 group touches start on distinct bank quads.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

constexpr int GBM = 64, GBN = 64, GBK = 32, GLD = GBK + 8;

__global__ __launch_bounds__(256) void moe_gemm_kernel(const bf16* __restrict__ A, int64_t lda,
                                                       const int* __restrict__ sorted_ids, int gather_div,
                                                       const bf16* __restrict__ W, const int* __restrict__ offsets,
                                                       int E, int N, int K, bf16* __restrict__ out, int64_t ldo,
                                                       const bf16* __restrict__ bias) {
  __shared__ __attribute__((aligned(16))) bf16 sA[GBM * GLD];
  __shared__ __attribute__((aligned(16))) bf16 sB[GBN * GLD];
  __shared__ int s_tile[3];
  // ---- find (expert, m0) of this workgroup's tile ----
  if (threadIdx.x == 0) {
    int t = blockIdx.y, e = 0, found = 0;
    for (; e < E; ++e) {
      const int c = offsets[e + 1] - offsets[e];
      const int nt = (c + GBM - 1) / GBM;
      if (t < nt) {
        found = 1;
        break;
      }
      t -= nt;
    }
    s_tile[0] = found ? e : -1;
    s_tile[1] = found ? offsets[e] + t * GBM : 0;
    s_tile[2] = found ? offsets[e + 1] : 0;
  }
  __syncthreads();
  const int e = s_tile[0];
  if (e < 0) return;
  const int m0 = s_tile[1], m_end = s_tile[2];
  const int n0 = blockIdx.x * GBN;
  const bf16* We = W + (int64_t)e * N * K;

  const int tid = threadIdx.x;
  // global->LDS staging: each thread moves one 16-B chunk of A and one of B per k-step
  const int lr = tid >> 2, lc = (tid & 3) * 8;  // row 0..63, k offset 0/8/16/24
  const int arow = m0 + lr;
  int64_t a_off = -1;
  if (arow < m_end) {
    const int src = gather_div > 0 ? sorted_ids[arow] / gather_div : arow;
    a_off = (int64_t)src * lda;
  }
  const int brow = n0 + lr;
  const bf16* bptr = brow < N ? We + (int64_t)brow * K : nullptr;

  const int wave = tid >> 6, lane = tid & 63;
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  const int fr = lane & 15, fk = (lane >> 4) * 8;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 ra = {}, rb = {};
  if (a_off >= 0) ra = ld8(A + a_off + lc);
  if (bptr) rb = ld8(bptr + lc);
  for (int k0 = 0; k0 < K; k0 += GBK) {
    __syncthreads();
    *reinterpret_cast<bf16x8*>(&sA[lr * GLD + lc]) = ra;
    *reinterpret_cast<bf16x8*>(&sB[lr * GLD + lc]) = rb;
    __syncthreads();
    if (k0 + GBK < K) {  // prefetch the next k-step while this one computes
      if (a_off >= 0) ra = ld8(A + a_off + k0 + GBK + lc);
      if (bptr) rb = ld8(bptr + k0 + GBK + lc);
    }
    bf16x8 af[2], bfr[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) af[i] = *reinterpret_cast<const bf16x8*>(&sA[(wm + 16 * i + fr) * GLD + fk]);
#pragma unroll
    for (int j = 0; j < 2; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(&sB[(wn + 16 * j + fr) * GLD + fk]);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
  }
  // ---- epilogue: C lane map row = 4*(l>>4)+r, col = l&15 ----
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm + 16 * i + 4 * (lane >> 4) + r;
        const int col = n0 + wn + 16 * j + (lane & 15);
        if (row < m_end && col < N) {
          const float b = bias != nullptr ? (float)bias[(int64_t)e * N + col] : 0.f;  // per-expert bias (GPT-OSS)
          out[(int64_t)row * ldo + col] = (bf16)(acc[i][j][r] + b);
        }
      }
}

// ------------------------------------------------------------------------------------------
// grouped GEMM v2: the same 64x64 tile / 2x2-wave layout, but a BK = 64 or 128 k-step staged
// through DOUBLE-buffered LDS: the next step's global loads are issued before this step's MFMAs
// and written to the other buffer after them, so one barrier per k-step (v1: two per 32) and
// BK/32 x 16 B of W + A in flight per thread.  Decode-time MoE GEMMs are weight-streaming
// (tens of rows per expert), so this is a bandwidth kernel: the win is bytes in flight.
// ------------------------------------------------------------------------------------------
template <int BM, int BN, int BK>
__global__ __launch_bounds__(256) void moe_gemm_v2_kernel(const bf16* __restrict__ A, int64_t lda,
                                                          const int* __restrict__ sorted_ids, int gather_div,
                                                          const bf16* __restrict__ W, const int* __restrict__ offsets,
                                                          int E, int N, int K, bf16* __restrict__ out, int64_t ldo,
                                                          const bf16* __restrict__ bias) {
  constexpr int LD = BK + 8, CPR = BK / 8;           // padded LDS row, 16-B chunks per row
  constexpr int CA = BM * CPR / 256, CB = BN * CPR / 256;  // chunks per thread per operand
  constexpr int MI = BM / 32, NJ = BN / 32;          // 16x16 MFMA tiles per wave (waves 2 x 2)
  static_assert(CA >= 1 && CB >= 1 && 2 * (BM + BN) * LD * 2 <= 65536, "tile");
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * (BM + BN) * LD];
  __shared__ int s_tile[3];
  bf16* sA = smem;                  // [2][BM * LD]
  bf16* sB = smem + 2 * BM * LD;    // [2][BN * LD]
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  // ---- (expert, m0) of this tile: wave 0 prefix-sums the per-expert tile counts 64 at a time ----
  if (tid == 0) s_tile[0] = -1;
  __syncthreads();
  if (wave == 0) {
    int base = 0;
    const int y = blockIdx.y;
    for (int e0 = 0; e0 < E; e0 += 64) {
      const int e = e0 + lane;
      const int nt = e < E ? (offsets[e + 1] - offsets[e] + BM - 1) / BM : 0;
      int incl = nt;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int v = __shfl_up(incl, d);
        if (lane >= d) incl += v;
      }
      const int t = y - base;
      if (t >= incl - nt && t < incl) {
        s_tile[0] = e;
        s_tile[1] = offsets[e] + (t - (incl - nt)) * BM;
        s_tile[2] = offsets[e + 1];
      }
      base += __shfl(incl, 63);
      if (y < base) break;
    }
  }
  __syncthreads();
  const int e = s_tile[0];
  if (e < 0) return;
  const int m0 = s_tile[1], m_end = s_tile[2];
  const int n0 = blockIdx.x * BN;
  const bf16* We = W + (int64_t)e * N * K;
  const int lc = (tid % CPR) * 8;
  int64_t a_off[CA];
  const bf16* bptr[CB];
#pragma unroll
  for (int j = 0; j < CA; ++j) {
    const int arow = m0 + (tid + 256 * j) / CPR;
    a_off[j] = -1;
    if (arow < m_end) a_off[j] = (int64_t)(gather_div > 0 ? sorted_ids[arow] / gather_div : arow) * lda;
  }
#pragma unroll
  for (int j = 0; j < CB; ++j) {
    const int r = n0 + (tid + 256 * j) / CPR;
    bptr[j] = r < N ? We + (int64_t)r * K : nullptr;
  }
  const int wm = (wave >> 1) * (BM / 2), wn = (wave & 1) * (BN / 2);
  const int fr = lane & 15, fk = (lane >> 4) * 8;
  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 ra[CA], rb[CB];
  auto gload = [&](int k0) {
#pragma unroll
    for (int j = 0; j < CA; ++j) ra[j] = a_off[j] >= 0 ? ld8(A + a_off[j] + k0 + lc) : bf16x8{};
#pragma unroll
    for (int j = 0; j < CB; ++j) rb[j] = bptr[j] ? ld8(bptr[j] + k0 + lc) : bf16x8{};
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int j = 0; j < CA; ++j)
      *reinterpret_cast<bf16x8*>(&sA[buf * BM * LD + ((tid + 256 * j) / CPR) * LD + lc]) = ra[j];
#pragma unroll
    for (int j = 0; j < CB; ++j)
      *reinterpret_cast<bf16x8*>(&sB[buf * BN * LD + ((tid + 256 * j) / CPR) * LD + lc]) = rb[j];
  };
  const int nk = K / BK;
  gload(0);
  lstore(0);
  __syncthreads();
  for (int ks = 0; ks < nk; ++ks) {
    const int cur = ks & 1;
    if (ks + 1 < nk) gload((ks + 1) * BK);  // in flight during this step's MFMAs
    const bf16* a_s = sA + cur * BM * LD;
    const bf16* b_s = sB + cur * BN * LD;
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      bf16x8 af[MI], bfr[NJ];
#pragma unroll
      for (int i = 0; i < MI; ++i) af[i] = *reinterpret_cast<const bf16x8*>(&a_s[(wm + 16 * i + fr) * LD + kk + fk]);
#pragma unroll
      for (int j = 0; j < NJ; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(&b_s[(wn + 16 * j + fr) * LD + kk + fk]);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    }
    if (ks + 1 < nk) lstore(cur ^ 1);  // the other buffer was last read before the previous barrier
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm + 16 * i + 4 * (lane >> 4) + r;
        const int col = n0 + wn + 16 * j + (lane & 15);
        if (row < m_end && col < N) {
          const float b = bias != nullptr ? (float)bias[(int64_t)e * N + col] : 0.f;
          out[(int64_t)row * ldo + col] = (bf16)(acc[i][j][r] + b);
        }
      }
}

static int moe_gemm_variant() {
  const char* s = getenv("OME_MOE_GEMM");  // 1 = v1 (64x64, BK 32, single buffer); default v2
  return s ? atoi(s) : 2;
}

// bias: optional per-expert bias [E, N] added in the epilogue.  tile_m 128: the 128x128 prefill
// tile (max_m_tiles must then count 128-row tiles); otherwise the 64x64 decode tile.
OME_API int ome_moe_gemm(const void* A, int64_t lda, const int* sorted_ids, int gather_div, const void* W,
                         const int* offsets, int E, int N, int K, int max_m_tiles, void* out, int64_t ldo,
                         const void* bias, int tile_m, hipStream_t stream) {
  if (max_m_tiles <= 0) return 0;
  if (K % GBK != 0 || lda % 8 != 0) return -2;
  if (max_m_tiles > 65535) return -3;
  const int v = moe_gemm_variant();
  if (tile_m == 128 && v != 1) {
    dim3 grid((N + 127) / 128, max_m_tiles);
    moe_gemm_v2_kernel<128, 128, 32><<<grid, 256, 0, stream>>>((const bf16*)A, lda, sorted_ids, gather_div,
                                                               (const bf16*)W, offsets, E, N, K, (bf16*)out, ldo,
                                                               (const bf16*)bias);
  } else {
    if (tile_m == 128) return -4;  // the v1 kernel only has the 64-row tile
    dim3 grid((N + GBN - 1) / GBN, max_m_tiles);
    if (v != 1 && K % 64 == 0) {
      moe_gemm_v2_kernel<64, 64, 64><<<grid, 256, 0, stream>>>((const bf16*)A, lda, sorted_ids, gather_div,
                                                               (const bf16*)W, offsets, E, N, K, (bf16*)out, ldo,
                                                               (const bf16*)bias);
    } else {
      moe_gemm_kernel<<<grid, 256, 0, stream>>>((const bf16*)A, lda, sorted_ids, gather_div, (const bf16*)W, offsets,
                                                E, N, K, (bf16*)out, ldo, (const bf16*)bias);
    }
  }
  OME_CHECK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------------------------------------
// combine
// ------------------------------------------------------------------------------------------
// add (optional, may alias out): out = add + scale * sum -- an always-on shared expert's output
// folded into the combine instead of a separate elementwise add
__global__ __launch_bounds__(256) void moe_combine_kernel(const bf16* __restrict__ Y, const float* __restrict__ w,
                                                          const int* __restrict__ inv, int k, int H,
                                                          bf16* out, const bf16* add, float scale) {
  const int t = blockIdx.x;
  for (int c = threadIdx.x; c < H / 8; c += blockDim.x) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < k; ++j) {
      const float wj = w[(int64_t)t * k + j];
      const bf16x8 y = ld8(Y + (int64_t)inv[(int64_t)t * k + j] * H + c * 8);
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += wj * (float)y[q];
    }
    bf16x8 o;
    if (add != nullptr) {
      const bf16x8 a = ld8(add + (int64_t)t * H + c * 8);
#pragma unroll
      for (int q = 0; q < 8; ++q) o[q] = (bf16)((float)a[q] + acc[q] * scale);
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) o[q] = (bf16)(acc[q] * scale);
    }
    st8(out + (int64_t)t * H + c * 8, o);
  }
}

OME_API int ome_moe_combine_add(const void* Y, const float* w, const int* inv, int n_tok, int k, int H, void* out,
                                const void* add, float scale, hipStream_t stream) {
  if (n_tok <= 0) return 0;
  if (H % 8) return -2;
  moe_combine_kernel<<<n_tok, 256, 0, stream>>>((const bf16*)Y, w, inv, k, H, (bf16*)out, (const bf16*)add, scale);
  OME_CHECK_LAUNCH();
  return 0;
}

OME_API int ome_moe_combine(const void* Y, const float* w, const int* inv, int n_tok, int k, int H, void* out,
                            float scale, hipStream_t stream) {
  return ome_moe_combine_add(Y, w, inv, n_tok, k, H, out, nullptr, scale, stream);
}

// ------------------------------------------------------------------------------------------
// FP8 block-scaled grouped GEMM (DeepSeek-V3 / Kimi-K2 `quantization: fp8` experts, SURVEY.md
// §2.9 K11): out[p, :] = dequant(A[row(p), :]) . dequant(W[e(p)])^T, A e4m3 with 1x128 group
// scales sa[row][K/128] (row = the gathered source row), W e4m3 [E][N][K] with 128x128 block scales
// sw[E][N/128][K/128].  The experts stay fp8 in HBM (half the bytes of the bf16 path, which is
// what a decode-time MoE layer is bound by).  64 x 128 tile, 4 waves (2 x 2, 32 x 64 each), one
// 128-deep K block per step = ONE v_mfma_scale_f32_16x16x128_f8f6f4 per 16 x 16 block at unit MX
// scales (2x the bf16 MFMA rate), the block's fp32 scales applied to its product with a VALU FMA.
// Operands go global -> LDS by global_load_lds (per-lane gathered source rows, lane-linear
// destination, XOR-swizzled chunks), double buffered.
// ------------------------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void moe_lds_t;
typedef __attribute__((address_space(1))) void moe_glb_t;
typedef int mi32x8 __attribute__((ext_vector_type(8)));
typedef int mi32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int mswz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

__device__ __forceinline__ mi32x8 mfrag32(const char* lds, int row, int c) {
  const mi32x4 lo = *reinterpret_cast<const mi32x4*>(lds + row * 128 + mswz(row, 2 * c) * 16);
  const mi32x4 hi = *reinterpret_cast<const mi32x4*>(lds + row * 128 + mswz(row, 2 * c + 1) * 16);
  return mi32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// NST LDS stages: 2 = one K block in flight during compute, waited with vmcnt(0) at the next
// step; 3 = the block two steps ahead in flight across the barrier (counted vmcnt + raw s_barrier,
// cdna_hip_programming.md "Pipelining across barriers"), at 1.5x the LDS.  All LDS is one array
// (the tile descriptor at its end): a second __shared__ object can make hipcc drain vmcnt before
// every K step's first LDS read.
template <int BMF, int BNF, int NST = 2>
__global__ __launch_bounds__(256) void moe_gemm_fp8_kernel(const uint8_t* __restrict__ A, int64_t lda,
                                                           const float* __restrict__ sa, const int* __restrict__ sorted_ids,
                                                           int gather_div, const uint8_t* __restrict__ W,
                                                           const float* __restrict__ sw, const int* __restrict__ offsets,
                                                           int E, int N, int K, bf16* __restrict__ out, int64_t ldo) {
  constexpr int ABYTES = BMF * 128, WBYTES = BNF * 128;
  static_assert(NST == 2 || NST == 3, "NST");
  // NST == 3 stages also carry the K block's A-row scales (4 x 256 B, one 4-byte DMA per wave):
  // an ordinary VGPR load beside the DMA makes hipcc wait vmcnt(0) and drain the ring
  constexpr int SCB = NST == 3 ? 1024 : 0, STG = ABYTES + WBYTES + SCB;
  __shared__ __attribute__((aligned(16))) char smem[NST * STG + 16];
  int* s_tile = reinterpret_cast<int*>(smem + NST * STG);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  if (tid == 0) s_tile[0] = -1;
  __syncthreads();
  if (wave == 0) {   // (expert, first row) of this m-tile: prefix sum of per-expert tile counts
    int base = 0;
    const int y = blockIdx.y;
    for (int e0 = 0; e0 < E; e0 += 64) {
      const int e = e0 + lane;
      const int nt = e < E ? (offsets[e + 1] - offsets[e] + BMF - 1) / BMF : 0;
      int incl = nt;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int v = __shfl_up(incl, d);
        if (lane >= d) incl += v;
      }
      const int t = y - base;
      if (t >= incl - nt && t < incl) {
        s_tile[0] = e;
        s_tile[1] = offsets[e] + (t - (incl - nt)) * BMF;
        s_tile[2] = offsets[e + 1];
      }
      base += __shfl(incl, 63);
      if (y < base) break;
    }
  }
  __syncthreads();
  const int e = s_tile[0];
  if (e < 0) return;
  const int m0 = s_tile[1], m_end = s_tile[2];
  const int n0 = blockIdx.x * BNF;
  const int KB = K / 128, nt = KB;
  const uint8_t* We = W + (int64_t)e * N * K;
  const float* swe = sw + ((int64_t)e * (N / 128) + n0 / 128) * KB;
  // per-lane staging sources (gathered A rows, W rows), fixed over K
  constexpr int AI = BMF / 32, WI = BNF / 32;   // wave instructions per operand per wave (8 rows each)
  const uint8_t* asrc[AI];
  const uint8_t* wsrc[WI];
#pragma unroll
  for (int j = 0; j < AI; ++j) {
    const int r = (wave * AI + j) * 8 + (lane >> 3);
    int p = m0 + r;
    p = p < m_end ? p : m_end - 1;
    const int srow = gather_div > 0 ? sorted_ids[p] / gather_div : p;
    asrc[j] = A + (int64_t)srow * lda + mswz(r, lane & 7) * 16;
  }
#pragma unroll
  for (int j = 0; j < WI; ++j) {
    const int r = (wave * WI + j) * 8 + (lane >> 3);
    const int n = min(n0 + r, N - 1);
    wsrc[j] = We + (int64_t)n * K + mswz(r, lane & 7) * 16;
  }
  const float* scsrc = sa;   // NST == 3: this lane's A-row scale source (row wave*BMF/4 + lane, clamped)
  if constexpr (NST == 3) {
    const int r = wave * (BMF / 4) + min(lane, BMF / 4 - 1);
    int p = m0 + r;
    p = p < m_end ? p : m_end - 1;
    scsrc = sa + (int64_t)(gather_div > 0 ? sorted_ids[p] / gather_div : p) * (K / 128);
  }
  auto stage = [&](int buf, int kt) {
    char* la = smem + buf * STG;
    char* lw = la + ABYTES;
    if constexpr (NST == 3)
      __builtin_amdgcn_global_load_lds((moe_glb_t*)(scsrc + kt), (moe_lds_t*)(lw + WBYTES + wave * 256), 4, 0, 0);
#pragma unroll
    for (int j = 0; j < AI; ++j)
      __builtin_amdgcn_global_load_lds((moe_glb_t*)(asrc[j] + kt * 128), (moe_lds_t*)(la + (wave * AI + j) * 1024), 16,
                                       0, 0);
#pragma unroll
    for (int j = 0; j < WI; ++j)
      __builtin_amdgcn_global_load_lds((moe_glb_t*)(wsrc[j] + kt * 128), (moe_lds_t*)(lw + (wave * WI + j) * 1024), 16,
                                       0, 0);
  };
  const int wm = wave >> 1, wn = wave & 1;   // wave tile: rows [wm*BMF/2, +BMF/2), cols [wn*BNF/2, +BNF/2)
  constexpr int MJ = BMF / 32, NI = BNF / 32;
  const int fr = lane & 15, fc = lane >> 4;
  int srow[MJ];
#pragma unroll
  for (int j = 0; j < MJ; ++j) {
    int p = m0 + wm * (BMF / 2) + j * 16 + fr;
    p = p < m_end ? p : m_end - 1;
    srow[j] = gather_div > 0 ? sorted_ids[p] / gather_div : p;
  }
  f32x4 acc[NI][MJ];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < MJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // the K block's fp32 scales are prefetched one step ahead (they ride the step's vmcnt(0) wait
  // instead of adding a dependent global-load round trip to every step)
  const float* sar[MJ];
  float san[MJ];
  float swn = 0.f;
  if constexpr (NST == 2) {
#pragma unroll
    for (int j = 0; j < MJ; ++j) {
      sar[j] = sa + (int64_t)srow[j] * KB;
      san[j] = sar[j][0];
    }
    swn = swe[0];
  }
  constexpr int NL = AI + WI + (NST == 3);   // LDS-DMA instructions per thread per K block
  if constexpr (NST == 2) {
    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  } else {
    // blocks 0 and 1 in flight; the top of step t waits for block t with block t + 1 still out
    stage(0, 0);
    stage(1, min(1, nt - 1));
  }
  for (int t = 0; t < nt; ++t) {
    const int cur = NST == 2 ? (t & 1) : t % 3;
    if constexpr (NST == 3) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NL) : "memory");   // block t + 1 (maybe a clamped copy) stays out
      __builtin_amdgcn_s_barrier();   // every wave's block t landed; every wave done reading block t - 1
    }
    float s[MJ];
    if constexpr (NST == 3) {
      const char* lsc = smem + cur * STG + ABYTES + WBYTES;
      const float swv = swe[t];
#pragma unroll
      for (int j = 0; j < MJ; ++j) {
        const int r = wm * (BMF / 2) + j * 16 + fr;
        s[j] = *reinterpret_cast<const float*>(lsc + (r / (BMF / 4)) * 256 + (r % (BMF / 4)) * 4) * swv;
      }
    } else {
#pragma unroll
      for (int j = 0; j < MJ; ++j) s[j] = san[j] * swn;
    }
    if constexpr (NST == 2) {
      if (t + 1 < nt) {
#pragma unroll
        for (int j = 0; j < MJ; ++j) san[j] = sar[j][t + 1];
        swn = swe[t + 1];
        stage(cur ^ 1, t + 1);
      }
    } else {
      // branch-free: the DMA of block t + 2 (into the buffer block t - 1 left) is issued every
      // step, clamped to the last block past the end, so the counted wait above stays exact
      stage((t + 2) % 3, min(t + 2, nt - 1));
    }
    const char* la = smem + cur * STG;
    const char* lw = la + ABYTES;
    mi32x8 xa[MJ];
#pragma unroll
    for (int j = 0; j < MJ; ++j) xa[j] = mfrag32(la, wm * (BMF / 2) + j * 16 + fr, fc);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const mi32x8 wf = mfrag32(lw, wn * (BNF / 2) + i * 16 + fr, fc);
#pragma unroll
      for (int j = 0; j < MJ; ++j) {
        const f32x4 p = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(wf, xa[j], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0,
                                                                        127, 0, 127);
        acc[i][j] += p * s[j];
      }
    }
    if constexpr (NST == 2) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }
  if constexpr (NST == 3) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // clamped tail DMA retires before exit
  // lane (fr, fc) of block (i, j): row p = m0 + wm*BMF/2 + j*16 + fr, cols n = n0 + wn*BNF/2 + i*16 + 4fc .. +3
#pragma unroll
  for (int j = 0; j < MJ; ++j) {
    const int p = m0 + wm * (BMF / 2) + j * 16 + fr;
    if (p >= m_end) continue;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int n = n0 + wn * (BNF / 2) + i * 16 + 4 * fc;
      if (n >= N) continue;
      bf16x4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = (bf16)acc[i][j][r];
      *reinterpret_cast<bf16x4*>(out + (int64_t)p * ldo + n) = v;
    }
  }
}

// A [rows][K] e4m3 (gathered through sorted_ids / gather_div when gather_div > 0), sa [rows][K/128];
// W [E][N][K] e4m3, sw [E][N/128][K/128]; out [n_assign][N] bf16 in sorted order.  N % 128 == 0,
// K % 128 == 0.
// bm = 64: 64 x 128 tiles (decode: a few rows per expert, more workgroups per weight byte);
// bm = 128: 128 x 128 tiles, 64 x 64 per wave (prefill: twice the MFMAs per staged K block and the
// expert's weights read once per 128 gathered rows; 64 KB of LDS, 2 workgroups per CU).
// max_m_tiles: static upper bound of bm-row tiles (n_assign / bm + E).
OME_API int ome_moe_gemm_fp8_tile(const void* A, int64_t lda, const float* sa, const int* sorted_ids, int gather_div,
                                  const void* W, const float* sw, const int* offsets, int E, int N, int K,
                                  int max_m_tiles, int bm, void* out, int64_t ldo, hipStream_t stream) {
  if (max_m_tiles <= 0) return 0;
  if (N % 128 || K % 128 || lda % 16 || ((uintptr_t)A | (uintptr_t)W) % 16) return -2;
  if (max_m_tiles > 65535) return -3;
  // LDS stages (OME_MOE_FP8_NST): 3 for the 64-row tile (2 workgroups / CU, 2-5 % faster at
  // prefill sizes), 2 for the 128-row tile (3 stages = 96 KB would leave one workgroup per CU);
  // profiles/r05_fp8_moe_tiles.md
  static const int nst_env = getenv("OME_MOE_FP8_NST") ? atoi(getenv("OME_MOE_FP8_NST")) : 0;
  const int nst = nst_env ? nst_env : (bm == 64 ? 3 : 2);
#define MOE_FP8(BM, NS)                                                                                          \
  moe_gemm_fp8_kernel<BM, 128, NS><<<dim3(N / 128, max_m_tiles), 256, 0, stream>>>(                               \
      (const uint8_t*)A, lda, sa, sorted_ids, gather_div, (const uint8_t*)W, sw, offsets, E, N, K, (bf16*)out, ldo)
  if (bm == 128) {
    if (nst == 3) MOE_FP8(128, 3); else MOE_FP8(128, 2);
  } else if (bm == 64) {
    if (nst == 3) MOE_FP8(64, 3); else MOE_FP8(64, 2);
  } else {
    return -4;
  }
#undef MOE_FP8
  OME_CHECK_LAUNCH();
  return 0;
}

OME_API int ome_moe_gemm_fp8(const void* A, int64_t lda, const float* sa, const int* sorted_ids, int gather_div,
                             const void* W, const float* sw, const int* offsets, int E, int N, int K,
                             int max_m_tiles, void* out, int64_t ldo, hipStream_t stream) {
  return ome_moe_gemm_fp8_tile(A, lda, sa, sorted_ids, gather_div, W, sw, offsets, E, N, K, max_m_tiles, 64, out, ldo,
                               stream);
}
