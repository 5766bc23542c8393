// FP8-weight x bf16-activation ("W8A16") projections for decode row counts on gfx950
// (verdict r05 item 5: fix the small-N fp8 path instead of keeping bf16 copies).
//
// At M <= 256 a projection is a weight stream: the W8A8 path pays a separate activation-quant
// launch plus 128-row MFMA tiles it cannot fill, and on small-N shapes (qkv / o / q_a / shared
// experts) it streamed only 0.4-1.1 TB/s of fp8 bytes (profiles/r05_fp8_routed_bench.txt), so a
// dequantised bf16 copy of those weights used to serve decode.  Here the fp8 weight itself is
// streamed and widened in registers; the activation stays bf16 (no quantisation pass at all):
//
//   * w8_gemv_kernel, M <= 8: each wave owns R consecutive weight rows and walks K with 16-byte
//     loads (lane l covers k = 16 l + 1024 i: 16 e4m3 values, one load per row), U K steps in
//     flight, no LDS.  e4m3 -> bf16 is exact (v_cvt_scalef32_pk_bf16_fp8 with a unit scale), the
//     products run on v_dot2c_f32_bf16, fp32 accumulate.  Scales are applied to fp32 partial sums:
//     per channel once at the end, per 128x128 block once per 16-element chunk (a lane's chunk
//     never straddles a 128-wide K block).
//   * w8_skinny_kernel, 8 < M <= 256: the skinny MFMA tile (csrc/kernels/skinny_gemm.hip: one
//     workgroup = all M rows x 64 weight rows, split-K when the weight has few row tiles) with
//     the W step (64 rows x 64 k) loaded as 4 KiB of e4m3 -- one 16-byte load per thread -- and
//     widened to bf16 on its way into LDS.  3-4 K steps of both operands ride a register ring
//     (the first version waited one global round trip per 64-deep step: 0.4-0.8 TB/s) and the
//     LDS tiles are double-buffered, one barrier per step.  Per-channel scales multiply the fp32 accumulators in
//     the epilogue (exact widening, one rounding); block scales are folded into the widening of
//     each 64-deep K step (bf16(q * s), the same values the old dequantised bf16 copy held).
// Both end in the skinny kernel's deterministic split-K reduction (fixed split order, last
// arriver re-arms the tile counter: HIP-graph replayable).
#include "common.h"

namespace {

typedef __bf16 w8_bf16x2 __attribute__((ext_vector_type(2)));
typedef unsigned int w8_u32x4 __attribute__((ext_vector_type(4)));

// 4 e4m3 (one dword) -> 4 bf16, exact (unit scale)
__device__ __forceinline__ bf16x4 w8_cvt4(uint32_t v) {
  const w8_bf16x2 lo = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8((int)v, 1.0f, false);
  const w8_bf16x2 hi = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8((int)v, 1.0f, true);
  return bf16x4{lo[0], lo[1], hi[0], hi[1]};
}

// 8 e4m3 (two dwords) -> bf16x8, exact
__device__ __forceinline__ bf16x8 w8_cvt8(uint32_t a, uint32_t b) {
  const bf16x4 x = w8_cvt4(a), y = w8_cvt4(b);
  return bf16x8{x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
}

// 8 e4m3 -> bf16(q * s) (block-scaled weights: the scale folded into the widening)
__device__ __forceinline__ bf16x8 w8_cvt8_scaled(uint32_t a, uint32_t b, float s) {
  const f32x2 p0 = __builtin_amdgcn_cvt_pk_f32_fp8((int)a, false), p1 = __builtin_amdgcn_cvt_pk_f32_fp8((int)a, true);
  const f32x2 p2 = __builtin_amdgcn_cvt_pk_f32_fp8((int)b, false), p3 = __builtin_amdgcn_cvt_pk_f32_fp8((int)b, true);
  return bf16x8{(bf16)(p0.x * s), (bf16)(p0.y * s), (bf16)(p1.x * s), (bf16)(p1.y * s),
                (bf16)(p2.x * s), (bf16)(p2.y * s), (bf16)(p3.x * s), (bf16)(p3.y * s)};
}

__device__ __forceinline__ float w8_dot8(bf16x8 a, bf16x8 b, float acc) {
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(a, a, 0, 1), __builtin_shufflevector(b, b, 0, 1), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(a, a, 2, 3), __builtin_shufflevector(b, b, 2, 3), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(a, a, 4, 5), __builtin_shufflevector(b, b, 4, 5), acc, false);
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(a, a, 6, 7), __builtin_shufflevector(b, b, 6, 7), acc, false);
}

// ------------------------------------------------------------------------------------ GEMV
// BLK = 0: sw [N] per channel; BLK = 1: sw [ceil(N / 128), K / 128] per 128 x 128 block
template <int M, int R, int U, int BLK>
__global__ __launch_bounds__(256) void w8_gemv_kernel(const bf16* __restrict__ X, int64_t ldx,
                                                      const uint8_t* __restrict__ W, int64_t ldw,
                                                      const float* __restrict__ sw, const bf16* __restrict__ bias,
                                                      bf16* __restrict__ out, int64_t ldo, int N, int K) {
  const int lane = threadIdx.x & 63;
  const int n0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * R;
  if (n0 >= N) return;
  const int kb = K >> 7;
  const uint8_t* wr[R];
  const float* sr[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int n = min(n0 + r, N - 1);   // rows past N are computed, never stored
    wr[r] = W + (int64_t)n * ldw;
    sr[r] = BLK ? sw + (int64_t)(n >> 7) * kb : sw + n;
  }
  float acc[M][R];
#pragma unroll
  for (int m = 0; m < M; ++m)
#pragma unroll
    for (int r = 0; r < R; ++r) acc[m][r] = 0.f;

  auto step = [&](const w8_u32x4 (&w)[R], int k) {
    bf16x8 xa[M], xb[M];
#pragma unroll
    for (int m = 0; m < M; ++m) {
      xa[m] = ld8(X + m * ldx + k);
      xb[m] = ld8(X + m * ldx + k + 8);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const bf16x8 wa = w8_cvt8(w[r][0], w[r][1]), wb = w8_cvt8(w[r][2], w[r][3]);
      if constexpr (BLK) {
        const float s = sr[r][k >> 7];
#pragma unroll
        for (int m = 0; m < M; ++m) acc[m][r] += s * w8_dot8(xb[m], wb, w8_dot8(xa[m], wa, 0.f));
      } else {
#pragma unroll
        for (int m = 0; m < M; ++m) acc[m][r] = w8_dot8(xb[m], wb, w8_dot8(xa[m], wa, acc[m][r]));
      }
    }
  };

  int k = lane * 16;
  for (; k + (U - 1) * 1024 < K; k += U * 1024) {
    w8_u32x4 w[U][R];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int r = 0; r < R; ++r) w[u][r] = *reinterpret_cast<const w8_u32x4*>(wr[r] + k + 1024 * u);
#pragma unroll
    for (int u = 0; u < U; ++u) step(w[u], k + 1024 * u);
  }
  for (; k < K; k += 1024) {
    w8_u32x4 w[R];
#pragma unroll
    for (int r = 0; r < R; ++r) w[r] = *reinterpret_cast<const w8_u32x4*>(wr[r] + k);
    step(w, k);
  }
#pragma unroll
  for (int m = 0; m < M; ++m)
#pragma unroll
    for (int r = 0; r < R; ++r) acc[m][r] = wave_sum(acc[m][r]);
#pragma unroll
  for (int m = 0; m < M; ++m)
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (lane == m * R + r && n0 + r < N) {
        float v = acc[m][r];
        if constexpr (!BLK) v *= sr[r][0];
        out[(int64_t)m * ldo + n0 + r] = (bf16)(v + (bias ? (float)bias[n0 + r] : 0.f));
      }
}

// ------------------------------------------------------------------------------------ skinny MFMA
constexpr int NT = 64;   // weight rows per workgroup
constexpr int KB = 64;   // K per step

// workgroup barrier ordering LDS only: wait for this wave's LDS traffic, then s_barrier (global
// loads in flight stay in flight)
__device__ __forceinline__ void w8_lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ int w8_sw(int row, int chunk) { return row * 8 + (chunk ^ (row & 7)); }

template <int MB, int BLK>   // 16-row activation blocks per wave: Mp = 64 * MB
__global__ __launch_bounds__(256) void w8_skinny_kernel(const bf16* __restrict__ X, int64_t ldx,
                                                        const uint8_t* __restrict__ W, int64_t ldw,
                                                        const float* __restrict__ sw, const bf16* __restrict__ bias,
                                                        bf16* __restrict__ out, int64_t ldo, int M, int N, int K,
                                                        int splits, float* __restrict__ ws, int* __restrict__ cnt) {
  constexpr int MP = 64 * MB, XL = MP * 8 / 256;   // 16-byte X chunks per thread per step
  // PD K steps of operands in flight per thread (a register ring: one global round trip per PD
  // steps, not per step) and two LDS buffers (one barrier per step)
  constexpr int PD = MB == 4 ? 3 : 4;
  __shared__ __attribute__((aligned(16))) bf16 sX[2][MP * KB];
  __shared__ __attribute__((aligned(16))) bf16 sW[2][NT * KB];
  __shared__ int s_last;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int tile = blockIdx.x / splits, split = blockIdx.x - tile * splits;
  const int n0 = tile * NT;
  const int steps = K / KB, kb = K >> 7;
  const int s0 = (int)((int64_t)steps * split / splits), s1 = (int)((int64_t)steps * (split + 1) / splits);
  // this thread's W piece: row wrow, k chunk wc (16 e4m3 = bf16 chunks 2 wc, 2 wc + 1)
  const int wrow = tid >> 2, wc = tid & 3;
  const int wn = min(n0 + wrow, N - 1);
  const uint8_t* wp = W + (int64_t)wn * ldw + 16 * wc;
  const float* wsc = BLK ? sw + (int64_t)(wn >> 7) * kb : sw;

  bf16x8 rx[PD][XL];
  w8_u32x4 rw[PD];
  auto load = [&](int j, int s) {   // j: compile-time ring slot after unrolling
    const int k0 = s * KB;
#pragma unroll
    for (int i = 0; i < XL; ++i) {
      const int c = tid + 256 * i, row = c >> 3, ch = c & 7;
      rx[j][i] = row < M ? ld8(X + (int64_t)row * ldx + k0 + 8 * ch) : bf16x8{};
    }
    rw[j] = *reinterpret_cast<const w8_u32x4*>(wp + k0);
  };

  f32x4 acc[4][MB];
#pragma unroll
  for (int nb = 0; nb < 4; ++nb)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) acc[nb][mb] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int r0 = wave * 16 * MB, lr = lane & 15, lg = lane >> 4;
#pragma unroll
  for (int j = 0; j < PD; ++j)
    if (s0 + j < s1) load(j, s0 + j);
  for (int sb = s0; sb < s1; sb += PD) {
#pragma unroll
    for (int j = 0; j < PD; ++j) {
      const int s = sb + j;
      if (s >= s1) break;
      bf16* bx = sX[(s - s0) & 1];
      bf16* bw = sW[(s - s0) & 1];
#pragma unroll
      for (int i = 0; i < XL; ++i) {
        const int c = tid + 256 * i;
        *reinterpret_cast<bf16x8*>(&bx[w8_sw(c >> 3, c & 7) * 8]) = rx[j][i];
      }
      bf16x8 w0, w1;
      if constexpr (BLK) {
        const float sc = wsc[(s * KB) >> 7];
        w0 = w8_cvt8_scaled(rw[j][0], rw[j][1], sc);
        w1 = w8_cvt8_scaled(rw[j][2], rw[j][3], sc);
      } else {
        w0 = w8_cvt8(rw[j][0], rw[j][1]);
        w1 = w8_cvt8(rw[j][2], rw[j][3]);
      }
      *reinterpret_cast<bf16x8*>(&bw[w8_sw(wrow, 2 * wc) * 8]) = w0;
      *reinterpret_cast<bf16x8*>(&bw[w8_sw(wrow, 2 * wc + 1) * 8]) = w1;
      // this step's tile is visible; the buffer written here was last read two steps ago,
      // before the previous step's barrier.  LDS-only barrier: __syncthreads() would also drain
      // the register ring's global loads (vmcnt(0)) and serialise every step on a round trip
      w8_lds_barrier();
      load(j, min(s + PD, s1 - 1));   // unconditional (past the end: a re-read, never used) -- see w8_mgemv
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int ch = 4 * kk + lg;
        bf16x8 a[4], b[MB];
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) a[nb] = *reinterpret_cast<const bf16x8*>(&bw[w8_sw(nb * 16 + lr, ch) * 8]);
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
          b[mb] = *reinterpret_cast<const bf16x8*>(&bx[w8_sw(r0 + mb * 16 + lr, ch) * 8]);
#pragma unroll
        for (int nb = 0; nb < 4; ++nb)
#pragma unroll
          for (int mb = 0; mb < MB; ++mb)
            acc[nb][mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[nb], b[mb], acc[nb][mb], 0, 0, 0);
      }
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
    // publish: every wave drains its slab stores, one agent-scope release, then the ticket
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      s_last = __hip_atomic_fetch_add(&cnt[tile], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == splits - 1;
      if (s_last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
    if (!s_last) return;
    // fixed split order (deterministic); one split's fragments loaded together (see w8_mgemv)
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) acc[nb][mb] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int p = 0; p < splits; ++p) {
      const float* slab = ws + ((int64_t)tile * splits + p) * MP * NT;
      f32x4 v[4][MB];
#pragma unroll
      for (int nb = 0; nb < 4; ++nb)
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
          v[nb][mb] = *reinterpret_cast<const f32x4*>(slab + (r0 + 16 * mb + lr) * NT + 16 * nb + 4 * lg);
#pragma unroll
      for (int nb = 0; nb < 4; ++nb)
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) acc[nb][mb] += v[nb][mb];
    }
    if (tid == 0) cnt[tile] = 0;   // re-arm for the next launch / graph replay
  }
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) {
    const int n = n0 + 16 * nb + 4 * lg;
    float bv[4] = {0.f, 0.f, 0.f, 0.f}, sv[4] = {1.f, 1.f, 1.f, 1.f};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (bias) bv[r] = (float)bias[n + r];
      if constexpr (!BLK) sv[r] = sw[n + r];
    }
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const int m = r0 + 16 * mb + lr;
      if (m < M) {
        bf16x4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = (bf16)(acc[nb][mb][r] * sv[r] + bv[r]);
        *reinterpret_cast<bf16x4*>(out + (int64_t)m * ldo + n) = v;
      }
    }
  }
}


// ------------------------------------------------------------------------------------ MFMA GEMV
// 8 < M <= 64: the skinny tile's per-step LDS round trip of the weight (global -> VGPR -> LDS ->
// VGPR, two barriers) is what capped it at 0.5-1 TB/s.  Here the weight never touches LDS: lane l
// of a wave loads 16 e4m3 of weight row (l & 15) at k = kb + 16 (l >> 4) -- one 16-byte load per
// 16-row block and 64-deep K step -- and those 16 values are the A operands of TWO
// v_mfma_f32_16x16x32_bf16 (k permuted identically in A and B, so the sum is exact).  Only the
// activation slice (M x kslice bf16, <= 64 KiB, rows padded by 16 B so the 16 row reads of a lane
// group hit distinct banks) is staged in LDS, once per workgroup, and every wave reuses each X
// fragment for its 4 weight blocks.  A wave owns 64 weight rows; a workgroup 256 rows x one K
// slice; the K slices of a row tile meet in the skinny kernel's fixed-order slab reduction.
// Weight loads run 4 K steps ahead (16 x 16 B per lane in flight) with no barrier in the K loop.
constexpr int MG_NB = 4;                    // 16-row weight blocks per wave
constexpr int MG_ROWS = 4 * MG_NB * 16;     // weight rows per workgroup
constexpr int MG_U = 4;                     // K steps (64 deep) in flight per wave

// STEPS = kslice / 64, a template constant: the K loop is straight-line code, so the ring slot of
// every step and the refill distance are compile-time and hipcc's vmcnt counting stays exact
// (with a runtime trip count it drained the ring at every loop back-edge: 1-2 TB/s)
template <int MT, int BLK, int STEPS>   // MT: 16-row activation tiles (M <= 16 MT)
__global__ __launch_bounds__(256) void w8_mgemv_kernel(const bf16* __restrict__ X, int64_t ldx,
                                                       const uint8_t* __restrict__ W, int64_t ldw,
                                                       const float* __restrict__ sw, const bf16* __restrict__ bias,
                                                       bf16* __restrict__ out, int64_t ldo, int M, int N, int K,
                                                       int kslice, int splits, float* __restrict__ ws,
                                                       int* __restrict__ cnt) {
  constexpr int MP = 16 * MT;
  extern __shared__ __attribute__((aligned(16))) char mg_smem[];
  __shared__ int s_last;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int tile = blockIdx.x / splits, split = blockIdx.x - tile * splits;
  const int k0 = split * kslice;
  const int xs = kslice * 2 + 16;   // LDS row stride in bytes (padded)
  // ---- this wave's weight rows: issue the first MG_U steps before staging X
  const int lr = lane & 15, g = lane >> 4;
  const int nb0 = tile * MG_ROWS + wave * MG_NB * 16;
  const uint8_t* wp[MG_NB];
  const float* sc[MG_NB];
#pragma unroll
  for (int b = 0; b < MG_NB; ++b) {
    const int n = min(nb0 + 16 * b + lr, N - 1);   // rows past N are computed, never stored
    wp[b] = W + (int64_t)n * ldw + k0 + 16 * g;
    sc[b] = BLK ? sw + (int64_t)(n >> 7) * (K >> 7) + (k0 >> 7) : sw;
  }
  constexpr int R = STEPS < MG_U ? STEPS : MG_U;   // ring depth (K steps in flight)
  w8_u32x4 w[R][MG_NB];
#pragma unroll
  for (int u = 0; u < R; ++u)
#pragma unroll
    for (int b = 0; b < MG_NB; ++b) w[u][b] = *reinterpret_cast<const w8_u32x4*>(wp[b] + 64 * u);
  // ---- stage X[0:MP][k0:k0+kslice] (rows >= M zero)
  constexpr int CPR = STEPS * 8;   // 16-byte chunks per row
#pragma unroll
  for (int c0 = 0; c0 < MP * CPR; c0 += 256) {
    const int c = c0 + tid, r = c / CPR, ch = c - r * CPR;
    if (c < MP * CPR)
      *reinterpret_cast<bf16x8*>(mg_smem + r * xs + ch * 16) =
          r < M ? ld8(X + (int64_t)r * ldx + k0 + 8 * ch) : bf16x8{};
  }
  __syncthreads();

  f32x4 acc[MG_NB][MT];
#pragma unroll
  for (int b = 0; b < MG_NB; ++b)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[b][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < STEPS; ++j) {
    const int u = j % R, ks = 64 * j;
    bf16x8 xa[MT], xb[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const char* p = mg_smem + (mt * 16 + lr) * xs + (ks + 16 * g) * 2;
      xa[mt] = *reinterpret_cast<const bf16x8*>(p);
      xb[mt] = *reinterpret_cast<const bf16x8*>(p + 16);
    }
#pragma unroll
    for (int b = 0; b < MG_NB; ++b) {
      bf16x8 wa, wb;
      if constexpr (BLK) {
        const float f = sc[b][ks >> 7];
        wa = w8_cvt8_scaled(w[u][b][0], w[u][b][1], f);
        wb = w8_cvt8_scaled(w[u][b][2], w[u][b][3], f);
      } else {
        wa = w8_cvt8(w[u][b][0], w[u][b][1]);
        wb = w8_cvt8(w[u][b][2], w[u][b][3]);
      }
      if (j + R < STEPS) w[u][b] = *reinterpret_cast<const w8_u32x4*>(wp[b] + ks + 64 * R);   // compile-time guard
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        acc[b][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa, xa[mt], acc[b][mt], 0, 0, 0);
        acc[b][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb, xb[mt], acc[b][mt], 0, 0, 0);
      }
    }
  }

  // acc[b][mt][r] = C[m = 16 mt + lr][n = nb0 + 16 b + 4 g + r]
  if (splits > 1) {
    constexpr int TILE_F = MG_ROWS * MP;   // floats per (tile, split) slab
    float* part = ws + ((int64_t)tile * splits + split) * TILE_F;
#pragma unroll
    for (int b = 0; b < MG_NB; ++b)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        *reinterpret_cast<f32x4*>(part + (((wave * MG_NB + b) * MT + mt) * 64 + lane) * 4) = acc[b][mt];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      s_last = __hip_atomic_fetch_add(&cnt[tile], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == splits - 1;
      if (s_last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
    if (!s_last) return;
    // fixed split order (deterministic); each split's MG_NB x MT fragments are loaded together,
    // so the reduction costs `splits` memory round trips, not splits x MG_NB x MT dependent ones
#pragma unroll
    for (int b = 0; b < MG_NB; ++b)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[b][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int p = 0; p < splits; ++p) {
      const float* slab = ws + ((int64_t)tile * splits + p) * TILE_F;
      f32x4 v[MG_NB][MT];
#pragma unroll
      for (int b = 0; b < MG_NB; ++b)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
          v[b][mt] = *reinterpret_cast<const f32x4*>(slab + (((wave * MG_NB + b) * MT + mt) * 64 + lane) * 4);
#pragma unroll
      for (int b = 0; b < MG_NB; ++b)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) acc[b][mt] += v[b][mt];
    }
    if (tid == 0) cnt[tile] = 0;   // re-arm for the next launch / graph replay
  }
#pragma unroll
  for (int b = 0; b < MG_NB; ++b) {
    const int n = nb0 + 16 * b + 4 * g;
    if (n >= N) continue;   // N % 16 == 0 (host): a lane's 4 columns are all in or all out
    float bv[4] = {0.f, 0.f, 0.f, 0.f}, sv[4] = {1.f, 1.f, 1.f, 1.f};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (bias) bv[r] = (float)bias[n + r];
      if constexpr (!BLK) sv[r] = sw[n + r];
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int m = 16 * mt + lr;
      if (m < M) {
        bf16x4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = (bf16)(acc[b][mt][r] * sv[r] + bv[r]);
        *reinterpret_cast<bf16x4*>(out + (int64_t)m * ldo + n) = v;
      }
    }
  }
}

}  // namespace

// out[M, N] = X[M, K] (bf16, row stride ldx) . dequant(W)^T (+ bias); W [N, K] e4m3 (row stride ldw
// bytes, 16-byte aligned rows); block 0: sw [N] f32 per channel, block 128: sw [ceil(N/128), K/128].
// M <= 8: GEMV (K % 16 == 0); 8 < M <= 256: skinny MFMA (N % 64 == 0, K % 64 == 0; block 128 needs
// K % 128 == 0), splits > 1 needs ws (>= N / 64 * splits * Mp * 64 floats, Mp = 64 / 128 / 256 by
// M) and cnt (>= N / 64 ints, zero on first use; re-armed by the kernel).
OME_API int ome_w8a16_gemm(const void* X, int64_t ldx, const void* W, int64_t ldw, const float* sw, int block,
                           const void* bias, void* out, int64_t ldo, int M, int N, int K, int splits, float* ws,
                           int* cnt, hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (M > 256 || K <= 0 || ldx % 8 || ldw % 16 || (block != 0 && block != 128) || (block && K % 128)) return -2;
  const bool blk = block == 128;
  if (M <= 8) {
    if (K % 16) return -2;
    const bool narrow = N <= 4096;
#define W8GV(MV, RV, UV, BV)                                                                               \
  w8_gemv_kernel<MV, RV, UV, BV><<<dim3((N + 4 * RV - 1) / (4 * RV)), 256, 0, stream>>>(                  \
      (const bf16*)X, ldx, (const uint8_t*)W, ldw, sw, (const bf16*)bias, (bf16*)out, ldo, N, K)
#define W8GV_M(MV)                                                                                         \
  if (blk) { if (narrow) W8GV(MV, 2, (MV <= 4 ? 4 : 2), 1); else W8GV(MV, 4, (MV <= 4 ? 4 : 2), 1); }     \
  else { if (narrow) W8GV(MV, 2, (MV <= 4 ? 4 : 2), 0); else W8GV(MV, 4, (MV <= 4 ? 4 : 2), 0); }
    switch (M) {
      case 1: W8GV_M(1); break;
      case 2: W8GV_M(2); break;
      case 3: W8GV_M(3); break;
      case 4: W8GV_M(4); break;
      case 5: W8GV_M(5); break;
      case 6: W8GV_M(6); break;
      case 7: W8GV_M(7); break;
      default: W8GV_M(8); break;
    }
#undef W8GV_M
#undef W8GV
    OME_CHECK_LAUNCH();
    return 0;
  }
  if (N % NT || K % KB || ldo % 4 || splits < 1 || splits > K / KB) return -2;
  if (splits > 1 && (!ws || !cnt)) return -3;
  dim3 grid((N / NT) * splits);
#define W8SK(MBV, BV)                                                                                       \
  w8_skinny_kernel<MBV, BV><<<grid, 256, 0, stream>>>((const bf16*)X, ldx, (const uint8_t*)W, ldw, sw,       \
                                                      (const bf16*)bias, (bf16*)out, ldo, M, N, K, splits, ws, cnt)
  if (M <= 64) { if (blk) W8SK(1, 1); else W8SK(1, 0); }
  else if (M <= 128) { if (blk) W8SK(2, 1); else W8SK(2, 0); }
  else { if (blk) W8SK(4, 1); else W8SK(4, 0); }
#undef W8SK
  OME_CHECK_LAUNCH();
  return 0;
}

// 8 < M <= 32 on the MFMA GEMV (w8_mgemv_kernel): K % 256 == 0, N % 16 == 0, kslice 256 / 512 / 1024
// dividing K with MP x (2 kslice + 16) <= 64 KiB (MP = 16 / 32 by M); splits = K / kslice > 1
// needs ws (>= ceil(N / 256) * splits * 256 * MP floats) and cnt (>= ceil(N / 256) ints, zero on
// first use; re-armed by the kernel).  ldo % 4 == 0.
OME_API int ome_w8a16_mgemv(const void* X, int64_t ldx, const void* W, int64_t ldw, const float* sw, int block,
                            const void* bias, void* out, int64_t ldo, int M, int N, int K, int kslice, float* ws,
                            int* cnt, hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (M > 64 || K % 256 || N % 16 || ldx % 8 || ldw % 16 || ldo % 4 || (block != 0 && block != 128)) return -2;
  if (kslice <= 0 || kslice % 256 || K % kslice) return -2;
  const int MT = M <= 16 ? 1 : 2;
  const size_t lds = (size_t)16 * MT * (2 * kslice + 16);
  if (M > 32 || lds > 65536 || (kslice != 256 && kslice != 512 && kslice != 1024)) return -2;
  const int splits = K / kslice, tiles = (N + MG_ROWS - 1) / MG_ROWS;
  if (splits > 1 && (!ws || !cnt)) return -3;
  dim3 grid(tiles * splits);
#define W8MG(MTV, BV, SV)                                                                                    \
  w8_mgemv_kernel<MTV, BV, SV><<<grid, 256, lds, stream>>>((const bf16*)X, ldx, (const uint8_t*)W, ldw, sw,    \
                                                           (const bf16*)bias, (bf16*)out, ldo, M, N, K, kslice,  \
                                                           splits, ws, cnt)
#define W8MG_S(MTV, BV)                                                                                      \
  if (kslice == 256) W8MG(MTV, BV, 4);                                                                       \
  else if (kslice == 512) W8MG(MTV, BV, 8);                                                                  \
  else W8MG(MTV, BV, 16)
  const bool blk = block == 128;
  if (MT == 1) { if (blk) { W8MG_S(1, 1); } else { W8MG_S(1, 0); } }
  else { if (blk) { W8MG_S(2, 1); } else { W8MG_S(2, 0); } }
#undef W8MG_S
#undef W8MG
  OME_CHECK_LAUNCH();
  return 0;
}
