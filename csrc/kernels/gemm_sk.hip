// Stream-K bf16 GEMM for the decoder projections, "NT" layout:
//   C[M][N] = X[M][K] . W[N][K]^T  (+ bias)          (= F.linear(x, w))
//
// Round-4 redesign of the decomposition around the 256-row MFMA tile of gemm.hip.  The tile body
// (256 x BN output per 512-thread workgroup, BK = 64, v_mfma_f32_16x16x32_bf16, W as the MFMA A
// operand so every lane owns 4 consecutive output columns, global_load_lds staging into
// lane-linear LDS with the XOR swizzle on the source address) was measured at ~5 TF/CU; what
// lost to hipBLASLt was tile-count quantisation (24 output tiles for 256 CUs at decode M = 256)
// and the split-K fp32 round trip through a second launch (profiles/r03_bf16_gemm_tile_vs_hipblaslt.txt).
//
// Decomposition (per XCD, persistent):
//   * the T output tiles are cut into 8 contiguous ranges, one per XCD group (blocks b with the
//     same b % 8 share an XCD under round-robin dispatch -- a speed assumption only, nothing
//     below depends on placement for correctness);
//   * the nwg / 8 blocks of a group split the group's (tile, k-step) units evenly and walk
//     them in order: a block computes the end of one tile, whole tiles, and the head of the next;
//   * a segment that covers a whole tile stores through the fused epilogue directly; a partial
//     segment writes its fp32 accumulators to a slab in FRAGMENT order (thread-private, 1 KiB
//     contiguous per wave instruction) and takes a ticket; the tile's last arriver acquires the
//     slabs and adds them into its own registers element-wise (the slab layout is its own
//     accumulator layout, so no shuffle) and runs the epilogue.  Nothing ever waits on another
//     workgroup (no co-residency assumption).  Hand-off = MI355X_MICROARCH.md "Valid forms"
//     producer / consumer protocol: every storing wave vmcnt(0) -> barrier -> lane-0 agent
//     release -> vmcnt(0) -> relaxed agent ticket; last arriver: agent acquire -> vmcnt(0) ->
//     barrier -> plain loads.
//   * nwg = T (with T % 8 == 0) degenerates to plain data-parallel tiles; nwg = 256 is full
//     stream-K.  ops.gemm_sk_plan picks per shape from a measured table.
// Pipeline: NBUF = 2 (BN = 256: 128 KiB LDS) or 3 (BN = 128: 3 x 48 KiB) K-tiles in LDS; with
// three, the DMA of tile t+2 stays in flight across the barrier that publishes tile t+1
// (counted vmcnt + raw s_barrier, cdna_hip_programming.md "Pipelining across barriers").
// Epilogues: bf16 (+bias), SiLU(gate) * up for gate/up weights interleaved in 16-row blocks.
//
// FP8 (OCP e4m3) W8A8 on the same decomposition (Q = 1: per-token x per-channel scales, Q = 2:
// DeepSeek 1 x 128 activation groups x 128 x 128 weight blocks).  A K-tile is 128 bytes of a row
// in both dtypes, so the DMA pieces, the LDS images and the fragment reads are byte-identical to
// the bf16 path; the bf16 path's kk = 0 and kk = 1 chunks of a row, side by side, are the 32-byte
// operand of ONE v_mfma_scale_f32_16x16x128_f8f6f4 (unit MX scales; the same K permutation on both
// operands, so the sum is exact) -- half the MFMAs at twice the rate per instruction, half the
// weight bytes per K.  Q = 2 adds one 4-byte DMA piece per wave and K-tile that lands the tile's
// activation group scales (and the W block scales) in LDS next to the operands, so the scale
// traffic rides the same counted vmcnt pipeline; each block product is scaled by a VALU FMA.
#include "common.h"

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;

namespace {

constexpr int BK = 64, NTHR = 512;
enum { SK_BF16 = 0, SK_SILU = 2 };

__device__ __forceinline__ int sk_swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

// ROWS x 64 bf16 rows into lane-linear LDS: one wave instruction = 8 rows x 128 B.  Rows past
// `rows` re-read the last valid row (their products are never stored).
template <int ROWS>
__device__ __forceinline__ void sk_stage(char* lds, const bf16* __restrict__ g, int64_t ld, int row0, int rows, int k0,
                                         int wave, int lane) {
  constexpr int PER = ROWS / 64;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int blk = wave * PER + j;
    const int r = blk * 8 + (lane >> 3);
    int gr = row0 + r;
    gr = gr < rows ? gr : rows - 1;
    const bf16* src = g + (int64_t)gr * ld + k0 + sk_swz(r, lane & 7) * 8;
    __builtin_amdgcn_global_load_lds((glb_void_t*)src, (lds_void_t*)(lds + blk * 1024), 16, 0, 0);
  }
}

// LDS-DMA of 16 B per lane: buffer_load_dwordx4 ... lds (a non-template wrapper: the builtin
// only exists for the device target, and inside the kernel template the host pass dropped the
// kernel's stub)
__device__ __forceinline__ void sk_buf_lds(__amdgpu_buffer_rsrc_t rs, char* lds, uint32_t voff, uint32_t soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)lds, 16, voff, soff, 0, 0);
}
__device__ __forceinline__ void sk_buf_lds_nt(__amdgpu_buffer_rsrc_t rs, char* lds, uint32_t voff, uint32_t soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)lds, 16, voff, soff, 0, 2);
}

__device__ __forceinline__ bf16x8 sk_frag(const char* lds, int row, int chunk) {
  return *reinterpret_cast<const bf16x8*>(lds + row * 128 + sk_swz(row, chunk) * 16);
}

typedef unsigned int sk_u32x4 __attribute__((ext_vector_type(4)));
typedef int sk_i32x4 __attribute__((ext_vector_type(4)));
typedef int sk_i32x8 __attribute__((ext_vector_type(8)));

// fp8 operand: chunks fc and 4 + fc of the 128-byte row (the bf16 path's kk = 0 / kk = 1 reads)
__device__ __forceinline__ sk_i32x8 sk_frag8(const char* lds, int row, int fc) {
  const sk_i32x4 lo = *reinterpret_cast<const sk_i32x4*>(lds + row * 128 + sk_swz(row, fc) * 16);
  const sk_i32x4 hi = *reinterpret_cast<const sk_i32x4*>(lds + row * 128 + sk_swz(row, 4 + fc) * 16);
  return sk_i32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

__device__ __forceinline__ f32x4 sk_mfma8(sk_i32x8 a, sk_i32x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127, 0, 127);
}

// LDS-DMA of 4 B per lane (the Q = 2 scale piece: 64 floats per wave instruction)
__device__ __forceinline__ void sk_buf_lds4(__amdgpu_buffer_rsrc_t rs, char* lds, uint32_t voff, uint32_t soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)lds, 4, voff, soff, 0, 0);
}

__device__ __forceinline__ float sk_silu(float x) { return x / (1.f + __expf(-x)); }

// first block (local index) whose unit range contains unit u, for B blocks splitting U units
// with block i covering [i*U/B, (i+1)*U/B)
__device__ __forceinline__ int sk_block_of(int64_t u, int64_t U, int B) {
  return (int)(((u + 1) * B + U - 1) / U) - 1;
}

// X, W: byte pointers with byte row strides; kt = K-tiles of 128 bytes (bf16: K / 64, fp8: K / 128)
// OCC = 2: two workgroups per CU (128 VGPRs, NBUF = 2 x 32 KiB LDS) -- the decode-GEMM diagnosis
// (profiles/r05_decode_gemm_diagnosis.md) found one workgroup per CU idle on its own DMA round trip.
// NTW = 1: the W pieces stream with the non-temporal policy (MI355X_MICROARCH.md nt-weights).
template <int BM, int BN, int NBUF, int EPI, int Q, int OCC = 1, int NTW = 0>
__global__ __launch_bounds__(NTHR, OCC == 2 ? 4 : 1) void gemm_sk_kernel(const char* __restrict__ X, int64_t ldx,
                                                          const char* __restrict__ W, int64_t ldw,
                                                          const float* __restrict__ sa, const float* __restrict__ sw,
                                                          const bf16* __restrict__ bias, bf16* __restrict__ out,
                                                          int64_t ldo, int M, int N, int kt,
                                                          float* __restrict__ ws, int* __restrict__ cnt) {
  // LDS per buffer: W image, X image, (Q = 2) BM activation scales + 64 W-block scale slots + 64 dummy
  constexpr int WT = BN * 128, XT = BM * 128, ST = Q == 2 ? BM * 4 + 512 : 0, BUF = WT + XT + ST;
  // 8 waves = (BM / 64) X-row groups x WNS W-row groups; every wave owns 64 X rows x BN / WNS W rows
  constexpr int WNS = 8 / (BM / 64);
  constexpr int WR = BN / WNS;         // W rows per wave
  constexpr int NI = WR / 16;          // 16-row W blocks per wave
  constexpr int NH = NI / 2;
  constexpr int LPT = (BN + BM) / 64 + (Q == 2);  // LDS-DMA pieces per thread per K-tile
  static_assert(BM == 128 || BM == 256, "BM");
  static_assert(Q == 0 || NH <= 2, "fp8: 64 accumulator + 2 x 32 X + 2 x 8 NH W fragment registers");
  static_assert(NH >= 1 && NBUF >= 2 && NBUF <= 4, "tile");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wn = wave % WNS, wm = wave / WNS, fr = lane & 15, fc = lane >> 4;

  const int tiles_m = (M + BM - 1) / BM, T = tiles_m * (N / BN);
  const int grp = blockIdx.x & 7, lb = blockIdx.x >> 3, B = gridDim.x >> 3;
  const int tile_lo = (int)((int64_t)T * grp / 8), tile_hi = (int)((int64_t)T * (grp + 1) / 8);
  // whole tiles round-robin over the group's blocks (round r: tiles tile_lo + r*B + 0..B-1, so the
  // blocks running together share W panels and X row tiles in the XCD's L2), then the remaining
  // tiles' (tile, k-step) units split evenly: stream-K
  const int R = (tile_hi - tile_lo) / B;
  const int sk_lo = tile_lo + R * B;
  const int64_t U = (int64_t)(tile_hi - sk_lo) * kt;
  const int64_t u_beg = (int64_t)lb * U / B, u_end = (int64_t)(lb + 1) * U / B;

  auto bw = [&](int b) { return smem + b * BUF; };
  auto bx = [&](int b) { return smem + b * BUF + WT; };
  auto bs = [&](int b) { return smem + b * BUF + WT + XT; };

  f32x4 acc[NI][4];
  bf16x8 x0[4], x1[4], wa[NH], wb[NH];
  sk_i32x8 xa8[4], xb8[4], wa8[NH], wb8[NH];   // fp8 path (dead code for Q = 0)
  float sc0[5], sc1[5];                          // Q = 2: 4 row scales + the W block scale per K-tile

  int r = 0;
  int64_t u = u_beg;
  while (true) {
    int tile, t0, t1, tl = 0;
    if (r < R) {
      tile = tile_lo + r * B + lb;
      t0 = 0;
      t1 = kt;
      ++r;
    } else if (u < u_end) {
      tl = (int)(u / kt);                          // tile index inside the stream-K range
      tile = sk_lo + tl;
      t0 = (int)(u - (int64_t)tl * kt);
      const int64_t te = (int64_t)(tl + 1) * kt;
      t1 = (int)((u_end < te ? u_end : te) - (int64_t)tl * kt);
      u += t1 - t0;
    } else {
      break;
    }
    const int nt = t1 - t0;
    const int tn = tile / tiles_m, tm = tile - tn * tiles_m;
    const int m0 = tm * BM, n0 = tn * BN;

#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // One K-tile = LPT DMA pieces per thread (piece q < BN/64: 8 W rows x 128 B per wave
    // instruction, else 8 X rows).  The pieces of tile T are threaded through the MFMA phases:
    // S4 of them in phase 4 of iteration T - NBUF (right after the barrier that frees buffer
    // T % NBUF), S1 in phase 1 and S2 in phase 2 of iteration T - NBUF + 1 -- an LDS-DMA issue
    // costs 60-185 cycles, and issued as one burst by every wave right after a barrier it left
    // the MFMA pipe idle (measured: ~25 % of the kernel, profiles/r04_gemm_sk_probe.txt).
    constexpr int PW = BN / 64;
    constexpr int S4 = (LPT + 2) / 3, S1 = (LPT + 1) / 3, S2 = LPT - S4 - S1;
    // buffer_load ... lds: scalar base per segment (the tile's first W / X row), one 32-bit
    // loop-invariant row offset per piece and the K offset in soffset -- 1 VGPR per piece
    // instead of a 64-bit address (the 64-bit form spilled at BN = 256)
    const auto rsw = __builtin_amdgcn_make_buffer_rsrc((void*)(W + (int64_t)n0 * ldw), (short)0, 0x7fffffff,
                                                       0x00020000);
    const auto rsx = __builtin_amdgcn_make_buffer_rsrc((void*)(X + (int64_t)m0 * ldx), (short)0, 0x7fffffff,
                                                       0x00020000);
    // Q = 2 scale piece: waves < BM/64 land 64 activation-row scales each, wave BM/64 the tile's
    // W block scales (lanes < BN/128), the rest re-read those into a dummy slot (uniform counts)
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    const auto rss = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(Q != 2 ? (const float*)X : wv < BM / 64 ? sa + (int64_t)m0 * kt : sw + (int64_t)(n0 >> 7) * kt),
        (short)0, 0x7fffffff, 0x00020000);
    const int sdst = wv < BM / 64 ? wv * 256 : wv == BM / 64 ? BM * 4 : BM * 4 + 256;
    uint32_t vo[LPT];
#pragma unroll
    for (int q = 0; q < LPT; ++q) {
      if (q < PW) {
        const int r = (wave * PW + q) * 8 + (lane >> 3);
        vo[q] = (uint32_t)(r * ldw + sk_swz(r, lane & 7) * 16);
      } else if (q < PW + BM / 64) {
        const int r = (wave * (BM / 64) + (q - PW)) * 8 + (lane >> 3);
        const int rr = m0 + r < M ? r : M - 1 - m0;   // rows past M re-read the last row
        vo[q] = (uint32_t)(rr * ldx + sk_swz(r, lane & 7) * 16);
      } else if (wv < BM / 64) {
        const int r = wv * 64 + lane;
        vo[q] = (uint32_t)((m0 + r < M ? r : M - 1 - m0) * kt * 4);
      } else {
        vo[q] = (uint32_t)((lane < BN / 128 ? lane : 0) * kt * 4);
      }
    }
    auto piece = [&](int t, int b, auto q_tag) {
      constexpr int q = decltype(q_tag)::value;
      if constexpr (q < PW && NTW)
        sk_buf_lds_nt(rsw, bw(b) + (wave * PW + q) * 1024, vo[q], t * 128);
      else if constexpr (q < PW)
        sk_buf_lds(rsw, bw(b) + (wave * PW + q) * 1024, vo[q], t * 128);
      else if constexpr (q < PW + BM / 64)
        sk_buf_lds(rsx, bx(b) + (wave * (BM / 64) + q - PW) * 1024, vo[q], t * 128);
      else
        sk_buf_lds4(rss, bs(b) + sdst, vo[q], t * 4);
    };
    auto pieces = [&](int T, int b, auto q0_tag, auto q1_tag) {   // pieces [q0, q1) of relative tile T
      constexpr int q0 = decltype(q0_tag)::value, q1 = decltype(q1_tag)::value;
      // issued unconditionally (no branch: a branch cuts the scheduling region and the pieces
      // could not be threaded between MFMAs); past the segment's last K-tile they re-read that
      // tile into a buffer nothing reads any more -- in bounds, and retired in issue order by the
      // next vmcnt wait, before any later DMA into the same buffer lands
      const int t = t0 + (T < nt ? T : nt - 1);
      if constexpr (q0 < q1) piece(t, b, std::integral_constant<int, q0>{});
      if constexpr (q0 + 1 < q1) piece(t, b, std::integral_constant<int, q0 + 1>{});
      if constexpr (q0 + 2 < q1) piece(t, b, std::integral_constant<int, q0 + 2>{});
      if constexpr (q0 + 3 < q1) piece(t, b, std::integral_constant<int, q0 + 3>{});
    };
    using I0 = std::integral_constant<int, 0>;
    using IS4 = std::integral_constant<int, S4>;
    using IS41 = std::integral_constant<int, S4 + S1>;
    using ILPT = std::integral_constant<int, LPT>;
    auto stage_all = [&](int T, int b) {
      pieces(T, b, I0{}, IS4{});
      pieces(T, b, IS4{}, IS41{});
      pieces(T, b, IS41{}, ILPT{});
    };
    auto rdx = [&](bf16x8 (&fx)[4], const char* lx, int kk) {
#pragma unroll
      for (int j = 0; j < 4; ++j) fx[j] = sk_frag(lx, wm * 64 + j * 16 + fr, kk * 4 + fc);
    };
    auto rdw = [&](bf16x8 (&fw)[NH], const char* lw, int kk, int ih) {
#pragma unroll
      for (int i = 0; i < NH; ++i) fw[i] = sk_frag(lw, wn * WR + (ih * NH + i) * 16 + fr, kk * 4 + fc);
    };
    auto mm = [&](const bf16x8 (&fx)[4], const bf16x8 (&fw)[NH], int ih) {
#pragma unroll
      for (int i = 0; i < NH; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[ih * NH + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[i], fx[j], acc[ih * NH + i][j], 0, 0, 0);
    };
    // schedule of one phase: its MFMAs with NV DMA pieces and the NR fragment reads of the NEXT
    // phase (issued after them in program order) threaded one per MFMA gap, so the reads land
    // while the MFMAs run and the next phase's MFMAs find their operands without a wait (T19)
    auto interleave = [&](auto nr_tag, auto nv_tag) {
      constexpr int NR = decltype(nr_tag)::value, NV = decltype(nv_tag)::value;
#pragma unroll
      for (int k = 0; k < 4 * NH; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);             // 1 MFMA
        if (k < NV) __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);  // 1 LDS-DMA piece
        if (k < NR) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 DS read
      }
    };
    auto bufp = [&](int k) { return k >= NBUF ? k - NBUF : k; };   // k < 2 * NBUF

    // ---- prologue: tiles 0 .. NBUF-2 whole, the phase-4 share of tile NBUF-1, wait for tile 0
    // (tiles past the segment's end are clamped re-reads, so the counted wait is exact either way)
    stage_all(0, 0);
    if constexpr (NBUF >= 3) stage_all(1, 1);
    if constexpr (NBUF >= 4) stage_all(2, 2);
    constexpr int INFL = (NBUF - 2) * LPT;   // pieces younger than the tile being waited for
    if (INFL > 0 && nt > 1)
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(INFL) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    pieces(NBUF - 1, NBUF - 1, I0{}, IS4{});
    int cur = 0;
    if constexpr (Q != 0) {
      // ---- fp8: two phases of 4*NH MFMAs per K-tile (W half ih = 0, 1); X fragments double-
      // buffered across K-tiles (xa8 / xb8: the iteration body is unrolled twice)
      auto rdx8 = [&](sk_i32x8 (&fx)[4], float (&sc)[5], int b) {
#pragma unroll
        for (int j = 0; j < 4; ++j) fx[j] = sk_frag8(bx(b), wm * 64 + j * 16 + fr, fc);
        if constexpr (Q == 2) {
          const char* ls = bs(b);
#pragma unroll
          for (int j = 0; j < 4; ++j) sc[j] = *reinterpret_cast<const float*>(ls + (wm * 64 + j * 16 + fr) * 4);
          sc[4] = *reinterpret_cast<const float*>(ls + BM * 4 + ((wn * WR) >> 7) * 4);
        }
      };
      auto rdw8 = [&](sk_i32x8 (&fw)[NH], int b, int ih) {
#pragma unroll
        for (int i = 0; i < NH; ++i) fw[i] = sk_frag8(bw(b), wn * WR + (ih * NH + i) * 16 + fr, fc);
      };
      auto mm8 = [&](const sk_i32x8 (&fx)[4], const sk_i32x8 (&fw)[NH], int ih, const float (&sc)[5]) {
#pragma unroll
        for (int i = 0; i < NH; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if constexpr (Q == 2) {
              const f32x4 p = sk_mfma8(fw[i], fx[j], f32x4{0.f, 0.f, 0.f, 0.f});
              acc[ih * NH + i][j] += p * (sc[j] * sc[4]);
            } else {
              acc[ih * NH + i][j] = sk_mfma8(fw[i], fx[j], acc[ih * NH + i][j]);
            }
          }
      };
      // up to 3 fragment reads per MFMA gap (a 16x16x128 fp8 MFMA is twice a bf16 one)
      auto interleave8 = [&](auto nr_tag, auto nv_tag) {
        constexpr int NR = decltype(nr_tag)::value, NV = decltype(nv_tag)::value;
        constexpr int PER = (NR + 4 * NH - 1) / (4 * NH);
#pragma unroll
        for (int k = 0; k < 4 * NH; ++k) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          if (k < NV) __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);
          if (k * PER < NR) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          if (PER > 1 && k * PER + 1 < NR) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          if (PER > 2 && k * PER + 2 < NR) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
      };
      constexpr int NRX = 8 + (Q == 2 ? 5 : 0);
      auto it8 = [&](int i, sk_i32x8 (&xc)[4], sk_i32x8 (&xn)[4], float (&sc)[5], float (&sn)[5]) {
        const int nb = bufp(cur + NBUF - 1);
        mm8(xc, wa8, 0, sc);
        rdw8(wb8, cur, 1);
        pieces(i + NBUF - 1, nb, IS4{}, ILPT{});
        interleave8(std::integral_constant<int, 2 * NH>{}, std::integral_constant<int, LPT - S4>{});
        if (INFL > 0 && i + 2 < nt)
          asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(INFL) : "memory");
        else
          asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        const int freed = cur;
        cur = cur + 1 == NBUF ? 0 : cur + 1;
        mm8(xc, wb8, 1, sc);
        rdx8(xn, sn, cur);
        rdw8(wa8, cur, 0);
        pieces(i + NBUF, freed, I0{}, IS4{});
        interleave8(std::integral_constant<int, NRX + 2 * NH>{}, std::integral_constant<int, S4>{});
      };
      rdx8(xa8, sc0, 0);
      rdw8(wa8, 0, 0);
      int i = 0;
      for (; i + 1 < nt; i += 2) {
        it8(i, xa8, xb8, sc0, sc1);
        it8(i + 1, xb8, xa8, sc1, sc0);
      }
      if (i < nt) it8(i, xa8, xb8, sc0, sc1);
    } else {
    rdx(x0, bx(0), 0);
    rdw(wa, bw(0), 0, 0);
    for (int i = 0; i < nt; ++i) {
      const char* lw = bw(cur);
      const char* lx = bx(cur);
      const int nb = bufp(cur + NBUF - 1);   // buffer of tile i + NBUF - 1 (freed in iteration i - 1)
      // four phases of 4*NH MFMAs (k-half kk, W half ih); each threads the next phase's reads
      mm(x0, wa, 0);                       // (kk0, ih0)
      rdw(wb, lw, 0, 1);
      pieces(i + NBUF - 1, nb, IS4{}, IS41{});
      interleave(std::integral_constant<int, NH>{}, std::integral_constant<int, S1>{});
      mm(x0, wb, 1);                       // (kk0, ih1)
      rdx(x1, lx, 1);
      rdw(wa, lw, 1, 0);
      pieces(i + NBUF - 1, nb, IS41{}, ILPT{});
      interleave(std::integral_constant<int, 4 + NH>{}, std::integral_constant<int, S2>{});
      mm(x1, wa, 0);                       // (kk1, ih0)
      rdw(wb, lw, 1, 1);
      interleave(std::integral_constant<int, NH>{}, I0{});
      // K-tile i + 1 landed for this wave (tiles i + 2 .. i + NBUF - 1 may stay in flight), every
      // LDS read of tile i retired, then the barrier publishes tile i + 1
      if (INFL > 0 && i + 2 < nt)
        asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(INFL) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      const int freed = cur;
      cur = cur + 1 == NBUF ? 0 : cur + 1;
      mm(x1, wb, 1);                       // (kk1, ih1) + the next tile's first fragments
      rdx(x0, bx(cur), 0);                 // (read unconditionally: past the last tile they are
      rdw(wa, bw(cur), 0, 0);              //  unused in-bounds LDS words)
      pieces(i + NBUF, freed, I0{}, IS4{});   // tile i + NBUF into the buffer tile i just left
      interleave(std::integral_constant<int, 4 + NH>{}, std::integral_constant<int, S4>{});
    }
    }

    // ---- partial tile: fp32 slab in fragment order + ticket; the last arriver reduces.
    // Write-through (sc1) slab stores and sc1 loads, so no release / acquire fence is needed
    // (MI355X_MICROARCH.md "Valid forms", table row 1: every storing wave vmcnt(0) -> barrier ->
    // one lane's relaxed agent-scope add; the last adder's workgroup loads every slab with sc1
    // loads).  A fence here would write back the XCD L2's whole dirty set (~128 KiB per block).
    if (nt != kt) {
      const int64_t ts = (int64_t)tl * kt, te = ts + kt;   // the tile's units
      const int first = sk_block_of(ts, U, B);
      auto slab = [&](int blk) {   // one slab per (block, head-of-tile?) -> unique per segment
        const int gb = blk * 8 + grp;
        return __builtin_amdgcn_make_buffer_rsrc(ws + ((int64_t)gb * 2 + (blk == first ? 1 : 0)) * (int64_t)(BM * BN),
                                                 (short)0, BM * BN * 4, 0x00020000);
      };
      {
        const auto rs = slab(lb);
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(sk_u32x4, acc[i][j]), rs,
                                                   ((i * 4 + j) * NTHR + tid) * 16, 0, 16 /* sc1 */);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();   // every wave's slab stores are complete; every wave is past its LDS reads
      int narr = 0;      // arrivals = non-empty blocks whose range meets the tile
      for (int blk = first;;) {
        ++narr;
        const int64_t nu = (int64_t)(blk + 1) * U / B;
        if (nu >= te) break;
        blk = sk_block_of(nu, U, B);
      }
      int* flag = reinterpret_cast<int*>(smem);
      if (tid == 0) {
        const int tk = __hip_atomic_fetch_add(&cnt[tile], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        flag[0] = tk == narr - 1;
        if (tk == narr - 1) __hip_atomic_store(&cnt[tile], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // re-arm
      }
      __syncthreads();
      const bool is_last = flag[0] != 0;
      __syncthreads();   // flag word read by every wave before the next segment's DMA reuses LDS
      if (!is_last) continue;
      for (int blk = first;;) {
        if (blk != lb) {
          const auto rs = slab(blk);
#pragma unroll
          for (int ih = 0; ih < 2; ++ih) {   // half a slab per pass: 16 (BN 256) / 8 loads in flight
            f32x4 v[NH][4];
#pragma unroll
            for (int i = 0; i < NH; ++i)
#pragma unroll
              for (int j = 0; j < 4; ++j)
                v[i][j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                        rs, (((ih * NH + i) * 4 + j) * NTHR + tid) * 16, 0, 16));
#pragma unroll
            for (int i = 0; i < NH; ++i)
#pragma unroll
              for (int j = 0; j < 4; ++j) acc[ih * NH + i][j] += v[i][j];
          }
        }
        const int64_t nu = (int64_t)(blk + 1) * U / B;
        if (nu >= te) break;
        blk = sk_block_of(nu, U, B);
      }
    }

    // ---- epilogue: lane (fr, fc) of (i, j) holds C[m0 + wm*64 + j*16 + fr][n0 + wn*WR + i*16 + 4fc .. +3]
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = m0 + wm * 64 + j * 16 + fr;
      if (m >= M) continue;
      if constexpr (Q == 1) {   // per-token x per-channel (W row) scales
        const float srow = sa[m];
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          const f32x4 sv = *reinterpret_cast<const f32x4*>(sw + n0 + wn * WR + i * 16 + 4 * fc);
          acc[i][j] *= sv * srow;
        }
      }
      if constexpr (EPI == SK_BF16) {
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          const int n = n0 + wn * WR + i * 16 + 4 * fc;
          bf16x4 v;
          if (bias) {
            const bf16x4 bv = *reinterpret_cast<const bf16x4*>(bias + n);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = (bf16)(acc[i][j][r] + (float)bv[r]);
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = (bf16)acc[i][j][r];
          }
          *reinterpret_cast<bf16x4*>(out + (int64_t)m * ldo + n) = v;
        }
      } else {
        // gate / up weight rows interleaved in 16-row blocks: W block 2i = gate, 2i + 1 = up
#pragma unroll
        for (int i = 0; i < NI; i += 2) {
          const int n = ((n0 + wn * WR + i * 16) >> 1) + 4 * fc;
          bf16x4 v;
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = (bf16)(sk_silu(acc[i][j][r]) * acc[i + 1][j][r]);
          *reinterpret_cast<bf16x4*>(out + (int64_t)m * ldo + n) = v;
        }
      }
    }
  }
}

template <int BM, int BN, int NBUF, int EPI, int Q, int OCC = 1, int NTW = 0>
int launch_sk(const void* X, int64_t ldx, const void* W, int64_t ldw, const float* sa, const float* sw,
              const void* bias, void* out, int64_t ldo, int M, int N, int kt, int nwg, float* ws, int* cnt,
              hipStream_t stream) {
  constexpr int LDS = NBUF * ((BN + BM) * 128 + (Q == 2 ? BM * 4 + 512 : 0));
  static_assert(LDS <= 160 * 1024, "LDS");
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)gemm_sk_kernel<BM, BN, NBUF, EPI, Q, OCC, NTW>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  gemm_sk_kernel<BM, BN, NBUF, EPI, Q, OCC, NTW><<<nwg, NTHR, LDS, stream>>>((const char*)X, ldx, (const char*)W, ldw, sa, sw,
                                                              (const bf16*)bias, (bf16*)out, ldo, M, N, kt, ws, cnt);
  return (int)hipGetLastError();
}

}  // namespace

// X [M][K] (row stride ldx), W [N][K] (row stride ldw), out [M][N] (or [M][N/2] for epi = 2).
// Tiles (bm x bn): 256 x 256 (2 LDS buffers, 128 KiB), 256 x 128 (3, 144 KiB), 128 x 256 (3,
// 144 KiB: twice the W bytes in flight per CU of 256 x 128 -- the decode shapes are HBM-latency
// bound), 128 x 128 (4, 128 KiB).  N % bn == 0, K % 64 == 0, nwg % 8 == 0 (1..4096 blocks, one
// per CU resident).  ws: >= nwg * 2 * bm * bn floats; cnt: >= ceil(M/bm) * N/bn ints, zero
// before the first launch (the kernel re-arms them: HIP-graph replayable).  epi 0: bf16
// (+ optional bias[N]); epi 2: SiLU(gate) * up with gate/up rows interleaved in 16-row blocks.
OME_API int ome_gemm_sk(const void* X, int64_t ldx, const void* W, int64_t ldw, const void* bias, void* out,
                        int64_t ldo, int M, int N, int K, int bm, int bn, int epi, int nwg, void* ws, void* cnt,
                        hipStream_t stream) {
  if (M <= 0) return 0;
  if ((bm != 128 && bm != 256) || (bn != 128 && bn != 256) || N % bn || K % BK || K <= 0 || nwg < 8 ||
      nwg % 8 || nwg > 4096)
    return -2;
  if (ldx % 8 || ldw % 8 || ((uintptr_t)X | (uintptr_t)W) % 16 || ldo % 4 || (uintptr_t)out % 8) return -3;
  if (epi != SK_BF16 && epi != SK_SILU) return -4;
  if (epi == SK_SILU && bias) return -4;
  if (!ws || !cnt) return -5;
  float* w = (float*)ws;
  int* c = (int*)cnt;
#define SK_GO(BMV, BNV, NB)                                                                                     \
  return epi == SK_BF16 ? launch_sk<BMV, BNV, NB, SK_BF16, 0>(X, ldx * 2, W, ldw * 2, nullptr, nullptr, bias, out, \
                                                             ldo, M, N, K / BK, nwg, w, c, stream)                \
                        : launch_sk<BMV, BNV, NB, SK_SILU, 0>(X, ldx * 2, W, ldw * 2, nullptr, nullptr, bias, out, \
                                                             ldo, M, N, K / BK, nwg, w, c, stream)
  // decode-GEMM variants (OME_SK_VARIANT, 128 x 128 only): 1 = two workgroups per CU, 2 = nt W
  // stream, 3 = both
  static const int var = getenv("OME_SK_VARIANT") ? atoi(getenv("OME_SK_VARIANT")) : 0;
  if (bm == 128 && bn == 128 && var) {
#define SK_V(NB, OC, NT)                                                                                          \
  return epi == SK_BF16 ? launch_sk<128, 128, NB, SK_BF16, 0, OC, NT>(X, ldx * 2, W, ldw * 2, nullptr, nullptr,   \
                                                                      bias, out, ldo, M, N, K / BK, nwg, w, c,   \
                                                                      stream)                                    \
                        : launch_sk<128, 128, NB, SK_SILU, 0, OC, NT>(X, ldx * 2, W, ldw * 2, nullptr, nullptr,   \
                                                                      bias, out, ldo, M, N, K / BK, nwg, w, c,   \
                                                                      stream)
    if (var == 1) SK_V(2, 2, 0);
    if (var == 2) SK_V(4, 1, 1);
    SK_V(2, 2, 1);
#undef SK_V
  }
  if (bm == 256 && bn == 256) SK_GO(256, 256, 2);
  if (bm == 256) SK_GO(256, 128, 3);
  if (bn == 256) SK_GO(128, 256, 3);
  SK_GO(128, 128, 4);
#undef SK_GO
}

// FP8 W8A8: X [M][K] e4m3 (row stride ldx bytes), W [N][K] e4m3; block 0: sa [M] per token, sw [N]
// per channel; block 128: sa [M][K/128], sw [N/128][K/128].  Tiles 128 x 128, 128 x 256 (per-channel
// only) (K % 128 == 0); epi / nwg / ws / cnt as ome_gemm_sk (epi 2 needs sw in the interleaved row order).
OME_API int ome_gemm_sk_fp8(const void* X, int64_t ldx, const float* sa, const void* W, int64_t ldw, const float* sw,
                            int block, const void* bias, void* out, int64_t ldo, int M, int N, int K, int bm, int bn,
                            int epi, int nwg, void* ws, void* cnt, hipStream_t stream) {
  if (M <= 0) return 0;
  if (bm != 128 || (bn != 128 && bn != 256) || N % bn || K % 128 ||
      K <= 0 || nwg < 8 || nwg % 8 || nwg > 4096 || (block != 0 && block != 128))
    return -2;
  if (ldx % 16 || ldw % 16 || ((uintptr_t)X | (uintptr_t)W) % 16 || ldo % 4 || (uintptr_t)out % 8) return -3;
  if ((uintptr_t)sw % 16 || !sa || !sw) return -3;
  if (epi != SK_BF16 && epi != SK_SILU) return -4;
  if (epi == SK_SILU && bias) return -4;
  if (!ws || !cnt) return -5;
  float* w = (float*)ws;
  int* c = (int*)cnt;
  const int kt = K / 128;
#define SK8_Q(BMV, BNV, NB, QV)                                                                                      \
  return epi == SK_BF16 ? launch_sk<BMV, BNV, NB, SK_BF16, QV>(X, ldx, W, ldw, sa, sw, bias, out, ldo, M, N, kt, nwg, \
                                                               w, c, stream)                                          \
                        : launch_sk<BMV, BNV, NB, SK_SILU, QV>(X, ldx, W, ldw, sa, sw, bias, out, ldo, M, N, kt, nwg, \
                                                               w, c, stream)
  // 256 x 128 and the block-scaled 128 x 256 spill at 256 VGPRs: not offered
  if (bn == 256) {
    if (block) return -2;
    SK8_Q(128, 256, 3, 1);
  }
  if (block) SK8_Q(128, 128, 4, 2);
  SK8_Q(128, 128, 4, 1);
#undef SK8_Q
}
