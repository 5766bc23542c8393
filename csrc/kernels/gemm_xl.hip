// Large-tile bf16 GEMM for the mixed-step / prefill projections, "NT" layout:
//   C[M][N] = X[M][K] . W[N][K]^T  (+ bias)          (= F.linear(x, w))
//
// Round-6 body (after gemm_pp.hip measured 1.15-1.2 PF at 4096^3 with 8 waves in ping-pong, its
// LDS-DMA issue not hidden between the 16-cycle 16x16x32 MFMAs):
//   * ONE wave per SIMD (256 threads, up to 512 registers per lane): every wave owns a 128 (m) x
//     BN/2 (n) output tile as 4 x BN/64 accumulators of v_mfma_f32_32x32x16_bf16 (256 AGPRs at
//     BN = 256).  A 32x32x16 MFMA holds the SIMD's issue for 8 of its 32 cycles, so each MFMA gap
//     has room for a fragment read and a DMA piece (MI355X_MICROARCH.md, cycle constants) without a
//     partner wave; the LDS fragment bytes per FLOP are those of a 128 x 128 wave tile (half of the
//     128 x 64 tile of gemm_pp).
//   * BK = 32 K-tiles (64-byte LDS image rows) in NBUF = 4..6 LDS stages filled by buffer_load ... lds
//     (lane-linear images, bank swizzle on the SOURCE address: chunk ^ ((row >> 2) & 3)); the DMA of
//     tile t + NBUF - 1 is issued while tile t computes, so every piece has NBUF - 2 K-tiles (>= 2
//     x 1024 MFMA cycles) to land -- counted vmcnt, one raw s_barrier per K-tile.
//   * Per K-tile two half-steps (k 0..15, 16..31): the MFMAs of one half run while the fragments of
//     the next half are read (double-buffered fragment registers), threaded one per MFMA gap with
//     sched_group_barrier.
//   * Decomposition: the persistent per-XCD stream-K of gemm_sk.hip (whole tiles round-robin, the
//     rest split into (tile, k-tile) units; partial tiles go through fp32 slabs in fragment order,
//     write-through stores + relaxed agent ticket, the tile's last arriver adds them into its own
//     registers and runs the epilogue), so N = 4096 / 6144 projections at M = 512..2304 fill all
//     256 CUs with 256 x 256 or 256 x 128 tiles.
//   * Epilogues: bf16 (+bias), SiLU(gate) * up for gate/up weights interleaved in 16-row blocks
//     (ops.interleave_gate_up: a 32-row W fragment = one gate block + one up block).
// Probe builds (PROBE = 1: no DMA in the K loop; 2: no DMA and no fragment reads) time the
// skeleton, as scripts/gemm_xl_bench.py --probe does.
#include "common.h"

typedef __attribute__((address_space(3))) void xl_lds_t;

namespace {

constexpr int XL_NT = 256, XL_BM = 256;
enum { XL_BF16 = 0, XL_SILU = 2 };

typedef short xl_s16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int xl_u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int xl_swz(int row, int chunk) { return chunk ^ ((row >> 2) & 3); }

__device__ __forceinline__ void xl_dma(__amdgpu_buffer_rsrc_t rs, char* lds, uint32_t voff, uint32_t soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (xl_lds_t*)lds, 16, voff, soff, 0, 0);
}

// 32 rows x 16 k of a 64-byte-row image: lane l reads row (l & 31), 16-byte chunk s * 2 + (l >> 5)
__device__ __forceinline__ bf16x8 xl_frag(const char* img, int row, int chunk) {
  return *reinterpret_cast<const bf16x8*>(img + row * 64 + xl_swz(row, chunk) * 16);
}

__device__ __forceinline__ f32x16 xl_mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float xl_silu(float x) { return x / (1.f + __expf(-x)); }

__device__ __forceinline__ int xl_block_of(int64_t u, int64_t U, int B) {
  return (int)(((u + 1) * B + U - 1) / U) - 1;
}

// X, W: bf16 with element row strides; kt = K / 32
template <int BN, int NBUF, int EPI, int PROBE, int STG>
__global__ __launch_bounds__(STG == 2 ? 2 * XL_NT : XL_NT, 1) void gemm_xl_kernel(const bf16* __restrict__ X, int64_t ldx,
                                                           const bf16* __restrict__ W, int64_t ldw,
                                                           const bf16* __restrict__ bias, bf16* __restrict__ out,
                                                           int64_t ldo, int M, int N, int kt,
                                                           float* __restrict__ ws, int* __restrict__ cnt) {
  constexpr int BM = XL_BM;
  constexpr int NW = BN / 64;                 // 32-row W fragments per wave (wave owns BN / 2 W rows)
  constexpr int WT = BN * 64, BUF = WT + BM * 64;
  constexpr int P = (BN + BM) / 64;           // DMA pieces (16 rows x 64 B) per thread per K-tile
  constexpr int PA = (P + 1) / 2, PB = P - PA;   // pieces issued in half A / half B
  constexpr int INFL = P * (NBUF - 3) + PA;   // pieces younger than tile t + 1 at iteration t's barrier
  static_assert((STG == 1 ? NBUF == 3 : NBUF >= 4 && NBUF <= 6) && NBUF * BUF <= 160 * 1024, "stages");
  static_assert(STG != 2 || BN == 128, "warp-specialised body: 128 acc registers per MFMA wave");
  static_assert(STG == 0 || PROBE == 0, "probes run on the LDS-DMA body");
  static_assert(INFL < 64, "vmcnt");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // STG = 2: waves 0-3 compute (MFMA + fragment reads only), waves 4-7 only stage (LDS-DMA):
  // a DMA issue (60-185 cycles, MI355X_MICROARCH.md) then never stalls an MFMA stream
  const bool producer = STG == 2 && wave >= 4;
  const int pw = STG == 2 ? (wave & 3) : wave;   // staging wave index
  const int wm = wave & 1, wn = (wave >> 1) & 1;
  const int l32 = lane & 31, lh = lane >> 5;

  const int tiles_m = (M + BM - 1) / BM, T = tiles_m * (N / BN);
  const int grp = blockIdx.x & 7, lb = blockIdx.x >> 3, B = gridDim.x >> 3;
  const int tile_lo = (int)((int64_t)T * grp / 8), tile_hi = (int)((int64_t)T * (grp + 1) / 8);
  const int R = (tile_hi - tile_lo) / B;
  const int sk_lo = tile_lo + R * B;
  const int64_t U = (int64_t)(tile_hi - sk_lo) * kt;
  const int64_t u_beg = (int64_t)lb * U / B, u_end = (int64_t)(lb + 1) * U / B;

  f32x16 acc[NW][4];
  bf16x8 fa[NW + 4], fb[NW + 4];   // fragments of half A / half B: W 0..NW-1, X NW..NW+3

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
      tl = (int)(u / kt);
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
    for (int i = 0; i < NW; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x16{};

    // piece q of this wave = image rows (wave * P + q) * 16 .. + 16 (W rows first, then X rows);
    // lane L: image row + (L >> 2), 16-byte slot L & 3.  The swizzle term ((row >> 2) & 3) =
    // (L >> 4) & 3 does not depend on q, so a piece's source offset is one per-lane VGPR (the
    // lane's row / chunk inside the piece) + a uniform SGPR (the piece's first row, the K-tile).
    // X rows past M read as zeros (the X resource ends at row M: buffer range check).
    const auto rsw = __builtin_amdgcn_make_buffer_rsrc((void*)(W + (int64_t)n0 * ldw), (short)0, 0x7fffffff,
                                                       0x00020000);
    const int xrec = (int)min((int64_t)(M - m0) * ldx * 2, (int64_t)0x7fffffff);
    const auto rsx = __builtin_amdgcn_make_buffer_rsrc((void*)(X + (int64_t)m0 * ldx), (short)0, xrec, 0x00020000);
    const int lsw = xl_swz(lane >> 2, lane & 3);   // DMA: source chunk landing in slot lane & 3
    const uint32_t vw = (uint32_t)((lane >> 2) * ldw * 2 + lsw * 16);
    const uint32_t vx = (uint32_t)((lane >> 2) * ldx * 2 + lsw * 16);
    auto prow = [&](int q) { return (pw * P + q) * 16; };   // first image row of piece q (uniform)
    auto poff = [&](int q) {   // uniform byte offset of piece q's first row in its operand
      return prow(q) < BN ? (uint32_t)(prow(q) * ldw * 2) : (uint32_t)((prow(q) - BN) * ldx * 2);
    };
    auto piece = [&](int tr, int q) {   // piece q of relative K-tile tr (clamped to the segment)
      const int t = t0 + (tr < nt ? tr : nt - 1);
      char* dst = smem + (tr % NBUF) * BUF + prow(q) * 64;
      const bool isw = prow(q) < BN;
      xl_dma(isw ? rsw : rsx, dst, isw ? vw : vx, poff(q) + (uint32_t)t * 64);
    };
    // pieces [q0, q1) of relative K-tile tr (q0, q1 compile-time after inlining; fully unrolled)
    auto pieces = [&](int tr, int q0, int q1) {
#pragma unroll
      for (int q = 0; q < P; ++q)
        if (q >= q0 && q < q1) piece(tr, q);
    };

    auto rd = [&](bf16x8 (&f)[NW + 4], int tr, int s) {   // half s of relative K-tile tr
      if constexpr (PROBE == 2) {
#pragma unroll
        for (int i = 0; i < NW + 4; ++i) asm volatile("" : "+v"(f[i]));
        return;
      }
      const char* img = smem + (tr % NBUF) * BUF;
      const int ch = s * 2 + lh;
#pragma unroll
      for (int i = 0; i < NW; ++i) f[i] = xl_frag(img, wn * (BN / 2) + i * 32 + l32, ch);
#pragma unroll
      for (int j = 0; j < 4; ++j) f[NW + j] = xl_frag(img, BN + wm * 128 + j * 32 + l32, ch);
    };
    auto mm = [&](const bf16x8 (&f)[NW + 4]) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < NW; ++i) acc[i][j] = xl_mfma(f[i], f[NW + j], acc[i][j]);
    };
    // one half-step: 4 NW MFMAs with NR fragment reads and NV DMA pieces threaded into the gaps
    auto interleave = [&](auto nr_tag, auto nv_tag) {
      constexpr int NR = decltype(nr_tag)::value, NV = decltype(nv_tag)::value;
      constexpr int NM = 4 * NW;
#pragma unroll
      for (int k = 0; k < NM; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // 1 MFMA
        if (k % 2 == 1 && k / 2 < NV) __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);   // 1 VMEM (DMA)
        if (k < NR) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // 1 DS read
      }
    };

    if constexpr (STG == 2) {
      if (producer) {
#pragma unroll
        for (int tr = 0; tr < NBUF - 1; ++tr) pieces(tr, 0, P);
        asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(P * (NBUF - 2)) : "memory");
#pragma unroll 1
        for (int t = 0; t < nt; ++t) {
          // tile t + NBUF - 1 into the stage tile t - 1 left (read before the last barrier);
          // tile t + 1 landed, then the barrier publishes it
          pieces(t + NBUF - 1, 0, P);
          asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(P * (NBUF - 2)) : "memory");
        }
      } else {
        asm volatile("s_barrier" ::: "memory");
        rd(fa, 0, 0);
#pragma unroll 1
        for (int t = 0; t < nt; ++t) {
          mm(fa);
          rd(fb, t, 1);
          interleave(std::integral_constant<int, NW + 4>{}, std::integral_constant<int, 0>{});
          asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
          mm(fb);
          rd(fa, t + 1, 0);
          interleave(std::integral_constant<int, NW + 4>{}, std::integral_constant<int, 0>{});
        }
      }
    } else if constexpr (STG == 1) {
      // ---- register staging (STG = 1): buffer_load_dwordx4 into 4 register sets, ds_write_b128
      // into 3 LDS stages with the swizzle on the WRITE address.  Tile u is loaded in iteration
      // u - 4 (half A), written in iteration u - 2 (half B) and read in iterations u - 1 / u; the
      // compiler counts the vmcnt of each write (only register-destination VMEM in the loop).
      // linear source chunk lane & 3, swizzled LDS write slot (the same involution as the reads)
      const uint32_t sw_ = (uint32_t)((lane >> 2) * ldw * 2 + (lane & 3) * 16);
      const uint32_t sx_ = (uint32_t)((lane >> 2) * ldx * 2 + (lane & 3) * 16);
      const uint32_t wl = (uint32_t)((lane >> 2) * 64 + xl_swz(lane >> 2, lane & 3) * 16);
      // NS register sets: tile u loaded in iteration u - NS (half A), written in u - 2 (half B)
      constexpr int NS = BN == 256 ? 3 : 4;
      xl_u32x4 sr[NS][P];
      auto gload = [&](int tr, auto set_tag) {
        constexpr int S = decltype(set_tag)::value;
        const uint32_t t = (uint32_t)(t0 + (tr < nt ? tr : nt - 1)) * 64;
#pragma unroll
        for (int q = 0; q < P; ++q)
          sr[S][q] = __builtin_amdgcn_raw_buffer_load_b128(prow(q) < BN ? rsw : rsx, prow(q) < BN ? sw_ : sx_,
                                                           poff(q) + t, 0);
      };
      auto swrite = [&](int tr, auto set_tag) {
        constexpr int S = decltype(set_tag)::value;
        char* st = smem + (tr % 3) * BUF;
#pragma unroll
        for (int q = 0; q < P; ++q) *reinterpret_cast<xl_u32x4*>(st + prow(q) * 64 + wl) = sr[S][q];
      };
      auto ilv_a = [&]() {   // half A: MFMAs + next fragments' reads + the global loads
        constexpr int NM = 4 * NW, NR = NW + 4;
#pragma unroll
        for (int k = 0; k < NM; ++k) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          if (k < P) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
          if (k < NR) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
      };
      auto ilv_b = [&]() {   // half B: MFMAs + the LDS writes + next fragments' reads
        constexpr int NM = 4 * NW, NR = NW + 4;
#pragma unroll
        for (int k = 0; k < NM; ++k) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          if (k < P) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
          if (k < NR) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
      };
      using S0 = std::integral_constant<int, 0>;
      using S1 = std::integral_constant<int, 1>;
      using S2 = std::integral_constant<int, 2>;
      using S3 = std::integral_constant<int, NS == 4 ? 3 : 0>;
      gload(0, S0{});
      gload(1, S1{});
      gload(2, S2{});
      if constexpr (NS == 4) gload(3, S3{});
      swrite(0, S0{});
      swrite(1, S1{});
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      rd(fa, 0, 0);
      auto iter = [&](int t, auto k_tag) {   // k = t % NS
        constexpr int k = decltype(k_tag)::value;
        mm(fa);
        rd(fb, t, 1);
        gload(t + NS, k_tag);
        ilv_a();
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        mm(fb);
        swrite(t + 2, std::integral_constant<int, (k + 2) % NS>{});
        rd(fa, t + 1, 0);
        ilv_b();
      };
#pragma unroll 1
      for (int t = 0; t < nt; t += NS) {
        iter(t, S0{});
        if (t + 1 >= nt) break;
        iter(t + 1, S1{});
        if (t + 2 >= nt) break;
        iter(t + 2, S2{});
        if constexpr (NS == 4) {
          if (t + 3 >= nt) break;
          iter(t + 3, S3{});
        }
      }
      asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    } else {
    // ---- prologue: relative tiles 0 .. NBUF-2, wait for tile 0, read its first half
    if constexpr (PROBE == 0) {
#pragma unroll
      for (int tr = 0; tr < NBUF - 1; ++tr) pieces(tr, 0, P);
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(P * (NBUF - 2)) : "memory");
    } else {   // probes: stage every buffer once, then the loop runs on resident data
#pragma unroll
      for (int tr = 0; tr < NBUF; ++tr) pieces(tr, 0, P);
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    }
    rd(fa, 0, 0);

#pragma unroll 1
    for (int t = 0; t < nt; ++t) {
      // half A: MFMAs on (t, k 0..15); read (t, k 16..31); DMA of tile t + NBUF - 1 (its stage was
      // last read in iteration t - 1, before that iteration's barrier)
      mm(fa);
      rd(fb, t, 1);
      if constexpr (PROBE == 0) pieces(t + NBUF - 1, 0, PA);
      interleave(std::integral_constant<int, NW + 4>{}, std::integral_constant<int, PROBE == 0 ? PA : 0>{});
      // tile t + 1 landed for this wave, every fragment read of tile t retired; the barrier
      // publishes tile t + 1 and frees stage t for the DMA issued in iteration t + 1
      if constexpr (PROBE == 0)
        asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(INFL) : "memory");
      else
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      // half B: MFMAs on (t, k 16..31); read (t + 1, k 0..15) (past the last tile: unused words)
      mm(fb);
      rd(fa, PROBE == 0 ? t + 1 : (t + 1) % NBUF, 0);
      if constexpr (PROBE == 0) pieces(t + NBUF - 1, PA, P);
      interleave(std::integral_constant<int, NW + 4>{}, std::integral_constant<int, PROBE == 0 ? PB : 0>{});
    }
    }
    // clamped tail pieces retire and every wave is past its reads before the stages are reused
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");

    // ---- epilogue of one 32 x 32 accumulator (i, j) given its 16 values: lane l holds
    //      C[m0 + wm*128 + j*32 + (l & 31)][n0 + wn*BN/2 + i*32 + 8g + 4(l >> 5) + e] in value 4g + e
    auto emit = [&](int i, int j, const f32x16& a) {
      const int m = m0 + wm * 128 + j * 32 + l32;
      if (m >= M) return;
      bf16* orow = out + (int64_t)m * ldo;
      if constexpr (EPI == XL_BF16) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int n = n0 + wn * (BN / 2) + i * 32 + 8 * g + 4 * lh;
          bf16x4 v;
          if (bias) {
            const bf16x4 bv = *reinterpret_cast<const bf16x4*>(bias + n);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = (bf16)(a[4 * g + e] + (float)bv[e]);
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = (bf16)a[4 * g + e];
          }
          *reinterpret_cast<bf16x4*>(orow + n) = v;
        }
      } else {
        // W fragment i = rows i*32 .. +32 = gate block (16 rows) + up block (16 rows)
#pragma unroll
        for (int g = 0; g < 2; ++g) {
          const int n = ((n0 + wn * (BN / 2) + i * 32) >> 1) + 8 * g + 4 * lh;
          bf16x4 v;
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = (bf16)(xl_silu(a[4 * g + e]) * a[4 * (g + 2) + e]);
          *reinterpret_cast<bf16x4*>(orow + n) = v;
        }
      }
    };

    // ---- partial tile: every arrival stores its fp32 slab (fragment order, write-through) and
    // takes a ticket; the last arriver sums ALL the tile's slabs one accumulator at a time straight
    // into the epilogue (the registers of the K loop are dead by then: few live VGPRs).  Hand-off:
    // MI355X_MICROARCH.md "Valid forms", row 1 (sc1 stores, vmcnt(0), barrier, one relaxed agent
    // add; sc1 loads by the last adder).
    if (nt != kt) {
      const int64_t ts = (int64_t)tl * kt, te = ts + kt;
      const int first = xl_block_of(ts, U, B);
      auto slab = [&](int blk) {
        const int gb = blk * 8 + grp;
        return __builtin_amdgcn_make_buffer_rsrc(ws + ((int64_t)gb * 2 + (blk == first ? 1 : 0)) * (int64_t)(BM * BN),
                                                 (short)0, BM * BN * 4, 0x00020000);
      };
      if (!producer) {
        const auto rs = slab(lb);
#pragma unroll
        for (int i = 0; i < NW; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const f32x4 v{acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]};
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(xl_u32x4, v), rs,
                                                     (((i * 4 + j) * 4 + q) * XL_NT + tid) * 16, 0, 16 /* sc1 */);
            }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      int narr = 0;
      for (int blk = first;;) {
        ++narr;
        const int64_t nu = (int64_t)(blk + 1) * U / B;
        if (nu >= te) break;
        blk = xl_block_of(nu, U, B);
      }
      int* flag = reinterpret_cast<int*>(smem);
      if (tid == 0) {
        const int tk = __hip_atomic_fetch_add(&cnt[tile], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        flag[0] = tk == narr - 1;
        if (tk == narr - 1) __hip_atomic_store(&cnt[tile], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
      const bool is_last = flag[0] != 0;
      __syncthreads();
      if (!is_last || producer) continue;
#pragma unroll 1
      for (int ij = 0; ij < NW * 4; ++ij) {
        f32x16 a = {};
        for (int blk = first;;) {
          const auto rs = slab(blk);
          f32x4 v[4];
#pragma unroll
          for (int q = 0; q < 4; ++q)
            v[q] = __builtin_bit_cast(f32x4,
                                      __builtin_amdgcn_raw_buffer_load_b128(rs, ((ij * 4 + q) * XL_NT + tid) * 16, 0, 16));
#pragma unroll
          for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int e = 0; e < 4; ++e) a[4 * q + e] += v[q][e];
          const int64_t nu = (int64_t)(blk + 1) * U / B;
          if (nu >= te) break;
          blk = xl_block_of(nu, U, B);
        }
        emit(ij >> 2, ij & 3, a);
      }
      continue;
    }

    if (producer) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < NW; ++i) emit(i, j, acc[i][j]);
  }
}

template <int BN, int NBUF, int EPI, int PROBE, int STG = 0>
int launch_xl(const bf16* X, int64_t ldx, const bf16* W, int64_t ldw, const bf16* bias, bf16* out, int64_t ldo, int M,
              int N, int K, int nwg, float* ws, int* cnt, hipStream_t stream) {
  constexpr int LDS = NBUF * (BN + XL_BM) * 64;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)gemm_xl_kernel<BN, NBUF, EPI, PROBE, STG>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  gemm_xl_kernel<BN, NBUF, EPI, PROBE, STG><<<nwg, STG == 2 ? 2 * XL_NT : XL_NT, LDS, stream>>>(X, ldx, W, ldw, bias, out, ldo, M, N, K / 32, ws,
                                                                  cnt);
  return (int)hipGetLastError();
}

}  // namespace

// X [M][K] (row stride ldx), W [N][K] (row stride ldw), out [M][N] (or [M][N/2] for epi = 2).
// bn 256 (4 LDS stages, 128 KiB) or 128 (6 stages, 144 KiB); bm = 256.  N % bn == 0, K % 32 == 0,
// nwg % 8 == 0 (8..256).  ws >= nwg * 2 * 256 * bn floats, cnt >= ceil(M/256) * N/bn ints, zero
// before the first launch (re-armed by the kernel: HIP-graph replayable).  probe 1 / 2: the
// diagnostic skeletons (wrong results by design).
OME_API int ome_gemm_xl(const void* X, int64_t ldx, const void* W, int64_t ldw, const void* bias, void* out,
                        int64_t ldo, int M, int N, int K, int bn, int epi, int nwg, void* ws, void* cnt, int probe,
                        hipStream_t stream) {
  if (M <= 0) return 0;
  if ((bn != 128 && bn != 256) || N % bn || K % 32 || K <= 0 || nwg < 8 || nwg % 8 || nwg > 256) return -2;
  if (ldx % 8 || ldw % 8 || ((uintptr_t)X | (uintptr_t)W) % 16 || ldo % 4 || (uintptr_t)out % 8) return -3;
  if ((int64_t)XL_BM * ldx * 2 >= 0x7fffffffLL || (int64_t)bn * ldw * 2 >= 0x7fffffffLL ||
      (int64_t)K * 2 >= 0x7fffffffLL)
    return -3;   // 32-bit DMA offsets
  if (epi != XL_BF16 && epi != XL_SILU) return -4;
  if (epi == XL_SILU && bias) return -4;
  if (bias && (uintptr_t)bias % 8) return -3;
  if (!ws || !cnt) return -5;
  const bf16 *x = (const bf16*)X, *w = (const bf16*)W, *b = (const bf16*)bias;
  bf16* o = (bf16*)out;
  float* wsp = (float*)ws;
  int* c = (int*)cnt;
#define XL_GO(BNV, NB, EP, PR) return launch_xl<BNV, NB, EP, PR>(x, ldx, w, ldw, b, o, ldo, M, N, K, nwg, wsp, c, stream)
  if (probe == 5) {   // warp-specialised body (4 MFMA waves + 4 DMA waves), 256 x 128 tiles
    if (epi == XL_SILU) return launch_xl<128, 6, XL_SILU, 0, 2>(x, ldx, w, ldw, b, o, ldo, M, N, K, nwg, wsp, c, stream);
    return launch_xl<128, 6, XL_BF16, 0, 2>(x, ldx, w, ldw, b, o, ldo, M, N, K, nwg, wsp, c, stream);
  }
  if (probe == 4) {   // LDS-DMA body (A/B against register staging)
    if (bn == 256) {
      if (epi == XL_SILU) XL_GO(256, 4, XL_SILU, 0);
      XL_GO(256, 4, XL_BF16, 0);
    }
    if (epi == XL_SILU) XL_GO(128, 6, XL_SILU, 0);
    XL_GO(128, 6, XL_BF16, 0);
  }
  if (probe == 1 && epi == XL_BF16) {
    if (bn == 256) XL_GO(256, 4, XL_BF16, 1);
    XL_GO(128, 6, XL_BF16, 1);
  }
  if (probe == 2 && epi == XL_BF16) {
    if (bn == 256) XL_GO(256, 4, XL_BF16, 2);
    XL_GO(128, 6, XL_BF16, 2);
  }
#define XL_GR(BNV, EP) return launch_xl<BNV, 3, EP, 0, 1>(x, ldx, w, ldw, b, o, ldo, M, N, K, nwg, wsp, c, stream)
  static const int stg = getenv("OME_XL_STG") ? atoi(getenv("OME_XL_STG")) : 1;
  if (stg == 1 || probe == 3) {   // register staging (probe 3: forced, for A/B runs)
    if (bn == 256) {
      if (epi == XL_SILU) XL_GR(256, XL_SILU);
      XL_GR(256, XL_BF16);
    }
    if (epi == XL_SILU) XL_GR(128, XL_SILU);
    XL_GR(128, XL_BF16);
  }
  if (bn == 256) {
    if (epi == XL_SILU) XL_GO(256, 4, XL_SILU, 0);
    XL_GO(256, 4, XL_BF16, 0);
  }
  if (epi == XL_SILU) XL_GO(128, 6, XL_SILU, 0);
  XL_GO(128, 6, XL_BF16, 0);
#undef XL_GO
#undef XL_GR
}
