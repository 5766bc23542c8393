// Ping-pong 256 x 256 bf16 GEMM for the prefill / mixed-step projections,
// "NT" layout:  C[M][N] = X[M][K] . W[N][K]^T  (= F.linear(x, w)), fp32 accumulation.
//
// Why a second GEMM body next to gemm_sk.hip: the stream-K kernel runs its 8 waves in lockstep
// (every wave interleaves its own fragment reads and DMA issue between its MFMAs, one barrier per
// K-tile) and measured 50-66 % of MFMA peak in its LDS -> MFMA loop even with the global loads
// removed (docs/ROUND4.md), so it lost to hipBLASLt at M >= 384.  This body splits each SIMD's two
// waves into two wave GROUPS that run one barrier apart (cdna_hip_programming.md §5 "The 256²
// 8-phase template", MI355X_MICROARCH.md "Two waves per SIMD"): in every barrier interval one
// group only issues MFMAs (a 16-MFMA quadrant, 256 matrix-pipe cycles) while its SIMD partner
// issues the next quadrant's LDS fragment reads and its share of the LDS-DMA staging, then they
// swap.  The matrix pipe of each SIMD alternates between the two waves' MFMA clusters.
//
// Geometry: 512 threads, 1 workgroup / CU, output tile 256 (m) x 256 (n), BK = 64, two LDS
// buffers of {W image 256 x 128 B, X image 256 x 128 B} = 128 KiB.  Wave w: group g = w >> 2
// owns W rows g*128 .. +128 (8 blocks of 16), wi = w & 3 owns X rows wi*64 .. +64 (4 blocks).
// MFMA v_mfma_f32_16x16x32_bf16 with W as the A operand (rows = n) so every lane ends with 4
// consecutive output columns of one row (8-byte bf16 stores).  Per K-tile a wave runs four
// phases (quadrants of its 128 x 64 tile over K = 64, 16 MFMAs each):
//   P0 (W 0-3, X 0-1): reads W0 (8 frags) + Xa (4)     P1 (W 0-3, X 2-3): reads Xb (4) + 4 DMA pieces
//   P2 (W 4-7, X 2-3): reads W1 (8)                    P3 (W 4-7, X 0-1): vmcnt(0), 4 DMA pieces
// Staging: group 0 DMAs the W image, group 1 the X image (8 x 1 KiB pieces per thread and K-tile,
// buffer_load ... lds into lane-linear LDS, the bank swizzle applied on the SOURCE address,
// rule 21).  K-tile t + 2 goes into buffer t & 1: pieces 0-3 in P3 of tile t (the buffer's last
// reader, group 1's P2 of tile t, is one interval behind), pieces 4-7 in P1 of tile t + 1; each
// wave waits vmcnt(0) for its own pieces of tile t + 1 in P3 of tile t, and the barriers after
// both groups' P3 publish it -- the DMA of a tile is in flight across 4-6 barrier intervals.
// Tiles: XCD-aware bijective remap (blocks b, b + 8 share an XCD; each XCD gets a contiguous run
// of tiles, m fastest, so concurrently running tiles share W panels in that XCD's L2).
// Epilogues: bf16 (+bias), SiLU(gate) * up on gate/up rows interleaved in 16-row blocks (the
// act_and_mul pass disappears), and + residual (bf16, the o / down projections).
#include "common.h"

typedef __attribute__((address_space(3))) void pp_lds_t;

namespace {

constexpr int PP_NT = 512, PP_IMG = 256 * 128, PP_BUF = 2 * PP_IMG;
enum { PP_BF16 = 0, PP_RES = 1, PP_SILU = 2 };

__device__ __forceinline__ int pp_swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

__device__ __forceinline__ void pp_dma(__amdgpu_buffer_rsrc_t rs, char* lds, uint32_t voff, uint32_t soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (pp_lds_t*)lds, 16, voff, soff, 0, 0);
}

__device__ __forceinline__ bf16x8 pp_frag(const char* img, int row, int chunk) {
  return *reinterpret_cast<const bf16x8*>(img + row * 128 + pp_swz(row, chunk) * 16);
}

// id -> (m tile, n tile).  gm = 0: m fastest over the whole M extent.  gm > 0: groups of gm m-tiles,
// m fastest inside a group, so the ~32 tiles an XCD runs at once span gm m-panels x 32 / gm
// n-panels (12 distinct panels at gm = 8 instead of 1 W + 32 X panels at M = 8192): fewer L2
// misses per K step.
__device__ __forceinline__ void pp_tile(int id, int tiles_m, int tiles_n, int gm, int& tm, int& tn) {
  if (gm <= 0 || gm >= tiles_m) {
    tn = id / tiles_m;
    tm = id - tn * tiles_m;
    return;
  }
  const int per = gm * tiles_n, g = id / per, first = g * gm, r = id - g * per;
  const int h = min(tiles_m - first, gm);
  tm = first + r % h;
  tn = r / h;
}

__device__ __forceinline__ float pp_silu(float x) { return x / (1.f + __expf(-x)); }

// s_waitcnt lgkmcnt(0) (vmcnt / expcnt left at their maxima), then the barrier; the compiler
// must not move MFMAs or LDS reads across it
__device__ __forceinline__ void pp_bar_lgkm() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
__device__ __forceinline__ void pp_bar() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <int EPI, bool BIAS, int PROBE = 0>
__global__ __launch_bounds__(PP_NT, 1) void gemm_pp_kernel(const bf16* __restrict__ X, int64_t ldx,
                                                           const bf16* __restrict__ W, int64_t ldw,
                                                           const bf16* __restrict__ bias,
                                                           const bf16* __restrict__ res, int64_t ldr,
                                                           bf16* __restrict__ out, int64_t ldo, int M, int N, int kt,
                                                           int gm) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = wave >> 2, wi = wave & 3;
  const int fr = lane & 15, fc = lane >> 4;

  // ---- tile of this workgroup: bijective XCD remap over T tiles, m fastest
  const int tiles_m = (M + 255) >> 8, T = tiles_m * (N >> 8);
  const int b = blockIdx.x, xcd = b & 7, q8 = T >> 3, r8 = T & 7;
  const int id = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  int tm, tn;
  pp_tile(id, tiles_m, N >> 8, gm, tm, tn);
  const int m0 = tm << 8, n0 = tn << 8;

  // ---- staging: group 0 -> W image, group 1 -> X image, 8 pieces of 8 rows x 128 B per wave and
  // K-tile, lane L one 16-byte chunk of row (L >> 3).  Pieces 0-3 of every wave hold the rows the
  // first phase reads (W rows g*128 + 0..63 of both groups, X rows wi*64 + 0..31), pieces 4-7 the
  // rows first read in P1 (X) or P2 (W), so they may land two phases later.
  const auto rs = g == 0 ? __builtin_amdgcn_make_buffer_rsrc((void*)(W + (int64_t)n0 * ldw), (short)0, 0x7fffffff,
                                                            0x00020000)
                         : __builtin_amdgcn_make_buffer_rsrc((void*)(X + (int64_t)m0 * ldx), (short)0, 0x7fffffff,
                                                            0x00020000);
  const int img_off = g == 0 ? 0 : PP_IMG;
  uint32_t vo[8];
  int prow[8];   // first image row of each piece
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    if (g == 0) {   // W: P0 rows {0..63, 128..191}, P2 rows {64..127, 192..255}
      const int blk = wi * 4 + (p & 3);   // 0..15
      prow[p] = (blk & 8) * 16 + (blk & 7) * 8 + (p >> 2) * 64;
    } else {        // X: wave wi's rows wi*64 .. +64, P0 half first
      prow[p] = wi * 64 + p * 8;
    }
    const int row = prow[p] + (lane >> 3);
    const int chunk = pp_swz(row, lane & 7);   // involution: the chunk whose swizzled slot is lane & 7
    if (g == 0) {
      vo[p] = (uint32_t)(row * ldw * 2 + chunk * 16);
    } else {
      const int rr = m0 + row < M ? row : M - 1 - m0;   // rows past M re-read the last row (never stored)
      vo[p] = (uint32_t)(rr * ldx * 2 + chunk * 16);
    }
  }
  auto dma = [&](int t, int buf, int p0, int np) {   // pieces p0 .. p0 + np - 1 of K-tile t into buffer buf
    char* base = smem + buf * PP_BUF + img_off;
#pragma unroll
    for (int p = p0; p < p0 + np; ++p) pp_dma(rs, base + prow[p] * 128, vo[p], (uint32_t)t * 128);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 wf[4][2], xa[2][2], xb[2][2];
  if constexpr (PROBE == 2) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) wf[i][kk] = pp_frag(smem, i * 16 + fr, kk * 4 + fc);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) xa[j][kk] = xb[j][kk] = pp_frag(smem, j * 16 + fr, kk * 4 + fc);
  }

  auto rd_w = [&](const char* img, int i0) {   // W blocks i0 .. i0 + 3 of this group, both K halves
    if constexpr (PROBE == 2) {   // diagnostic build: no LDS reads, opaque operands
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) asm volatile("" : "+v"(wf[i][kk]));
      return;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) wf[i][kk] = pp_frag(img, g * 128 + (i0 + i) * 16 + fr, kk * 4 + fc);
  };
  auto rd_x = [&](bf16x8 (&xf)[2][2], const char* img, int j0) {
    if constexpr (PROBE == 2) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) asm volatile("" : "+v"(xf[j][kk]));
      return;
    }
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) xf[j][kk] = pp_frag(img, wi * 64 + (j0 + j) * 16 + fr, kk * 4 + fc);
  };
  auto mma = [&](const bf16x8 (&xf)[2][2], int i0, int j0) {   // one quadrant: 4 x 2 blocks x K 64
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i0 + i][j0 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i][kk], xf[j][kk], acc[i0 + i][j0 + j],
                                                                       0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // ---- prologue: K-tiles 0 and 1 whole (clamped re-read when kt == 1), wait for tile 0
  const int t1 = kt > 1 ? 1 : 0;
  dma(0, 0, 0, 8);
  dma(t1, 1, 0, 8);
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  pp_bar();
  if (g == 1) pp_bar();   // the stagger: group 1 runs one barrier interval behind group 0

  // DMA schedule of K-tile u >= 2 (into buffer u & 1, free once group 1 has done P2 of tile u - 2):
  // pieces 0,1 in P3(u-2), 2,3 in P0(u-1), 4,5 in P1(u-1), 6,7 in P2(u-1).  Waits (counted, the
  // youngest pieces stay in flight): pieces 0-3 in P3(u-1) before its own issue (vmcnt(4): 4-7 of u
  // in flight), pieces 4-7 in P0(u) (vmcnt(2): 0,1 of u + 1 in flight).  Each wait is followed by
  // the barrier that ends the read segment, so the partner group reads the rows one interval later.
#pragma unroll 1
  for (int t = 0; t < kt; ++t) {
    const char* img_w = smem + (t & 1) * PP_BUF;
    const char* img_x = img_w + PP_IMG;
    const bool nxt = t >= 1 && t + 1 < kt;   // tile t + 1's pieces 2..7 are issued in this tile
    // P0
    if (t + 1 < kt)
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    rd_w(img_w, 0);
    rd_x(xa, img_x, 0);
    if (PROBE == 0 && nxt) dma(t + 1, (t + 1) & 1, 2, 2);
    pp_bar_lgkm();
    mma(xa, 0, 0);
    pp_bar();
    // P1
    rd_x(xb, img_x, 2);
    if (PROBE == 0 && nxt) dma(t + 1, (t + 1) & 1, 4, 2);
    pp_bar_lgkm();
    mma(xb, 0, 2);
    pp_bar();
    // P2
    rd_w(img_w, 4);
    if (PROBE == 0 && nxt) dma(t + 1, (t + 1) & 1, 6, 2);
    pp_bar_lgkm();
    mma(xb, 4, 2);
    pp_bar();
    // P3: pieces 0-3 of tile t + 1 landed; pieces 0,1 of tile t + 2 go into this tile's buffer,
    // whose last reader (group 1's P2 of tile t) is one interval behind
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    if (PROBE == 0 && t + 2 < kt) dma(t + 2, t & 1, 0, 2);
    pp_bar_lgkm();
    mma(xa, 4, 0);
    pp_bar();
  }

  // ---- epilogue: lane (fr, fc) of block (i, j) holds C[m0 + wi*64 + j*16 + fr][n0 + g*128 + i*16 + 4fc .. +3]
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int m = m0 + wi * 64 + j * 16 + fr;
    if (m < M) {
      if constexpr (EPI == PP_SILU) {
#pragma unroll
        for (int i = 0; i < 8; i += 2) {
          const int n = ((n0 + g * 128 + i * 16) >> 1) + 4 * fc;
          bf16x4 v;
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = (bf16)(pp_silu(acc[i][j][r]) * acc[i + 1][j][r]);
          *reinterpret_cast<bf16x4*>(out + (int64_t)m * ldo + n) = v;
        }
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int n = n0 + g * 128 + i * 16 + 4 * fc;
          f32x4 a = acc[i][j];
          if constexpr (BIAS) {
            const bf16x4 bv = *reinterpret_cast<const bf16x4*>(bias + n);
#pragma unroll
            for (int r = 0; r < 4; ++r) a[r] += (float)bv[r];
          }
          if constexpr (EPI == PP_RES) {
            const bf16x4 rv = *reinterpret_cast<const bf16x4*>(res + (int64_t)m * ldr + n);
#pragma unroll
            for (int r = 0; r < 4; ++r) a[r] += (float)rv[r];
          }
          bf16x4 v;
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = (bf16)a[r];
          *reinterpret_cast<bf16x4*>(out + (int64_t)m * ldo + n) = v;
        }
      }
    }
  }
  if (g == 0) pp_bar();   // pairs with group 1's last barrier (barrier counts match per wave)
}

// ---- K32 body: BK = 32, NB LDS stages of {W image 256 x 64 B, X image 256 x 64 B} (32 KiB each,
// NB = 5: 160 KiB), ONE phase per K-tile: read segment = the tile's 8 W + 4 X fragments, 4 DMA
// pieces of tile t + NB - 1 and the wait for tile t + 1 (the pieces of 2 .. NB - 2 tiles ahead
// stay in flight: vmcnt(4 (NB - 2))); compute segment = 32 MFMAs (512 matrix-pipe cycles).  The
// DMA of a tile is issued 2 (NB - 2) barrier intervals before it must have landed (LDS-DMA issue
// -> landed is ~1.1 us under load, MI355X_MICROARCH.md ldsdma-fill; the BK = 64 two-buffer body
// above gives it 2-6 intervals and measured ~25 % slower than the same body without DMA).
// 64-byte image rows: 16 B chunk c of row r sits at slot c ^ (-(r >> 2) & 3), which keeps every
// 16-lane group of a ds_read_b128 fragment read (16 rows x one chunk column per 4 lanes) on 16
// distinct 16-byte bank slots.
__device__ __forceinline__ int pp_swz32(int row, int chunk) { return chunk ^ ((-(row >> 2)) & 3); }

__device__ __forceinline__ bf16x8 pp_frag32(const char* img, int row, int chunk) {
  return *reinterpret_cast<const bf16x8*>(img + row * 64 + pp_swz32(row, chunk) * 16);
}

template <int EPI, bool BIAS, int NB, int PROBE>
__global__ __launch_bounds__(PP_NT, 1) void gemm_pp32_kernel(const bf16* __restrict__ X, int64_t ldx,
                                                             const bf16* __restrict__ W, int64_t ldw,
                                                             const bf16* __restrict__ bias,
                                                             const bf16* __restrict__ res, int64_t ldr,
                                                             bf16* __restrict__ out, int64_t ldo, int M, int N, int kt,
                                                             int gm) {
  constexpr int IMG = 256 * 64, STG = 2 * IMG;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = wave >> 2, wi = wave & 3;
  const int fr = lane & 15, fc = lane >> 4;

  const int tiles_m = (M + 255) >> 8, T = tiles_m * (N >> 8);
  const int b = blockIdx.x, xcd = b & 7, q8 = T >> 3, r8 = T & 7;
  const int id = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  int tm, tn;
  pp_tile(id, tiles_m, N >> 8, gm, tm, tn);
  const int m0 = tm << 8, n0 = tn << 8;

  // staging: group 0 -> W image, group 1 -> X image; piece p of wave wi = image rows
  // (wi * 4 + p) * 16 .. + 16, lane L: row L >> 2, 16-byte slot L & 3
  const auto rs = g == 0 ? __builtin_amdgcn_make_buffer_rsrc((void*)(W + (int64_t)n0 * ldw), (short)0, 0x7fffffff,
                                                            0x00020000)
                         : __builtin_amdgcn_make_buffer_rsrc((void*)(X + (int64_t)m0 * ldx), (short)0, 0x7fffffff,
                                                            0x00020000);
  const int img_off = g == 0 ? 0 : IMG;
  uint32_t vo[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int row = (wi * 4 + p) * 16 + (lane >> 2);
    const int chunk = pp_swz32(row, lane & 3);
    if (g == 0) {
      vo[p] = (uint32_t)(row * ldw * 2 + chunk * 16);
    } else {
      const int rr = m0 + row < M ? row : M - 1 - m0;
      vo[p] = (uint32_t)(rr * ldx * 2 + chunk * 16);
    }
  }
  auto dma = [&](int t) {   // the 4 pieces of K-tile t (clamped re-read past the end: never read)
    const int tc = t < kt ? t : kt - 1;
    char* base = smem + (t % NB) * STG + img_off + wi * 4 * 1024;
#pragma unroll
    for (int p = 0; p < 4; ++p) pp_dma(rs, base + p * 1024, vo[p], (uint32_t)tc * 64);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 wf[8], xf[4];

  // prologue: tiles 0 .. NB - 2 (every thread always issues 4 pieces per tile, clamped past the
  // end, so the counted waits are exact), wait for tile 0
#pragma unroll
  for (int t = 0; t < NB - 1; ++t) dma(t);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * (NB - 2)) : "memory");
  pp_bar();
  if (g == 1) pp_bar();   // the stagger

#pragma unroll 1
  for (int t = 0; t < kt; ++t) {
    const char* img_w = smem + (t % NB) * STG;
    const char* img_x = img_w + IMG;
    // ---- read segment: this tile's fragments, DMA of tile t + NB - 1 into the stage tile t - 1
    // left (its last reader, group 1, finished one interval ago), wait for tile t + 1
    if constexpr (PROBE == 2) {
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("" : "+v"(wf[i]));
#pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" : "+v"(xf[j]));
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) wf[i] = pp_frag32(img_w, g * 128 + i * 16 + fr, fc);
#pragma unroll
      for (int j = 0; j < 4; ++j) xf[j] = pp_frag32(img_x, wi * 64 + j * 16 + fr, fc);
    }
    if constexpr (PROBE == 0) {
      dma(t + NB - 1);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * (NB - 2)) : "memory");
    }
    pp_bar_lgkm();
    // ---- compute segment
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i], xf[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    pp_bar();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // clamped tail pieces retire before the waves exit

#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int m = m0 + wi * 64 + j * 16 + fr;
    if (m < M) {
      if constexpr (EPI == PP_SILU) {
#pragma unroll
        for (int i = 0; i < 8; i += 2) {
          const int n = ((n0 + g * 128 + i * 16) >> 1) + 4 * fc;
          bf16x4 v;
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = (bf16)(pp_silu(acc[i][j][r]) * acc[i + 1][j][r]);
          *reinterpret_cast<bf16x4*>(out + (int64_t)m * ldo + n) = v;
        }
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int n = n0 + g * 128 + i * 16 + 4 * fc;
          f32x4 a = acc[i][j];
          if constexpr (BIAS) {
            const bf16x4 bv = *reinterpret_cast<const bf16x4*>(bias + n);
#pragma unroll
            for (int r = 0; r < 4; ++r) a[r] += (float)bv[r];
          }
          if constexpr (EPI == PP_RES) {
            const bf16x4 rv = *reinterpret_cast<const bf16x4*>(res + (int64_t)m * ldr + n);
#pragma unroll
            for (int r = 0; r < 4; ++r) a[r] += (float)rv[r];
          }
          bf16x4 v;
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = (bf16)a[r];
          *reinterpret_cast<bf16x4*>(out + (int64_t)m * ldo + n) = v;
        }
      }
    }
  }
  if (g == 0) pp_bar();
}

// tile-group height (OME_PP_GM, default 4; 0 = m fastest over all of M)
static int pp_gm() {
  static const int gm = getenv("OME_PP_GM") ? atoi(getenv("OME_PP_GM")) : 4;
  return gm;
}

template <int EPI, bool BIAS, int NB, int PROBE = 0>
int launch_pp32(const bf16* X, int64_t ldx, const bf16* W, int64_t ldw, const bf16* bias, const bf16* res,
                int64_t ldr, bf16* out, int64_t ldo, int M, int N, int K, hipStream_t stream) {
  constexpr int LDS = NB * 2 * 256 * 64;
  static_assert(LDS <= 160 * 1024, "LDS");
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)gemm_pp32_kernel<EPI, BIAS, NB, PROBE>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  const int T = ((M + 255) / 256) * (N / 256);
  gemm_pp32_kernel<EPI, BIAS, NB, PROBE><<<T, PP_NT, LDS, stream>>>(X, ldx, W, ldw, bias, res, ldr, out, ldo, M, N,
                                                                     K / 32, pp_gm());
  return (int)hipGetLastError();
}

template <int EPI, bool BIAS, int PROBE = 0>
int launch_pp(const bf16* X, int64_t ldx, const bf16* W, int64_t ldw, const bf16* bias, const bf16* res,
              int64_t ldr, bf16* out, int64_t ldo, int M, int N, int K, hipStream_t stream) {
  constexpr int LDS = 2 * PP_BUF;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)gemm_pp_kernel<EPI, BIAS, PROBE>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       LDS);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  const int T = ((M + 255) / 256) * (N / 256);
  gemm_pp_kernel<EPI, BIAS, PROBE><<<T, PP_NT, LDS, stream>>>(X, ldx, W, ldw, bias, res, ldr, out, ldo, M, N, K / 64, pp_gm());
  return (int)hipGetLastError();
}

}  // namespace

// X [M][K] (row stride ldx), W [N][K] (row stride ldw), out [M][N] (or [M][N/2] for epi = 2).
// N % 256 == 0, K % 64 == 0, 16-byte aligned operand rows.  epi 0: bf16 (+ optional bias[N]);
// epi 1: + res [M][N] (row stride ldr, may alias out); epi 2: SiLU(gate) * up with gate/up rows
// interleaved in 16-row blocks (ops.interleave_gate_up).
OME_API int ome_gemm_pp(const void* X, int64_t ldx, const void* W, int64_t ldw, const void* bias, const void* res,
                        int64_t ldr, void* out, int64_t ldo, int M, int N, int K, int epi, hipStream_t stream) {
  if (M <= 0) return 0;
  if (N % 256 || K % 64 || K <= 0 || N <= 0) return -2;
  if (ldx % 8 || ldw % 8 || ((uintptr_t)X | (uintptr_t)W) % 16 || ldo % 4 || (uintptr_t)out % 8) return -3;
  if ((int64_t)M * ldx * 2 >= 0x7fffffffLL || 256LL * ldw * 2 >= 0x7fffffffLL) return -3;   // 32-bit DMA offsets
  if (epi == PP_RES && (!res || ldr % 4 || (uintptr_t)res % 8)) return -3;
  if (epi == PP_SILU && bias) return -4;
  if (epi != PP_BF16 && epi != PP_RES && epi != PP_SILU) return -4;
  const bf16 *x = (const bf16*)X, *w = (const bf16*)W, *b = (const bf16*)bias, *r = (const bf16*)res;
  bf16* o = (bf16*)out;
  static const int probe = getenv("OME_PP_PROBE") ? atoi(getenv("OME_PP_PROBE")) : 0;   // diagnostic builds
  static const int body = getenv("OME_PP_BODY") ? atoi(getenv("OME_PP_BODY")) : 5;     // 64 | 4 | 5
  if (body != 64) {
#define PP32(NBV)                                                                                          \
  if (probe == 1 && epi == PP_BF16 && !b)                                                                  \
    return launch_pp32<PP_BF16, false, NBV, 1>(x, ldx, w, ldw, b, r, ldr, o, ldo, M, N, K, stream);        \
  if (probe == 2 && epi == PP_BF16 && !b)                                                                  \
    return launch_pp32<PP_BF16, false, NBV, 2>(x, ldx, w, ldw, b, r, ldr, o, ldo, M, N, K, stream);        \
  if (epi == PP_BF16)                                                                                      \
    return b ? launch_pp32<PP_BF16, true, NBV>(x, ldx, w, ldw, b, r, ldr, o, ldo, M, N, K, stream)         \
             : launch_pp32<PP_BF16, false, NBV>(x, ldx, w, ldw, b, r, ldr, o, ldo, M, N, K, stream);       \
  if (epi == PP_RES)                                                                                       \
    return b ? launch_pp32<PP_RES, true, NBV>(x, ldx, w, ldw, b, r, ldr, o, ldo, M, N, K, stream)          \
             : launch_pp32<PP_RES, false, NBV>(x, ldx, w, ldw, b, r, ldr, o, ldo, M, N, K, stream);        \
  return launch_pp32<PP_SILU, false, NBV>(x, ldx, w, ldw, b, r, ldr, o, ldo, M, N, K, stream);
    if (body == 4) { PP32(4) }
    PP32(5)
#undef PP32
  }
  if (epi == PP_BF16 && !b && probe == 1)
    return launch_pp<PP_BF16, false, 1>(x, ldx, w, ldw, b, r, ldr, o, ldo, M, N, K, stream);
  if (epi == PP_BF16 && !b && probe == 2)
    return launch_pp<PP_BF16, false, 2>(x, ldx, w, ldw, b, r, ldr, o, ldo, M, N, K, stream);
  if (epi == PP_BF16)
    return b ? launch_pp<PP_BF16, true>(x, ldx, w, ldw, b, r, ldr, o, ldo, M, N, K, stream)
             : launch_pp<PP_BF16, false>(x, ldx, w, ldw, b, r, ldr, o, ldo, M, N, K, stream);
  if (epi == PP_RES)
    return b ? launch_pp<PP_RES, true>(x, ldx, w, ldw, b, r, ldr, o, ldo, M, N, K, stream)
             : launch_pp<PP_RES, false>(x, ldx, w, ldw, b, r, ldr, o, ldo, M, N, K, stream);
  return launch_pp<PP_SILU, false>(x, ldx, w, ldw, b, r, ldr, o, ldo, M, N, K, stream);
}
