// Dense bf16 GEMM on MFMA for the decoder projections, "NT" layout:
//   C[M][N] = A[M][K] · B[N][K]^T        A = activations (K contiguous), B = weight rows (K contiguous)
// i.e. exactly F.linear(x, w).  Written for gfx950 (cdna_hip_programming.md §5):
//
// * 256 x 256 output tile per 512-thread workgroup (8 waves = 2 along N x 4 along M, 128 x 64
//   per wave, v_mfma_f32_16x16x32_bf16), BK = 64, one workgroup per CU (128 KiB of LDS).
// * Operands go global -> LDS with global_load_lds (16 B per lane, no VGPR round trip), double
//   buffered: the next K-tile's DMA is in flight while the current one feeds the MFMAs.
// * LDS images are lane-linear (the DMA writes base + lane * 16) with the XOR swizzle applied to
//   the SOURCE address (rule 21): 16-B chunk c of row r sits at chunk c ^ ((r >> 1) & 7), which
//   makes every 16-lane group of a fragment ds_read_b128 conflict-free.
// * The MFMA "A" operand is the weight tile and "B" the activations, so the accumulator holds
//   C^T: each lane owns 4 consecutive output columns of one row (8-byte stores) and, for the
//   gate/up projection stored interleaved in 16-row blocks (gate 16, up 16, ...), the SiLU(gate)
//   * up epilogue is lane-local (accumulator tiles 2i and 2i + 1).
// * XCD-aware tile order (T1): the workgroups that share a weight panel run back to back on one
//   XCD, so the panel is fetched from HBM once into that XCD's L2.
// * Split-K (grid.z) writes fp32 partial slabs; gemm_reduce_kernel sums them (and applies the
//   epilogue) in a second launch.
#include "common.h"

#include <cstdlib>

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;

namespace {

constexpr int BM = 256, BN = 256, BK = 64, NTHR = 512;
constexpr int TILE_BYTES = 256 * BK * 2;   // one operand tile: 256 rows x 128 B
constexpr int LDS_BYTES = 2 * 2 * TILE_BYTES;

enum { EPI_BF16 = 0, EPI_SILU_MUL = 2, EPI_F32_PARTIAL = 3 };

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

__device__ __forceinline__ f32x4 mfma(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float silu(float x) { return x / (1.f + __expf(-x)); }

// Stage one 256-row x 64-col bf16 tile into lane-linear LDS (8 rows per wave instruction, 4 per
// wave).  Rows past `rows` re-read the last valid row (their results are never stored).
__device__ __forceinline__ void stage_tile(char* lds, const bf16* __restrict__ g, int64_t ld, int row0, int rows,
                                           int k0, int wave, int lane) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = (wave * 4 + j) * 8 + (lane >> 3);
    const int cpos = lane & 7;
    int gr = row0 + r;
    gr = gr < rows ? gr : rows - 1;
    const bf16* src = g + (int64_t)gr * ld + k0 + swz(r, cpos) * 8;
    __builtin_amdgcn_global_load_lds((glb_void_t*)src, (lds_void_t*)(lds + (wave * 4 + j) * 1024), 16, 0, 0);
  }
}

// byte-addressed form (fp8 operands: a 128-byte row = 128 K elements)
__device__ __forceinline__ void stage_tile_b(char* lds, const uint8_t* __restrict__ g, int64_t ld, int row0, int rows,
                                             int64_t k0, int wave, int lane) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = (wave * 4 + j) * 8 + (lane >> 3);
    int gr = row0 + r;
    gr = gr < rows ? gr : rows - 1;
    const uint8_t* src = g + (int64_t)gr * ld + k0 + swz(r, lane & 7) * 16;
    __builtin_amdgcn_global_load_lds((glb_void_t*)src, (lds_void_t*)(lds + (wave * 4 + j) * 1024), 16, 0, 0);
  }
}

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

// 32 fp8 of row `row` starting at chunk 2c (16-B chunks 2c, 2c + 1): the MX MFMA operand of a lane
__device__ __forceinline__ i32x8 frag32(const char* lds, int row, int c) {
  const i32x4 lo = *reinterpret_cast<const i32x4*>(lds + row * 128 + swz(row, 2 * c) * 16);
  const i32x4 hi = *reinterpret_cast<const i32x4*>(lds + row * 128 + swz(row, 2 * c + 1) * 16);
  return i32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

__device__ __forceinline__ bf16x8 frag(const char* lds, int row, int chunk) {
  return *reinterpret_cast<const bf16x8*>(lds + row * 128 + swz(row, chunk) * 16);
}

// Bijective XCD remap (cdna_hip_programming.md §5 template): blocks b, b + 8, ... share an XCD;
// give each XCD a contiguous range of tile ids.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

template <int EPI, int VAR>
__global__ __launch_bounds__(NTHR, 1) void gemm_nt_kernel(const bf16* __restrict__ A, int64_t lda,
                                                          const bf16* __restrict__ B, int64_t ldb,
                                                          void* __restrict__ C, int64_t ldc, int M, int N,
                                                          int k_per_split, float* __restrict__ ws) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int tiles_m = (M + BM - 1) / BM, tiles_n = N / BN;
  const int L = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tn = L / tiles_m, tm = L - tn * tiles_m;  // the tiles_m tiles of one weight panel are adjacent
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = blockIdx.z * k_per_split;
  const int nt = k_per_split / BK;
  const int wn = wave & 1, wm = wave >> 1;  // wave tile: W rows [wn*128, +128) x activation rows [wm*64, +64)

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // buffer b: [W tile | A tile]
  auto buf_w = [&](int b) { return smem + b * 2 * TILE_BYTES; };
  auto buf_a = [&](int b) { return smem + b * 2 * TILE_BYTES + TILE_BYTES; };

  stage_tile(buf_w(0), B, ldb, n0, N, kbeg, wave, lane);
  stage_tile(buf_a(0), A, lda, m0, M, kbeg, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int fr = lane & 15, fc = lane >> 4;
  if constexpr (VAR == 1) {
    for (int t = 0; t < nt; ++t) {
      const int cur = t & 1;
      if (t + 1 < nt) {
        stage_tile(buf_w(cur ^ 1), B, ldb, n0, N, kbeg + (t + 1) * BK, wave, lane);
        stage_tile(buf_a(cur ^ 1), A, lda, m0, M, kbeg + (t + 1) * BK, wave, lane);
      }
      const char* lw = buf_w(cur);
      const char* la = buf_a(cur);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 xa[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) xa[j] = frag(la, wm * 64 + j * 16 + fr, kk * 4 + fc);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const bf16x8 wf = frag(lw, wn * 128 + i * 16 + fr, kk * 4 + fc);
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = mfma(wf, xa[j], acc[i][j]);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  } else if constexpr (VAR == 3) {
    // VAR 3: four 16-MFMA phases per K-tile ((k-half, weight-half) pairs); each phase's MFMAs
    // run while the next phase's fragments are read from LDS (4 + 4 fragment registers live).
    // The barrier that publishes tile t+1 sits before the last phase, whose MFMAs then cover the
    // first reads of tile t+1.
    bf16x8 x0[4], x1[4], wa[4], wb[4];
    auto rdx = [&](bf16x8 (&fx)[4], const char* la, int kk) {
#pragma unroll
      for (int j = 0; j < 4; ++j) fx[j] = frag(la, wm * 64 + j * 16 + fr, kk * 4 + fc);
    };
    auto rdw = [&](bf16x8 (&fw)[4], const char* lw, int kk, int ih) {
#pragma unroll
      for (int i = 0; i < 4; ++i) fw[i] = frag(lw, wn * 128 + (ih * 4 + i) * 16 + fr, kk * 4 + fc);
    };
    auto mm = [&](const bf16x8 (&fx)[4], const bf16x8 (&fw)[4], int ih) {
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[ih * 4 + i][j] = mfma(fw[i], fx[j], acc[ih * 4 + i][j]);
      __builtin_amdgcn_s_setprio(0);
    };
    rdx(x0, buf_a(0), 0);
    rdw(wa, buf_w(0), 0, 0);
    for (int t = 0; t < nt; ++t) {
      const int cur = t & 1;
      if (t + 1 < nt) {
        stage_tile(buf_w(cur ^ 1), B, ldb, n0, N, kbeg + (t + 1) * BK, wave, lane);
        stage_tile(buf_a(cur ^ 1), A, lda, m0, M, kbeg + (t + 1) * BK, wave, lane);
      }
      const char* lw = buf_w(cur);
      const char* la = buf_a(cur);
      rdw(wb, lw, 0, 1);
      mm(x0, wa, 0);
      rdx(x1, la, 1);
      rdw(wa, lw, 1, 0);
      mm(x0, wb, 1);
      rdw(wb, lw, 1, 1);
      mm(x1, wa, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (t + 1 < nt) {
        rdx(x0, buf_a(cur ^ 1), 0);
        rdw(wa, buf_w(cur ^ 1), 0, 0);
      }
      mm(x1, wb, 1);
    }
  } else {
    // VAR 2: the fragments of the next k-half are read from LDS while the MFMAs of the current
    // one run (two register sets P / Q); the first half of tile t+1 is read right after the
    // barrier that publishes it, behind the MFMAs of tile t's second half.
    bf16x8 px[4], pw[8], qx[4], qw[8];
    auto rd = [&](bf16x8 (&fx)[4], bf16x8 (&fw)[8], const char* la, const char* lw, int kk) {
#pragma unroll
      for (int j = 0; j < 4; ++j) fx[j] = frag(la, wm * 64 + j * 16 + fr, kk * 4 + fc);
#pragma unroll
      for (int i = 0; i < 8; ++i) fw[i] = frag(lw, wn * 128 + i * 16 + fr, kk * 4 + fc);
    };
    auto mm = [&](const bf16x8 (&fx)[4], const bf16x8 (&fw)[8]) {
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma(fw[i], fx[j], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
    };
    rd(px, pw, buf_a(0), buf_w(0), 0);
    for (int t = 0; t < nt; ++t) {
      const int cur = t & 1;
      if (t + 1 < nt) {
        stage_tile(buf_w(cur ^ 1), B, ldb, n0, N, kbeg + (t + 1) * BK, wave, lane);
        stage_tile(buf_a(cur ^ 1), A, lda, m0, M, kbeg + (t + 1) * BK, wave, lane);
      }
      rd(qx, qw, buf_a(cur), buf_w(cur), 1);
      mm(px, pw);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (t + 1 < nt) rd(px, pw, buf_a(cur ^ 1), buf_w(cur ^ 1), 0);
      mm(qx, qw);
    }
  }

  // ---- epilogue: lane (fr, fc) of tile (i, j) holds C[m = m0+wm*64+j*16+fr][n = n0+wn*128+i*16+4fc .. +3]
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int m = m0 + wm * 64 + j * 16 + fr;
    if (m >= M) continue;
    if constexpr (EPI == EPI_BF16) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int n = n0 + wn * 128 + i * 16 + 4 * fc;
        bf16x4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = (bf16)acc[i][j][r];
        *reinterpret_cast<bf16x4*>((bf16*)C + (int64_t)m * ldc + n) = v;
      }
    } else if constexpr (EPI == EPI_SILU_MUL) {
      // weight rows interleaved in 16-row blocks: tile 2i = gate, 2i + 1 = up of the same outputs
#pragma unroll
      for (int i = 0; i < 8; i += 2) {
        const int n = ((n0 + wn * 128 + i * 16) >> 1) + 4 * fc;
        bf16x4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = (bf16)(silu(acc[i][j][r]) * acc[i + 1][j][r]);
        *reinterpret_cast<bf16x4*>((bf16*)C + (int64_t)m * ldc + n) = v;
      }
    } else {  // fp32 partial slab of split blockIdx.z: ws[z][M][N]
      float* slab = ws + (int64_t)blockIdx.z * M * N;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int n = n0 + wn * 128 + i * 16 + 4 * fc;
        *reinterpret_cast<f32x4*>(slab + (int64_t)m * N + n) = acc[i][j];
      }
    }
  }
}

// out = epilogue(sum over `splits` fp32 slabs ws[z][M][N]); 4 columns per thread.
template <int EPI>
__global__ __launch_bounds__(256) void gemm_reduce_kernel(const float* __restrict__ ws, int splits, int M, int N,
                                                          bf16* __restrict__ C, int64_t ldc) {
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;   // index of a 4-column group
  const int64_t groups = (int64_t)M * (N / 4);
  if (q >= groups) return;
  const int64_t m = q / (N / 4);
  const int n = (int)(q - m * (N / 4)) * 4;
  f32x4 s = *reinterpret_cast<const f32x4*>(ws + m * N + n);
  for (int z = 1; z < splits; ++z) s += *reinterpret_cast<const f32x4*>(ws + (int64_t)z * M * N + m * N + n);
  if constexpr (EPI == EPI_BF16) {
    bf16x4 v;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = (bf16)s[r];
    *reinterpret_cast<bf16x4*>(C + m * ldc + n) = v;
  } else {
    // SILU_MUL: columns [32b, 32b+16) gate, [32b+16, 32b+32) up -> output 16b + (n mod 16)
    if ((n & 31) >= 16) return;
    const f32x4 u = *reinterpret_cast<const f32x4*>(ws + m * N + n + 16);
    f32x4 uu = u;
    for (int z = 1; z < splits; ++z) uu += *reinterpret_cast<const f32x4*>(ws + (int64_t)z * M * N + m * N + n + 16);
    bf16x4 v;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = (bf16)(silu(s[r]) * uu[r]);
    *reinterpret_cast<bf16x4*>(C + m * ldc + (n >> 5) * 16 + (n & 15)) = v;
  }
}

template <int EPI, int VAR>
int launch_gemm_v(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int M, int N,
                  int K, int splits, float* ws, hipStream_t stream) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)gemm_nt_kernel<EPI, VAR>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    if (e != hipSuccess) return (int)e;
    attr_set = true;
  }
  const int tiles = ((M + BM - 1) / BM) * (N / BN);
  gemm_nt_kernel<EPI, VAR><<<dim3(tiles, 1, splits), NTHR, LDS_BYTES, stream>>>(
      (const bf16*)A, lda, (const bf16*)B, ldb, C, ldc, M, N, K / splits, ws);
  return (int)hipGetLastError();
}

int g_variant = -1;  // pipeline variant (1 plain 2-phase, 2 / 3 fragment-prefetch), OME_GEMM_VAR

int gemm_variant() {
  if (g_variant < 0) {
    const char* e = getenv("OME_GEMM_VAR");
    g_variant = e ? atoi(e) : 3;
  }
  return g_variant;
}

template <int EPI>
int launch_gemm(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int M, int N, int K,
                int splits, float* ws, hipStream_t stream) {
  const int v = gemm_variant();
  if (v == 1) return launch_gemm_v<EPI, 1>(A, lda, B, ldb, C, ldc, M, N, K, splits, ws, stream);
  if (v == 2) return launch_gemm_v<EPI, 2>(A, lda, B, ldb, C, ldc, M, N, K, splits, ws, stream);
  return launch_gemm_v<EPI, 3>(A, lda, B, ldb, C, ldc, M, N, K, splits, ws, stream);
}


// ------------------------------------------------------------------------------------------
// FP8 (OCP e4m3) W8A8 on the same 256 x 256 tile: one K-tile = 128 K elements = 128-byte rows,
// so the DMA staging and LDS images are byte-identical to the bf16 kernel, and each tile is ONE
// v_mfma_scale_f32_16x16x128_f8f6f4 per (16 x 16) output block at unit MX scales -- twice the
// bf16 MFMA rate.  Every lane feeds 32 contiguous bytes of its row at K offset 32 * (lane >> 4)
// to both operands: the K order inside the block is the same permutation for A and B, so the
// sum is exact.  Scales: ROW = per-token sa[M] x per-channel sw[N] in the epilogue; BLOCK =
// DeepSeek 1x128 activation groups sa[M][K/128] and 128x128 weight blocks sw[N/128][K/128]
// applied per K-tile to the block's product (fp32 scales are not E8M0, so the MX scale operands
// stay at 1.0 and the scaling is a VALU FMA per accumulator element).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ f32x4 mfma_fp8(i32x8 a, i32x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127, 0, 127);
}

template <bool BLOCK>
__global__ __launch_bounds__(NTHR, 1) void gemm_fp8_nt_kernel(const uint8_t* __restrict__ A, int64_t lda,
                                                              const float* __restrict__ sa,
                                                              const uint8_t* __restrict__ B, int64_t ldb,
                                                              const float* __restrict__ sb, bf16* __restrict__ C,
                                                              int64_t ldc, int M, int N, int K,
                                                              const bf16* __restrict__ bias) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int tiles_m = (M + BM - 1) / BM, tiles_n = N / BN;
  const int L = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tn = L / tiles_m, tm = L - tn * tiles_m;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nt = K / 128, KB = K / 128;
  const int wn = wave & 1, wm = wave >> 1;
  const int fr = lane & 15, fc = lane >> 4;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto buf_w = [&](int b) { return smem + b * 2 * TILE_BYTES; };
  auto buf_a = [&](int b) { return smem + b * 2 * TILE_BYTES + TILE_BYTES; };
  int mrow[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int m = m0 + wm * 64 + j * 16 + fr;
    mrow[j] = m < M ? m : M - 1;
  }
  const int nblk = (n0 + wn * 128) >> 7;   // the wave's 128 output columns are one weight block

  stage_tile_b(buf_w(0), B, ldb, n0, N, 0, wave, lane);
  stage_tile_b(buf_a(0), A, lda, m0, M, 0, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1;
    if (t + 1 < nt) {
      stage_tile_b(buf_w(cur ^ 1), B, ldb, n0, N, (int64_t)(t + 1) * 128, wave, lane);
      stage_tile_b(buf_a(cur ^ 1), A, lda, m0, M, (int64_t)(t + 1) * 128, wave, lane);
    }
    const char* lw = buf_w(cur);
    const char* la = buf_a(cur);
    i32x8 xa[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) xa[j] = frag32(la, wm * 64 + j * 16 + fr, fc);
    if constexpr (BLOCK) {
      const float swv = sb[(int64_t)nblk * KB + t];
      float s[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) s[j] = sa[(int64_t)mrow[j] * KB + t] * swv;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const i32x8 wf = frag32(lw, wn * 128 + i * 16 + fr, fc);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const f32x4 p = mfma_fp8(wf, xa[j], f32x4{0.f, 0.f, 0.f, 0.f});
          acc[i][j] += p * s[j];
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const i32x8 wf = frag32(lw, wn * 128 + i * 16 + fr, fc);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma_fp8(wf, xa[j], acc[i][j]);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int m = m0 + wm * 64 + j * 16 + fr;
    if (m >= M) continue;
    const float srow = BLOCK ? 1.f : sa[m];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int n = n0 + wn * 128 + i * 16 + 4 * fc;
      bf16x4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float y = acc[i][j][r] * (BLOCK ? 1.f : srow * sb[n + r]);
        if (bias) y += (float)bias[n + r];
        v[r] = (bf16)y;
      }
      *reinterpret_cast<bf16x4*>(C + (int64_t)m * ldc + n) = v;
    }
  }
}

template <bool BLOCK>
int launch_fp8(const void* A, int64_t lda, const float* sa, const void* B, int64_t ldb, const float* sb, int M,
               int N, int K, void* out, int64_t ldo, const void* bias, hipStream_t stream) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)gemm_fp8_nt_kernel<BLOCK>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    if (e != hipSuccess) return (int)e;
    attr_set = true;
  }
  const int tiles = ((M + BM - 1) / BM) * (N / BN);
  gemm_fp8_nt_kernel<BLOCK><<<tiles, NTHR, LDS_BYTES, stream>>>((const uint8_t*)A, lda, sa, (const uint8_t*)B, ldb,
                                                                sb, (bf16*)out, ldo, M, N, K, (const bf16*)bias);
  return (int)hipGetLastError();
}

}  // namespace

OME_API int ome_gemm_set_variant(int v) {
  g_variant = v;
  return 0;
}

// epi: 0 = bf16 C, 2 = SiLU(gate) * up with gate/up interleaved in 16-row weight blocks (C has N/2
// columns).  splits > 1: fp32 slabs in `ws` (splits * M * N floats) + a reduce launch.
OME_API int ome_gemm(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int M, int N,
                     int K, int epi, int splits, void* ws, hipStream_t stream) {
  if (M <= 0) return 0;
  if (N % BN || K % BK || splits < 1 || (K / splits) % BK || K % splits) return -2;
  if ((lda | ldb) % 8 || ((uintptr_t)A | (uintptr_t)B) % 16) return -3;
  if (epi != EPI_BF16 && epi != EPI_SILU_MUL) return -4;
  if (splits == 1) {
    return epi == EPI_BF16 ? launch_gemm<EPI_BF16>(A, lda, B, ldb, C, ldc, M, N, K, 1, nullptr, stream)
                           : launch_gemm<EPI_SILU_MUL>(A, lda, B, ldb, C, ldc, M, N, K, 1, nullptr, stream);
  }
  if (ws == nullptr) return -5;
  int rc = launch_gemm<EPI_F32_PARTIAL>(A, lda, B, ldb, C, ldc, M, N, K, splits, (float*)ws, stream);
  if (rc) return rc;
  const int64_t groups = (int64_t)M * (N / 4);
  const int blocks = (int)((groups + 255) / 256);
  if (epi == EPI_BF16)
    gemm_reduce_kernel<EPI_BF16><<<blocks, 256, 0, stream>>>((const float*)ws, splits, M, N, (bf16*)C, ldc);
  else
    gemm_reduce_kernel<EPI_SILU_MUL><<<blocks, 256, 0, stream>>>((const float*)ws, splits, M, N, (bf16*)C, ldc);
  return (int)hipGetLastError();
}

// FP8 W8A8 on the 256 x 256 MX tile: A [M][K] e4m3 (lda bytes), B [N][K] e4m3; block_n = 0: sa [M],
// sb [N]; block_n = 128: sa [M][K/128], sb [N/128][K/128].  N % 256 == 0, K % 128 == 0.
OME_API int ome_fp8_gemm_mx(const void* A, int64_t lda, const float* sa, const void* B, int64_t ldb, const float* sb,
                            int M, int N, int K, int block_n, void* out, int64_t ldo, const void* bias,
                            hipStream_t stream) {
  if (M <= 0) return 0;
  if (N % BN || K % 128 || (lda | ldb) % 16 || ((uintptr_t)A | (uintptr_t)B) % 16) return -2;
  if (block_n && block_n != 128) return -2;
  return block_n ? launch_fp8<true>(A, lda, sa, B, ldb, sb, M, N, K, out, ldo, bias, stream)
                 : launch_fp8<false>(A, lda, sa, B, ldb, sb, M, N, K, out, ldo, bias, stream);
}
