// FP8 (OCP e4m3fn) W8A8 linear layers for gfx950: dynamic activation quantisation and an MFMA
// GEMM with either per-channel x per-token scales or DeepSeek-style block scales
// (weights 128x128 blocks, activations 1x128 groups).
//
// Reference behaviour: SURVEY.md §2.9 K8 — the runtimes OME deploys serve `quantization: fp8`
// checkpoints (reference `config/runtimes/srt/deepseek-rdma-pd-rt.yaml:21`, BaseModel
// `quantization: fp8 / fbgemm_fp8` in `pkg/apis/ome/v1beta1/model.go:262-268`).
//
// Design (CDNA4):
//  * both operands are K-contiguous ([M,K] activations, [N,K] weights), staged through LDS in
//    64x128-byte tiles (one 128-wide K block per step = one scale block);
//  * `v_mfma_f32_16x16x32_fp8_fp8` (8 fp8 per lane per operand); each lane reads 32 contiguous
//    bytes of its row (two ds_read_b128) and feeds them as the four K=32 sub-steps of the block —
//    the K order inside a block is permuted identically for A and B, so the sum is exact;
//  * block mode: the four MFMAs of a K block accumulate into a zeroed temporary which is scaled by
//    sa[row, kb] * sb[n/128, kb] and added to the fp32 accumulator (fp32 scales are not E8M0, so
//    the MX-scaled MFMA cannot carry them);
//  * the next K block's global loads are issued before the current block's MFMAs (register
//    double buffering), 4 waves x (32x32) per 64x64 tile, XCD-aware tile order.
#include "common.h"

typedef long fp8x8;  // 8 x e4m3 in one 64-bit operand
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

static constexpr float kFp8Max = 448.f;

__device__ __forceinline__ uint32_t pack4_fp8(float a, float b, float c, float d) {
  a = fminf(fmaxf(a, -kFp8Max), kFp8Max);
  b = fminf(fmaxf(b, -kFp8Max), kFp8Max);
  c = fminf(fmaxf(c, -kFp8Max), kFp8Max);
  d = fminf(fmaxf(d, -kFp8Max), kFp8Max);
  int v = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  v = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, v, true);
  return (uint32_t)v;
}

// ------------------------------------------------------------------------------------------
// dynamic activation quantisation: x [M, K] bf16 -> q [M, K] e4m3, scale [M, KB] f32
// GROUP = 0: one scale per row (KB = 1); GROUP = 128: one per 128-element group.
// ------------------------------------------------------------------------------------------
template <int GROUP>
__global__ __launch_bounds__(256) void fp8_quant_kernel(const bf16* __restrict__ x, int64_t ldx, int K,
                                                        uint8_t* __restrict__ q, float* __restrict__ scale,
                                                        int KB) {
  __shared__ float red[4];
  const int64_t row = blockIdx.x;
  const bf16* xr = x + row * ldx;
  uint8_t* qr = q + row * (int64_t)K;
  const int nc = K / 8;
  if constexpr (GROUP == 0) {
    float amax = 0.f;
    for (int c = threadIdx.x; c < nc; c += 256) {
      const bf16x8 v = ld8(xr + c * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf((float)v[j]));
    }
    amax = wave_max(amax);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = amax;
    __syncthreads();
    amax = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    const float s = amax > 0.f ? amax / kFp8Max : 1.f;
    const float inv = 1.f / s;
    if (threadIdx.x == 0) scale[row] = s;
    for (int c = threadIdx.x; c < nc; c += 256) {
      const bf16x8 v = ld8(xr + c * 8);
      uint2 o;
      o.x = pack4_fp8((float)v[0] * inv, (float)v[1] * inv, (float)v[2] * inv, (float)v[3] * inv);
      o.y = pack4_fp8((float)v[4] * inv, (float)v[5] * inv, (float)v[6] * inv, (float)v[7] * inv);
      *reinterpret_cast<uint2*>(qr + c * 8) = o;
    }
  } else {
    // 16 consecutive lanes own one 128-element group (16 x 8 elements)
    static_assert(GROUP == 128, "group size 128 only");
    for (int c = threadIdx.x; c < nc; c += 256) {
      const bf16x8 v = ld8(xr + c * 8);
      float amax = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf((float)v[j]));
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o));
      const float s = amax > 0.f ? amax / kFp8Max : 1.f;
      const float inv = 1.f / s;
      if ((c & 15) == 0) scale[row * KB + c / 16] = s;
      uint2 o;
      o.x = pack4_fp8((float)v[0] * inv, (float)v[1] * inv, (float)v[2] * inv, (float)v[3] * inv);
      o.y = pack4_fp8((float)v[4] * inv, (float)v[5] * inv, (float)v[6] * inv, (float)v[7] * inv);
      *reinterpret_cast<uint2*>(qr + c * 8) = o;
    }
  }
}

OME_API int ome_fp8_quant(const void* x, int64_t ldx, int M, int K, void* q, float* scale, int group,
                          hipStream_t stream) {
  if (M <= 0) return 0;
  if (K % 8 || (group && (group != 128 || K % 128))) return -2;
  if (group)
    fp8_quant_kernel<128><<<M, 256, 0, stream>>>((const bf16*)x, ldx, K, (uint8_t*)q, scale, K / 128);
  else
    fp8_quant_kernel<0><<<M, 256, 0, stream>>>((const bf16*)x, ldx, K, (uint8_t*)q, scale, 1);
  OME_CHECK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------------------------------------
// GEMM: out[M, N] = (A[M, K] . B[N, K]^T) with scales, bf16 out (+ optional bf16 bias)
// ------------------------------------------------------------------------------------------
static constexpr int FBM = 64, FBN = 64, FBK = 128, FLD = FBK + 16;  // LDS row: 144 B

template <bool BLOCK>
__global__ __launch_bounds__(256) void fp8_gemm_kernel(const uint8_t* __restrict__ A, int64_t lda,
                                                       const float* __restrict__ sa,
                                                       const uint8_t* __restrict__ B,
                                                       const float* __restrict__ sb, int M, int N, int K,
                                                       bf16* __restrict__ out, int64_t ldo,
                                                       const bf16* __restrict__ bias) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * FBM * FLD];
  uint8_t* sA = smem;
  uint8_t* sB = smem + FBM * FLD;
  const int n_tiles = N / FBN;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  // N tiles fastest within an M row of tiles: consecutive tiles of one XCD share the A rows
  const int m0 = (tile / n_tiles) * FBM, n0 = (tile % n_tiles) * FBN;
  const int KB = K / FBK;

  const int tid = threadIdx.x;
  const int lr = tid >> 2, lc = (tid & 3) * 32;  // staging: row 0..63, byte offset 0/32/64/96
  const bool a_ok = m0 + lr < M;
  const uint8_t* ap = A + (int64_t)(a_ok ? m0 + lr : 0) * lda + lc;
  const uint8_t* bp = B + (int64_t)(n0 + lr) * K + lc;

  const int wave = tid >> 6, lane = tid & 63;
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  const int fr = lane & 15, fk = (lane >> 4) * 32;

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  u32x4 ra0 = {0, 0, 0, 0}, ra1 = {0, 0, 0, 0}, rb0, rb1;
  if (a_ok) {
    ra0 = *reinterpret_cast<const u32x4*>(ap);
    ra1 = *reinterpret_cast<const u32x4*>(ap + 16);
  }
  rb0 = *reinterpret_cast<const u32x4*>(bp);
  rb1 = *reinterpret_cast<const u32x4*>(bp + 16);

  for (int kb = 0; kb < KB; ++kb) {
    __syncthreads();
    *reinterpret_cast<u32x4*>(&sA[lr * FLD + lc]) = ra0;
    *reinterpret_cast<u32x4*>(&sA[lr * FLD + lc + 16]) = ra1;
    *reinterpret_cast<u32x4*>(&sB[lr * FLD + lc]) = rb0;
    *reinterpret_cast<u32x4*>(&sB[lr * FLD + lc + 16]) = rb1;
    __syncthreads();
    if (kb + 1 < KB) {
      const int64_t o = (int64_t)(kb + 1) * FBK;
      if (a_ok) {
        ra0 = *reinterpret_cast<const u32x4*>(ap + o);
        ra1 = *reinterpret_cast<const u32x4*>(ap + o + 16);
      }
      rb0 = *reinterpret_cast<const u32x4*>(bp + o);
      rb1 = *reinterpret_cast<const u32x4*>(bp + o + 16);
    }
    fp8x8 af[2][4], bfr[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const uint8_t* p = &sA[(wm + 16 * i + fr) * FLD + fk];
      const u32x4 x0 = *reinterpret_cast<const u32x4*>(p), x1 = *reinterpret_cast<const u32x4*>(p + 16);
      af[i][0] = (fp8x8)(((uint64_t)x0.y << 32) | x0.x);
      af[i][1] = (fp8x8)(((uint64_t)x0.w << 32) | x0.z);
      af[i][2] = (fp8x8)(((uint64_t)x1.y << 32) | x1.x);
      af[i][3] = (fp8x8)(((uint64_t)x1.w << 32) | x1.z);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const uint8_t* p = &sB[(wn + 16 * j + fr) * FLD + fk];
      const u32x4 x0 = *reinterpret_cast<const u32x4*>(p), x1 = *reinterpret_cast<const u32x4*>(p + 16);
      bfr[j][0] = (fp8x8)(((uint64_t)x0.y << 32) | x0.x);
      bfr[j][1] = (fp8x8)(((uint64_t)x0.w << 32) | x0.z);
      bfr[j][2] = (fp8x8)(((uint64_t)x1.y << 32) | x1.x);
      bfr[j][3] = (fp8x8)(((uint64_t)x1.w << 32) | x1.z);
    }
    if constexpr (BLOCK) {
      const float sbv = sb[(int64_t)(n0 >> 7) * KB + kb];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        float s[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = m0 + wm + 16 * i + 4 * (lane >> 4) + r;
          s[r] = (row < M ? sa[(int64_t)row * KB + kb] : 0.f) * sbv;
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          f32x4 t = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int q = 0; q < 4; ++q) t = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(af[i][q], bfr[j][q], t, 0, 0, 0);
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][j][r] += t[r] * s[r];
        }
      }
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(af[i][q], bfr[j][q], acc[i][j], 0, 0, 0);
    }
  }
  // ---- epilogue: C lane map row = 4*(l>>4)+r, col = l&15 ----
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = n0 + wn + 16 * j + fr;
    const float cs = BLOCK ? 1.f : sb[col];
    const float bv = bias ? (float)bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm + 16 * i + 4 * (lane >> 4) + r;
        if (row < M) {
          const float rs = BLOCK ? 1.f : sa[row];
          out[(int64_t)row * ldo + col] = (bf16)(acc[i][j][r] * rs * cs + bv);
        }
      }
  }
}

// block_n: 0 = per-channel weight scales sb[N] with per-row activation scales sa[M];
//          128 = block scales sb[N/128, K/128], sa[M, K/128].
OME_API int ome_fp8_gemm(const void* A, int64_t lda, const float* sa, const void* B, const float* sb, int M, int N,
                         int K, int block_n, void* out, int64_t ldo, const void* bias, hipStream_t stream) {
  if (M <= 0) return 0;
  if (N % FBN || K % FBK || lda % 16 || (block_n && block_n != 128)) return -2;
  const int tiles = ((M + FBM - 1) / FBM) * (N / FBN);
  if (block_n)
    fp8_gemm_kernel<true><<<tiles, 256, 0, stream>>>((const uint8_t*)A, lda, sa, (const uint8_t*)B, sb, M, N, K,
                                                     (bf16*)out, ldo, (const bf16*)bias);
  else
    fp8_gemm_kernel<false><<<tiles, 256, 0, stream>>>((const uint8_t*)A, lda, sa, (const uint8_t*)B, sb, M, N, K,
                                                      (bf16*)out, ldo, (const bf16*)bias);
  OME_CHECK_LAUNCH();
  return 0;
}
