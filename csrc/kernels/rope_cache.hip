// Fused "QKV split -> RoPE -> paged KV-cache write" (kernels K2 + K3 of SURVEY.md §2.9).
//
// Input is the fused QKV projection output [T, (Hq + 2*Hkv) * D].  Q is rotated into a
// dense [T, Hq, D] buffer for the attention kernels; K is rotated and scattered into the
// paged K cache; V is scattered *transposed* into the paged V cache.
//
// Paged cache layouts (chosen for the MFMA attention kernels, see attention_*.hip):
//   K cache: [num_pages, Hkv, P, D]   — a page's keys are D-contiguous rows, so a lane can load
//                                       the A operand of S^T = K Q^T straight from HBM (16 B).
//   V cache: [num_pages, Hkv, D, P]   — transposed, so the A operand of O^T = V^T P^T is
//                                       P-contiguous (keys) and loads straight from HBM too.
// The cache element type is a template parameter (KVFmt in common.h): bf16, or OCP fp8
// e4m3 / e5m2 (`--kv-cache-dtype fp8*`, K15) stored as fp8(x / scale) with saturation.
// RoPE is the NeoX / HF "rotate_half" form; the cos/sin table [max_pos, rot_dim] (cos in the
// first half, sin in the second) is precomputed on the host with the model's rope scaling
// (llama3 / yarn / linear), so the kernel stays a pure streaming op (Appendix B, trig tables).
#include "common.h"

template <int D, int P, int F>
__global__ __launch_bounds__(256) void rope_qkv_cache_kernel(
    const bf16* __restrict__ qkv, int64_t qkv_stride, const int* __restrict__ positions,
    const float* __restrict__ cos_sin, int rot_dim, bf16* __restrict__ q_out,
    typename KVStore<F>::T* __restrict__ k_cache, typename KVStore<F>::T* __restrict__ v_cache,
    const int* __restrict__ slots, int Hq, int Hkv, int apply_rope, const bf16* __restrict__ q_norm_w,
    const bf16* __restrict__ k_norm_w, float qk_eps, float k_inv_scale, float v_inv_scale, int v_rowmajor) {
  const int t = blockIdx.x;
  const bf16* row = qkv + (int64_t)t * qkv_stride;
  const int pos = positions[t];
  const int slot = slots[t];
  const float* cs = cos_sin + (int64_t)pos * rot_dim;
  const int half = rot_dim >> 1;
  constexpr int DV = D / 8;  // 8-wide vectors per head row

  // ---- Q and K: optional per-head RMSNorm (Qwen3 qk-norm), then rotate ----
  // A head row is LPH = D/8 lanes (8 dims each); a wave processes 64/LPH head rows at once
  // (4 for D=128), so the 40 Q+K rows of a Llama-3 token take 3 wave-iterations, not 10, and
  // every lane of the wave is busy.  All reductions / partner shuffles stay inside a row group.
  constexpr int LPH = D / 8, HPW = 64 / LPH;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int sub = lane / LPH, l = lane % LPH, gbase = sub * LPH;
  const int nheads = Hq + Hkv;
  // grid.y splits a token's heads over several blocks (more waves in flight per CU at decode
  // batch sizes, where one 4-wave block per token leaves the kernel latency-bound)
  for (int h0 = (blockIdx.y * 4 + wave) * HPW; h0 < nheads; h0 += gridDim.y * 4 * HPW) {
    const int h = h0 + sub;
    const bool valid = h < nheads;
    const bool is_q = h < Hq;
    bf16x8 x = {};
    if (valid) x = ld8(row + (int64_t)h * D + l * 8);
    float f[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = (float)x[j];
    const bf16* nw = is_q ? q_norm_w : k_norm_w;
    if (nw != nullptr) {  // wave-uniform: q_norm_w and k_norm_w are both set or both null
      float ss = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += f[j] * f[j];
#pragma unroll
      for (int m = 1; m < LPH; m <<= 1) ss += __shfl_xor(ss, m);
      const float rs = rsqrtf(ss / (float)D + qk_eps);
      if (valid) {
        bf16x8 wv = ld8(nw + l * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = (float)(bf16)(f[j] * rs * (float)wv[j]);
      }
    }
    if (apply_rope) {
      const int d0 = l * 8;
      const int hl = half >> 3;  // lanes between a dim and its rotate_half partner
      const int partner = gbase + ((d0 < half) ? l + hl : l - hl);
      float g[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = __shfl(f[j], (partner >= gbase && partner < gbase + LPH) ? partner : lane);
      if (d0 < rot_dim) {
        const int i0 = (d0 < half) ? d0 : d0 - half;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float c = cs[i0 + j], sn = cs[half + i0 + j];
          f[j] = (d0 < half) ? (f[j] * c - g[j] * sn) : (f[j] * c + g[j] * sn);
        }
      }
    }
    if (valid) {
      if (is_q) {
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (bf16)f[j];
        st8(q_out + ((int64_t)t * Hq + h) * D + l * 8, o);
      } else if (slot >= 0) {
        const int kh = h - Hq;
        const int64_t page = slot / P, off = slot % P;
        if constexpr (F != KV_BF16) {
          // quantise the bf16-rounded key (the value a bf16 cache would have held)
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = (float)(bf16)f[j] * k_inv_scale;
        }
        kv_st8<F>(k_cache + ((page * Hkv + kh) * P + off) * D + l * 8, f);
      }
    }
  }
  // ---- V: transposed scatter into [page][kh][d][off] ----
  // lanes take CONSECUTIVE dims: one wave store then covers 64 dim rows 2*P bytes apart (2 KB,
  // 16 cache lines) instead of 64 rows 8 dims apart (64 lines), so the partial writes of a
  // token's column coalesce per line
  if (slot >= 0) {
    const int64_t page = slot / P, off = slot % P;
    const bf16* vsrc = row + (int64_t)(Hq + Hkv) * D;
    typename KVStore<F>::T* vbase = v_cache + page * Hkv * D * P + off;
    if (!v_rowmajor) {
      for (int i = blockIdx.y * blockDim.x + threadIdx.x; i < Hkv * D; i += gridDim.y * blockDim.x) {
        const float x = (float)vsrc[i];   // i = kh * D + d
        kv_st1<F>(vbase + (int64_t)i * P, F == KV_BF16 ? x : x * v_inv_scale);
      }
    } else {   // previous mapping (8 dims per lane), kept for A/B (OME_ROPE_VMAP=1)
      for (int i = blockIdx.y * blockDim.x + threadIdx.x; i < Hkv * DV; i += gridDim.y * blockDim.x) {
        const int kh = i / DV, dv = i % DV;
        bf16x8 x = ld8(vsrc + kh * D + dv * 8);
        typename KVStore<F>::T* dst = v_cache + ((page * Hkv + kh) * D + dv * 8) * P + off;
#pragma unroll
        for (int j = 0; j < 8; ++j) kv_st1<F>(dst + j * P, F == KV_BF16 ? (float)x[j] : (float)x[j] * v_inv_scale);
      }
    }
  }
}

// Plain paged-cache write of already-projected K [T, Hkv, D] and V [T, Hkv, D] (used by the
// PD-disaggregation receiver and by tests).
template <int D, int P, int F>
__global__ void kv_cache_write_kernel(const bf16* __restrict__ k, const bf16* __restrict__ v, int64_t kv_stride,
                                      typename KVStore<F>::T* __restrict__ k_cache,
                                      typename KVStore<F>::T* __restrict__ v_cache, const int* __restrict__ slots,
                                      int Hkv, float k_inv_scale, float v_inv_scale) {
  const int t = blockIdx.x;
  const int slot = slots[t];
  if (slot < 0) return;
  const int64_t page = slot / P, off = slot % P;
  constexpr int DV = D / 8;
  constexpr bool q8 = F != KV_BF16;
  for (int i = threadIdx.x; i < Hkv * DV; i += blockDim.x) {
    const int kh = i / DV, dv = i % DV;
    bf16x8 kx = ld8(k + t * kv_stride + kh * D + dv * 8);
    float f[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = q8 ? (float)kx[j] * k_inv_scale : (float)kx[j];
    kv_st8<F>(k_cache + ((page * Hkv + kh) * P + off) * D + dv * 8, f);
    bf16x8 vx = ld8(v + t * kv_stride + kh * D + dv * 8);
    typename KVStore<F>::T* dst = v_cache + ((page * Hkv + kh) * D + dv * 8) * P + off;
#pragma unroll
    for (int j = 0; j < 8; ++j) kv_st1<F>(dst + j * P, q8 ? (float)vx[j] * v_inv_scale : (float)vx[j]);
  }
}

static int g_rope_split = 0;  // blocks per token (0 = one per 16 Q/K heads)
OME_API int ome_rope_set_split(int ny) {
  if (ny < 0 || ny > 8) return -1;
  g_rope_split = ny;
  return 0;
}

// kv_fmt: KVFmt of the cache tensors; k_scale / v_scale: dequantisation scales (fp8 only)
static const int g_rope_vmap = [] {
  const char* e = getenv("OME_ROPE_VMAP");
  return e ? atoi(e) : 0;
}();

OME_API int ome_rope_qkv_cache(const void* qkv, int64_t qkv_stride, const int* positions, const float* cos_sin,
                               int rot_dim, void* q_out, void* k_cache, void* v_cache, const int* slots, int T,
                               int Hq, int Hkv, int D, int P, int apply_rope, const void* q_norm_w,
                               const void* k_norm_w, float qk_eps, int kv_fmt, float k_scale, float v_scale,
                               hipStream_t stream) {
  if (T <= 0) return 0;
  if (D != 128 && D != 64 && D != 256) return -2;
  if (rot_dim > D || rot_dim % 16 != 0) return -3;
  if (P != 16) return -4;
  if (kv_fmt < 0 || kv_fmt > 2) return -5;
  const float ki = 1.f / k_scale, vi = 1.f / v_scale;
  // blocks per token: enough 4-wave blocks that each covers at most one 4-head group per wave
  const int per_block = 4 * (512 / D);
  // (decode batches only: 5.4 vs 6.3 us at T = 256; no gain once T fills the chip)
  int ny = g_rope_split > 0 ? g_rope_split : (T < 512 ? (Hq + Hkv + per_block - 1) / per_block : 1);
  ny = ny < 1 ? 1 : (ny > 8 ? 8 : ny);
  const dim3 grid(T, ny);
#define LAUNCH(DD, FF)                                                                                          \
  rope_qkv_cache_kernel<DD, 16, FF><<<grid, 256, 0, stream>>>(                                                    \
      (const bf16*)qkv, qkv_stride, positions, cos_sin, rot_dim, (bf16*)q_out, (KVStore<FF>::T*)k_cache,       \
      (KVStore<FF>::T*)v_cache, slots, Hq, Hkv, apply_rope, (const bf16*)q_norm_w, (const bf16*)k_norm_w,      \
      qk_eps, ki, vi, g_rope_vmap)
  if (D == 128) {
    if (kv_fmt == KV_BF16) LAUNCH(128, KV_BF16);
    else if (kv_fmt == KV_E4M3) LAUNCH(128, KV_E4M3);
    else LAUNCH(128, KV_E5M2);
  } else if (D == 256) {
    if (kv_fmt == KV_BF16) LAUNCH(256, KV_BF16);
    else if (kv_fmt == KV_E4M3) LAUNCH(256, KV_E4M3);
    else LAUNCH(256, KV_E5M2);
  } else {
    if (kv_fmt == KV_BF16) LAUNCH(64, KV_BF16);
    else if (kv_fmt == KV_E4M3) LAUNCH(64, KV_E4M3);
    else LAUNCH(64, KV_E5M2);
  }
#undef LAUNCH
  OME_CHECK_LAUNCH();
  return 0;
}

OME_API int ome_kv_cache_write(const void* k, const void* v, int64_t kv_stride, void* k_cache, void* v_cache,
                               const int* slots, int T, int Hkv, int D, int P, int kv_fmt, float k_scale,
                               float v_scale, hipStream_t stream) {
  if (T <= 0) return 0;
  if ((D != 128 && D != 64 && D != 256) || P != 16) return -4;
  if (kv_fmt < 0 || kv_fmt > 2) return -5;
  const float ki = 1.f / k_scale, vi = 1.f / v_scale;
#define LAUNCH(DD, FF)                                                                                    \
  kv_cache_write_kernel<DD, 16, FF><<<T, 128, 0, stream>>>((const bf16*)k, (const bf16*)v, kv_stride,   \
                                                           (KVStore<FF>::T*)k_cache,                     \
                                                           (KVStore<FF>::T*)v_cache, slots, Hkv, ki, vi)
  if (D == 128) {
    if (kv_fmt == KV_BF16) LAUNCH(128, KV_BF16);
    else if (kv_fmt == KV_E4M3) LAUNCH(128, KV_E4M3);
    else LAUNCH(128, KV_E5M2);
  } else if (D == 256) {
    if (kv_fmt == KV_BF16) LAUNCH(256, KV_BF16);
    else if (kv_fmt == KV_E4M3) LAUNCH(256, KV_E4M3);
    else LAUNCH(256, KV_E5M2);
  } else {
    if (kv_fmt == KV_BF16) LAUNCH(64, KV_BF16);
    else if (kv_fmt == KV_E4M3) LAUNCH(64, KV_E4M3);
    else LAUNCH(64, KV_E5M2);
  }
#undef LAUNCH
  OME_CHECK_LAUNCH();
  return 0;
}
