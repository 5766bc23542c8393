// RMSNorm and fused residual-add + RMSNorm (kernel K1 of SURVEY.md §2.9).
//
// One workgroup per token row; each lane holds its slice of the row in registers as
// 16-byte bf16x8 vectors (vectorised per Guideline 13), so the row is read once and
// written once: the op is purely HBM-bound.
#include "common.h"

template <int NT, int CHUNKS>
__global__ __launch_bounds__(NT) void rmsnorm_kernel(const bf16* __restrict__ x, int64_t x_stride,
                                                     const bf16* __restrict__ w, bf16* __restrict__ out,
                                                     int64_t out_stride, int H, float eps) {
  __shared__ float red[NT / 64];
  const int row = blockIdx.x;
  const bf16* xr = x + row * x_stride;
  bf16* orow = out + row * out_stride;
  const int nvec = H >> 3;
  bf16x8 v[CHUNKS];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < CHUNKS; ++c) {
    const int i = threadIdx.x + c * NT;
    if (i < nvec) {
      v[c] = ld8(xr + i * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float f = (float)v[c][j];
        ss += f * f;
      }
    }
  }
  bf16x8 wv[CHUNKS];  // issue the weight loads before the reduction's barrier
#pragma unroll
  for (int c = 0; c < CHUNKS; ++c) {
    const int i = threadIdx.x + c * NT;
    if (i < nvec) wv[c] = ld8(w + i * 8);
  }
  ss = block_sum<NT>(ss, red);
  const float rs = rsqrtf(ss / (float)H + eps);
#pragma unroll
  for (int c = 0; c < CHUNKS; ++c) {
    const int i = threadIdx.x + c * NT;
    if (i < nvec) {
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (bf16)((float)v[c][j] * rs * (float)wv[c][j]);
      st8(orow + i * 8, o);
    }
  }
}

// residual <- x + residual ; x <- rmsnorm(residual) * w      (in place, vLLM/SGLang semantics)
template <int NT, int CHUNKS>
__global__ __launch_bounds__(NT) void fused_add_rmsnorm_kernel(bf16* __restrict__ x, int64_t x_stride,
                                                               bf16* __restrict__ res, int64_t res_stride,
                                                               const bf16* __restrict__ w, int H,
                                                               float eps) {
  __shared__ float red[NT / 64];
  const int row = blockIdx.x;
  bf16* xr = x + row * x_stride;
  bf16* rr = res + row * res_stride;
  const int nvec = H >> 3;
  bf16x8 v[CHUNKS];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < CHUNKS; ++c) {
    const int i = threadIdx.x + c * NT;
    if (i < nvec) {
      bf16x8 a = ld8(xr + i * 8), b = ld8(rr + i * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        // round the sum to bf16 first: the residual stream is stored in bf16
        bf16 s = (bf16)((float)a[j] + (float)b[j]);
        v[c][j] = s;
        float f = (float)s;
        ss += f * f;
      }
      st8(rr + i * 8, v[c]);
    }
  }
  bf16x8 wv[CHUNKS];  // issue the weight loads before the reduction's barrier
#pragma unroll
  for (int c = 0; c < CHUNKS; ++c) {
    const int i = threadIdx.x + c * NT;
    if (i < nvec) wv[c] = ld8(w + i * 8);
  }
  ss = block_sum<NT>(ss, red);
  const float rs = rsqrtf(ss / (float)H + eps);
#pragma unroll
  for (int c = 0; c < CHUNKS; ++c) {
    const int i = threadIdx.x + c * NT;
    if (i < nvec) {
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (bf16)((float)v[c][j] * rs * (float)wv[c][j]);
      st8(xr + i * 8, o);
    }
  }
}

// LayerNorm with bias (Starcoder2, GPT-NeoX): out = (x - mean) * rstd * w + b; with ``res`` set the
// residual add is fused in front (res <- x + res, normalise res, write x), like fused_add_rmsnorm.
template <int NT, int CHUNKS, bool ADD>
__global__ __launch_bounds__(NT) void layernorm_kernel(bf16* __restrict__ x, int64_t x_stride,
                                                       bf16* __restrict__ res, int64_t res_stride,
                                                       const bf16* __restrict__ w, const bf16* __restrict__ b,
                                                       bf16* __restrict__ out, int64_t out_stride, int H, float eps) {
  __shared__ float red[NT / 64];
  const int row = blockIdx.x;
  bf16* xr = x + row * x_stride;
  const int nvec = H >> 3;
  bf16x8 v[CHUNKS];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CHUNKS; ++c) {
    const int i = threadIdx.x + c * NT;
    if (i < nvec) {
      v[c] = ld8(xr + i * 8);
      if constexpr (ADD) {
        bf16* rr = res + row * res_stride;
        const bf16x8 r = ld8(rr + i * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] = (bf16)((float)v[c][j] + (float)r[j]);
        st8(rr + i * 8, v[c]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s += (float)v[c][j];
    }
  }
  const float mean = block_sum<NT>(s, red) / (float)H;
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < CHUNKS; ++c) {
    const int i = threadIdx.x + c * NT;
    if (i < nvec) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = (float)v[c][j] - mean;
        ss += d * d;
      }
    }
  }
  const float rstd = rsqrtf(block_sum<NT>(ss, red) / (float)H + eps);
  bf16* orow = ADD ? xr : out + row * out_stride;
#pragma unroll
  for (int c = 0; c < CHUNKS; ++c) {
    const int i = threadIdx.x + c * NT;
    if (i < nvec) {
      const bf16x8 wv = ld8(w + i * 8);
      bf16x8 bv = {};
      if (b != nullptr) bv = ld8(b + i * 8);
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (bf16)(((float)v[c][j] - mean) * rstd * (float)wv[j] + (float)bv[j]);
      st8(orow + i * 8, o);
    }
  }
}

#define DISPATCH_CHUNKS(H, NT, ...)                         \
  do {                                                      \
    const int _c = ((H) / 8 + (NT)-1) / (NT);               \
    if (_c <= 1) { constexpr int CH = 1; __VA_ARGS__; }     \
    else if (_c <= 2) { constexpr int CH = 2; __VA_ARGS__; } \
    else if (_c <= 4) { constexpr int CH = 4; __VA_ARGS__; } \
    else if (_c <= 8) { constexpr int CH = 8; __VA_ARGS__; } \
    else return -1;                                         \
  } while (0)

OME_API int ome_rmsnorm(const void* x, int64_t x_stride, const void* w, void* out, int64_t out_stride,
                        int rows, int H, float eps, hipStream_t stream) {
  if (H % 8 != 0 || rows <= 0) return rows == 0 ? 0 : -2;
  // Small batches (decode) use 128-thread blocks to keep more lanes' loads in flight per CU.
  if (rows < 512) {
    DISPATCH_CHUNKS(H, 128, (rmsnorm_kernel<128, CH><<<rows, 128, 0, stream>>>(
                                (const bf16*)x, x_stride, (const bf16*)w, (bf16*)out, out_stride, H, eps)));
  } else {
    DISPATCH_CHUNKS(H, 256, (rmsnorm_kernel<256, CH><<<rows, 256, 0, stream>>>(
                                (const bf16*)x, x_stride, (const bf16*)w, (bf16*)out, out_stride, H, eps)));
  }
  OME_CHECK_LAUNCH();
  return 0;
}

static int g_norm_threads = 0;  // 0 = measured default; 128 / 256 / 512 for experiments
OME_API int ome_norm_set_threads(int nt) {
  if (nt != 0 && nt != 128 && nt != 256 && nt != 512) return -1;
  g_norm_threads = nt;
  return 0;
}

OME_API int ome_fused_add_rmsnorm(void* x, int64_t x_stride, void* res, int64_t res_stride, const void* w,
                                  int rows, int H, float eps, hipStream_t stream) {
  if (H % 8 != 0 || rows <= 0) return rows == 0 ? 0 : -2;
  if (g_norm_threads == 512) {
    DISPATCH_CHUNKS(H, 512, (fused_add_rmsnorm_kernel<512, CH><<<rows, 512, 0, stream>>>(
                                (bf16*)x, x_stride, (bf16*)res, res_stride, (const bf16*)w, H, eps)));
  } else if (g_norm_threads == 256) {
    DISPATCH_CHUNKS(H, 256, (fused_add_rmsnorm_kernel<256, CH><<<rows, 256, 0, stream>>>(
                                (bf16*)x, x_stride, (bf16*)res, res_stride, (const bf16*)w, H, eps)));
  } else if (g_norm_threads == 128) {
    DISPATCH_CHUNKS(H, 128, (fused_add_rmsnorm_kernel<128, CH><<<rows, 128, 0, stream>>>(
                                (bf16*)x, x_stride, (bf16*)res, res_stride, (const bf16*)w, H, eps)));
  } else if (rows < 512) {
    // decode batches: 8 waves per row (3.05 vs 4.15 us for 128 threads at 256 x 4096,
    // profiles/r03_small_kernels.txt)
    DISPATCH_CHUNKS(H, 512, (fused_add_rmsnorm_kernel<512, CH><<<rows, 512, 0, stream>>>(
                                (bf16*)x, x_stride, (bf16*)res, res_stride, (const bf16*)w, H, eps)));
  } else {
    DISPATCH_CHUNKS(H, 256, (fused_add_rmsnorm_kernel<256, CH><<<rows, 256, 0, stream>>>(
                                (bf16*)x, x_stride, (bf16*)res, res_stride, (const bf16*)w, H, eps)));
  }
  OME_CHECK_LAUNCH();
  return 0;
}

// res == nullptr: out = LN(x); else res <- x + res, x <- LN(res) (out unused)
OME_API int ome_layernorm(void* x, int64_t x_stride, void* res, int64_t res_stride, const void* w, const void* b,
                          void* out, int64_t out_stride, int rows, int H, float eps, hipStream_t stream) {
  if (H % 8 != 0 || rows <= 0) return rows == 0 ? 0 : -2;
  if (res != nullptr) {
    DISPATCH_CHUNKS(H, 256, (layernorm_kernel<256, CH, true><<<rows, 256, 0, stream>>>(
                                (bf16*)x, x_stride, (bf16*)res, res_stride, (const bf16*)w, (const bf16*)b,
                                nullptr, 0, H, eps)));
  } else {
    DISPATCH_CHUNKS(H, 256, (layernorm_kernel<256, CH, false><<<rows, 256, 0, stream>>>(
                                (bf16*)x, x_stride, nullptr, 0, (const bf16*)w, (const bf16*)b, (bf16*)out,
                                out_stride, H, eps)));
  }
  OME_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------------------------
// Per-head RMSNorm + complex-pair RoPE + row scatter (Qwen-Image MMDiT q / k; v with no norm and
// no rotation): one wave per (row, head).  x row r, head h = x[r * xs + h * HD .. +HD); w [HD] (null:
// no norm); cs [T][HD/2][2] fp32 (cos, sin) (null: no rotation); the result goes to row
// dst[r] (null: r) of out (row stride os) -- the joint [text; image] sequence is assembled by
// the writes themselves, no gather pass.  Rounding as the eager path: normed value rounded to
// bf16 before the fp32 rotation.
template <int HD>
__global__ __launch_bounds__(256) void qk_norm_rope_kernel(const bf16* __restrict__ x, int64_t xs,
                                                           const bf16* __restrict__ w, const float* __restrict__ cs,
                                                           int T, int H, float eps, bf16* __restrict__ out,
                                                           int64_t os, const int* __restrict__ dst) {
  constexpr int NP = HD / 2, PPL = (NP + 63) / 64;   // complex pairs, pairs per lane
  const int lane = threadIdx.x & 63;
  const int64_t wid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (wid >= (int64_t)T * H) return;   // whole wave
  const int r = (int)(wid / H), h = (int)(wid - (int64_t)r * H);
  const bf16* xp = x + (int64_t)r * xs + (int64_t)h * HD;
  float v0[PPL], v1[PPL], ss = 0.f;
#pragma unroll
  for (int j = 0; j < PPL; ++j) {
    const int p = lane + 64 * j;
    v0[j] = v1[j] = 0.f;
    if (p < NP) {
      const bf16x2 t = *reinterpret_cast<const bf16x2*>(xp + 2 * p);
      v0[j] = (float)t[0];
      v1[j] = (float)t[1];
      ss += v0[j] * v0[j] + v1[j] * v1[j];
    }
  }
  if (w != nullptr) {
    const float inv = rsqrtf(wave_sum(ss) / HD + eps);
#pragma unroll
    for (int j = 0; j < PPL; ++j) {
      const int p = lane + 64 * j;
      if (p < NP) {
        v0[j] = (float)(bf16)((float)(bf16)(v0[j] * inv) * (float)w[2 * p]);
        v1[j] = (float)(bf16)((float)(bf16)(v1[j] * inv) * (float)w[2 * p + 1]);
      }
    }
  }
  bf16* op = out + (int64_t)(dst != nullptr ? dst[r] : r) * os + (int64_t)h * HD;
#pragma unroll
  for (int j = 0; j < PPL; ++j) {
    const int p = lane + 64 * j;
    if (p >= NP) continue;
    float a = v0[j], b = v1[j];
    if (cs != nullptr) {
      const float2 c = *reinterpret_cast<const float2*>(cs + ((int64_t)r * NP + p) * 2);
      a = v0[j] * c.x - v1[j] * c.y;
      b = v0[j] * c.y + v1[j] * c.x;
    }
    bf16x2 o;
    o[0] = (bf16)a;
    o[1] = (bf16)b;
    *reinterpret_cast<bf16x2*>(op + 2 * p) = o;
  }
}

OME_API int ome_qk_norm_rope(const void* x, int64_t xs, const void* w, const float* cs, int T, int H, int hd,
                             float eps, void* out, int64_t os, const int* dst, hipStream_t stream) {
  if (T <= 0 || H <= 0) return 0;
  if ((xs | os) & 1) return -3;
  const int64_t waves = (int64_t)T * H;
  dim3 grid((unsigned)((waves + 3) / 4));
  switch (hd) {
    case 64:
      qk_norm_rope_kernel<64><<<grid, 256, 0, stream>>>((const bf16*)x, xs, (const bf16*)w, cs, T, H, eps, (bf16*)out,
                                                        os, dst);
      break;
    case 128:
      qk_norm_rope_kernel<128><<<grid, 256, 0, stream>>>((const bf16*)x, xs, (const bf16*)w, cs, T, H, eps,
                                                         (bf16*)out, os, dst);
      break;
    case 256:
      qk_norm_rope_kernel<256><<<grid, 256, 0, stream>>>((const bf16*)x, xs, (const bf16*)w, cs, T, H, eps,
                                                         (bf16*)out, os, dst);
      break;
    default:
      return -2;
  }
  OME_CHECK_LAUNCH();
  return 0;
}
