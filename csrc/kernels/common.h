// ome_amd — shared device helpers for the gfx950 (CDNA4, MI355X) kernel library.
//
// Everything here is written for wave64 + MFMA.  bf16 is carried as clang's native
// `__bf16` (hipcc lowers f32->bf16 casts to v_cvt_pk_bf16_f32 on gfx950, which keeps
// NaNs as NaNs — see MI355X_MICROARCH.md "Correctness boundaries").
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define OME_API extern "C" __attribute__((visibility("default")))
#define WAVE 64

#define OME_CHECK_LAUNCH() \
  do {                                   \
    hipError_t _e = hipGetLastError();   \
    if (_e != hipSuccess) return (int)_e; \
  } while (0)

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

// Reductions over the 4 lane groups of 16 (lanes l, l^16, l^32, l^48: an MFMA 16x16 tile's
// row spread) on the gfx950 permlane swaps: v_permlane16_swap / v_permlane32_swap(x, x) leave
// x[l] in one result and x[l^16] (x[l^32]) in the other in EVERY lane, so max / sum of the pair
// is the xor-shuffle result bit for bit -- two VALU ops per level instead of a ds_bpermute round
// trip whose lgkmcnt wait also drains the wave's in-flight LDS reads.  v_max_f32 by asm: fmaxf
// on the swap results adds two canonicalising v_max per level.
__device__ __forceinline__ float vmax_f32(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float group4_max(float v) {
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = vmax_f32(__uint_as_float(a[0]), __uint_as_float(a[1]));
  auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return vmax_f32(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ float group4_sum(float v) {
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// Block-wide sum for blockDim.x == NT (multiple of 64). `red` must hold NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if constexpr (NT == 64) {
    return v;
  } else {
    if (l == 0) red[w] = v;
    __syncthreads();
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) t += red[i];
    __syncthreads();
    return t;
  }
}

__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }

// 16-byte vector load/store helpers (global_load_dwordx4 / global_store_dwordx4).
__device__ __forceinline__ bf16x8 ld8(const bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }
__device__ __forceinline__ void st8(bf16* p, bf16x8 v) { *reinterpret_cast<bf16x8*>(p) = v; }
__device__ __forceinline__ bf16x4 ld4(const bf16* p) { return *reinterpret_cast<const bf16x4*>(p); }

// ------------------------------------------------------------------------------------------
// Paged KV-cache element formats (K15, `--kv-cache-dtype`).  The attention kernels are
// templated on the format; fp8 entries are converted to bf16 in registers right before the
// MFMA (the hardware converters v_cvt_pk_f32_fp8 / _bf8 on gfx950 use the OCP encodings), and
// the per-layer scalar scales are folded into the softmax scale (K) and the output
// normalisation (V), so the inner loops never multiply by a scale.
// ------------------------------------------------------------------------------------------
enum KVFmt { KV_BF16 = 0, KV_E4M3 = 1, KV_E5M2 = 2 };

template <int F> struct KVStore { typedef uint8_t T; };
template <> struct KVStore<KV_BF16> { typedef bf16 T; };

typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int F>
__device__ __forceinline__ bf16x4 fp8x4_to_bf16(uint32_t v) {
  f32x2 lo, hi;
  if constexpr (F == KV_E4M3) {
    lo = __builtin_amdgcn_cvt_pk_f32_fp8((int)v, false);
    hi = __builtin_amdgcn_cvt_pk_f32_fp8((int)v, true);
  } else {
    lo = __builtin_amdgcn_cvt_pk_f32_bf8((int)v, false);
    hi = __builtin_amdgcn_cvt_pk_f32_bf8((int)v, true);
  }
  return bf16x4{(bf16)lo.x, (bf16)lo.y, (bf16)hi.x, (bf16)hi.y};
}

template <int F>
__device__ __forceinline__ bf16x8 fp8x8_to_bf16(uint2 v) {
  const bf16x4 a = fp8x4_to_bf16<F>(v.x), b = fp8x4_to_bf16<F>(v.y);
  return bf16x8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

// 8 / 4 consecutive cache elements -> bf16
template <int F>
__device__ __forceinline__ bf16x8 kv_ld8(const typename KVStore<F>::T* p) {
  if constexpr (F == KV_BF16) return ld8(p);
  else return fp8x8_to_bf16<F>(*reinterpret_cast<const uint2*>(p));
}
template <int F>
__device__ __forceinline__ bf16x4 kv_ld4(const typename KVStore<F>::T* p) {
  if constexpr (F == KV_BF16) return ld4(p);
  else return fp8x4_to_bf16<F>(*reinterpret_cast<const uint32_t*>(p));
}

// float pair -> saturated fp8 pair written into the low / high 16 bits of `old`
template <int F, bool HI>
__device__ __forceinline__ int fp8_pack2(float a, float b, int old) {
  constexpr float M = F == KV_E4M3 ? 448.f : 57344.f;
  a = fminf(fmaxf(a, -M), M);
  b = fminf(fmaxf(b, -M), M);
  if constexpr (F == KV_E4M3) return __builtin_amdgcn_cvt_pk_fp8_f32(a, b, old, HI);
  else return __builtin_amdgcn_cvt_pk_bf8_f32(a, b, old, HI);
}

// store 8 floats (already multiplied by the inverse scale) as cache elements
template <int F>
__device__ __forceinline__ void kv_st8(typename KVStore<F>::T* p, const float (&f)[8]) {
  if constexpr (F == KV_BF16) {
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16)f[j];
    st8(p, o);
  } else {
    uint2 o;
    o.x = (uint32_t)fp8_pack2<F, true>(f[2], f[3], fp8_pack2<F, false>(f[0], f[1], 0));
    o.y = (uint32_t)fp8_pack2<F, true>(f[6], f[7], fp8_pack2<F, false>(f[4], f[5], 0));
    *reinterpret_cast<uint2*>(p) = o;
  }
}

template <int F>
__device__ __forceinline__ void kv_st1(typename KVStore<F>::T* p, float f) {
  if constexpr (F == KV_BF16) *p = (bf16)f;
  else *p = (uint8_t)(fp8_pack2<F, false>(f, 0.f, 0) & 0xff);
}

// XCD-aware remap of a linear workgroup id (bijective for any nwg; T1 of the guide).
// Blocks b and b+8 share an XCD under round-robin dispatch, so give each XCD group a
// contiguous chunk of the logical id space.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8, x = bid % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}
