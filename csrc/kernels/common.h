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

// XCD-aware remap of a linear workgroup id (bijective for any nwg; T1 of the guide).
// Blocks b and b+8 share an XCD under round-robin dispatch, so give each XCD group a
// contiguous chunk of the logical id space.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8, x = bid % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}
