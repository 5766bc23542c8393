// Element-wise / gather kernels: SiLU-and-mul (K9), GELU-tanh-and-mul, vocab-parallel
// embedding gather (K13), residual add, and embedding pooling + L2 normalisation (K14).
// All memory-bound: 16-byte bf16x8 vectors per lane, grid-stride loops capped at
// 256 CUs x 8 blocks (Guideline 11).
#include "common.h"

__device__ __forceinline__ float silu(float x) { return x / (1.f + __expf(-x)); }
__device__ __forceinline__ float gelu_tanh(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  return 0.5f * x * (1.f + tanhf(k0 * (x + k1 * x * x * x)));
}

template <int ACT>
__global__ __launch_bounds__(256) void act_and_mul_kernel(const bf16* __restrict__ x, bf16* __restrict__ out,
                                                          int64_t rows, int I, bool il) {
  // grid (column blocks, rows): no per-element 64-bit division, every lane one 16-B vector.
  // il: gate / up columns interleaved in 16-column blocks (the layout of a gate_up weight
  // interleaved for the fused SiLU*mul GEMM epilogue, ops.interleave_gate_up)
  const int nv = I >> 3;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t r = blockIdx.y;
  if (c >= nv) return;
  const bf16* xr = x + r * 2 * I;
  const int gcol = il ? ((c * 8) >> 4) * 32 + ((c * 8) & 15) : c * 8;
  const int ucol = il ? gcol + 16 : I + c * 8;
  bf16x8 g = ld8(xr + gcol), u = ld8(xr + ucol), o;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float gf = (float)g[j];
    if constexpr (ACT == 2 || ACT == 3) {
      // clamped SwiGLU / GeGELU: (clamp(u, -L, L) + 1) * g' * sigmoid(1.702 g'), g' = min(g, L);
      // L = 7 (GPT-OSS), 20 (Phi-3-small gegelu_limit)
      constexpr float L = ACT == 2 ? 7.f : 20.f;
      const float g2 = fminf(gf, L);
      const float u2 = fminf(fmaxf((float)u[j], -L), L);
      o[j] = (bf16)((u2 + 1.f) * g2 / (1.f + __expf(-1.702f * g2)));
    } else {
      const float a = ACT == 0 ? silu(gf) : gelu_tanh(gf);
      o[j] = (bf16)(a * (float)u[j]);
    }
  }
  st8(out + r * I + c * 8, o);
}

// Non-gated activation (Starcoder2 / GPT-NeoX MLPs), in place on a contiguous bf16 tensor:
// ACT 1 = GELU-tanh, 3 = GELU (erf), 0 = SiLU, 4 = ReLU^2 (NemotronH, Persimmon, Arcee), 5 = ReLU (OPT)
template <int ACT>
__global__ __launch_bounds__(256) void act_kernel(bf16* __restrict__ x, int64_t nvec) {
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * blockDim.x) {
    bf16x8 a = ld8(x + v * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float f = (float)a[j];
      a[j] = (bf16)(ACT == 0   ? silu(f)
                     : ACT == 1 ? gelu_tanh(f)
                     : ACT == 4 ? fmaxf(f, 0.f) * fmaxf(f, 0.f)
                     : ACT == 5 ? fmaxf(f, 0.f)
                                : 0.5f * f * (1.f + erff(f * 0.7071067811865476f)));
    }
    st8(x + v * 8, a);
  }
}

static inline int grid_for(int64_t work, int nt) {
  int64_t g = (work + nt - 1) / nt;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

// act: 0 SiLU, 1 GELU-tanh, 2 GPT-OSS clamped SwiGLU (limit 7), 3 Phi-3-small GeGELU (limit 20);
// | 16: interleaved gate/up (16-col blocks)
OME_API int ome_act_and_mul(const void* x, void* out, int64_t rows, int I, int act, hipStream_t stream) {
  if (rows <= 0) return 0;
  const bool il = (act & 16) != 0;
  act &= 15;
  if (I % 8 || (il && I % 16)) return -2;
  for (int64_t r0 = 0; r0 < rows; r0 += 65535) {  // grid.y limit
    const int64_t n = rows - r0 < 65535 ? rows - r0 : 65535;
    const dim3 g((I / 8 + 255) / 256, (unsigned)n);
    const bf16* xp = (const bf16*)x + r0 * 2 * I;
    bf16* op = (bf16*)out + r0 * I;
    if (act == 0)
      act_and_mul_kernel<0><<<g, 256, 0, stream>>>(xp, op, n, I, il);
    else if (act == 1)
      act_and_mul_kernel<1><<<g, 256, 0, stream>>>(xp, op, n, I, il);
    else if (act == 2)
      act_and_mul_kernel<2><<<g, 256, 0, stream>>>(xp, op, n, I, il);
    else
      act_and_mul_kernel<3><<<g, 256, 0, stream>>>(xp, op, n, I, il);
  }
  OME_CHECK_LAUNCH();
  return 0;
}

OME_API int ome_act(void* x, int64_t n, int act, hipStream_t stream) {
  if (n <= 0) return 0;
  if (n % 8) return -2;
  const int64_t nv = n / 8;
  const int g = grid_for(nv, 256);
  if (act == 0) act_kernel<0><<<g, 256, 0, stream>>>((bf16*)x, nv);
  else if (act == 1) act_kernel<1><<<g, 256, 0, stream>>>((bf16*)x, nv);
  else if (act == 4) act_kernel<4><<<g, 256, 0, stream>>>((bf16*)x, nv);
  else if (act == 5) act_kernel<5><<<g, 256, 0, stream>>>((bf16*)x, nv);
  else if (act == 3) act_kernel<3><<<g, 256, 0, stream>>>((bf16*)x, nv);
  else return -3;
  OME_CHECK_LAUNCH();
  return 0;
}

// out[t] = table[ids[t] - vocab_start] if the id falls in this rank's shard, else 0.
__global__ __launch_bounds__(256) void embedding_kernel(const int* __restrict__ ids, const bf16* __restrict__ table,
                                                        bf16* __restrict__ out, int T, int H, int vocab_start,
                                                        int vocab_end) {
  const int nv = H >> 3;
  for (int t = blockIdx.x; t < T; t += gridDim.x) {
    const int id = ids[t];
    const bool own = id >= vocab_start && id < vocab_end;
    const bf16* src = table + (int64_t)(own ? id - vocab_start : 0) * H;
    for (int c = threadIdx.x; c < nv; c += blockDim.x) {
      bf16x8 v = {};
      if (own) v = ld8(src + c * 8);
      st8(out + (int64_t)t * H + c * 8, v);
    }
  }
}

OME_API int ome_embedding(const int* ids, const void* table, void* out, int T, int H, int vocab_start,
                          int vocab_end, hipStream_t stream) {
  if (T <= 0) return 0;
  if (H % 8) return -2;
  const int g = T < 4096 ? T : 4096;
  embedding_kernel<<<g, 256, 0, stream>>>(ids, (const bf16*)table, (bf16*)out, T, H, vocab_start, vocab_end);
  OME_CHECK_LAUNCH();
  return 0;
}

// Pooling for embedding models (--is-embedding): last-token or mean pooling over each sequence
// followed by optional L2 normalisation. hidden [T, H] bf16, cu_lens [S+1] -> out [S, H] f32.
__global__ __launch_bounds__(256) void pool_kernel(const bf16* __restrict__ hidden, const int* __restrict__ cu,
                                                   float* __restrict__ out, int H, int mode, int normalize) {
  __shared__ float red[4];
  const int s = blockIdx.x;
  const int b = cu[s], e = cu[s + 1];
  float ss = 0.f;
  for (int d = threadIdx.x; d < H; d += 256) {
    float v = 0.f;
    if (mode == 0) {
      v = (float)hidden[(int64_t)(e - 1) * H + d];
    } else if (mode == 2) {  // first token (CLS pooling: BERT / XLM-RoBERTa encoders)
      v = (float)hidden[(int64_t)b * H + d];
    } else {
      for (int t = b; t < e; ++t) v += (float)hidden[(int64_t)t * H + d];
      v /= (float)(e - b > 0 ? e - b : 1);
    }
    out[(int64_t)s * H + d] = v;
    ss += v * v;
  }
  if (!normalize) return;
  ss = block_sum<256>(ss, red);
  const float inv = 1.f / fmaxf(sqrtf(ss), 1e-12f);
  for (int d = threadIdx.x; d < H; d += 256) out[(int64_t)s * H + d] *= inv;
}

OME_API int ome_pool(const void* hidden, const int* cu_lens, void* out, int S, int H, int mode, int normalize,
                     hipStream_t stream) {
  if (S <= 0) return 0;
  pool_kernel<<<S, 256, 0, stream>>>((const bf16*)hidden, cu_lens, (float*)out, H, mode, normalize);
  OME_CHECK_LAUNCH();
  return 0;
}

// Overlapped scheduling: the next step is enqueued before the previous step's sampled ids
// reach the host, so rows whose input token is still "pending" take it from the previous
// step's device output: ids[i] = prev[src[i]] when src[i] >= 0 (one tiny kernel, no sync).
__global__ void fill_pending_kernel(int* __restrict__ ids, const int* __restrict__ src, const int* __restrict__ prev,
                                    int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const int s = src[i];
    if (s >= 0) ids[i] = prev[s];
  }
}

OME_API int ome_fill_pending(int* ids, const int* src, const int* prev, int n, hipStream_t stream) {
  if (n <= 0) return 0;
  fill_pending_kernel<<<(n + 255) / 256, 256, 0, stream>>>(ids, src, prev, n);
  OME_CHECK_LAUNCH();
  return 0;
}

// Byte copy between any two device-visible addresses, one of which may be pinned host memory
// mapped into the GPU's address space (hipHostMalloc).  The per-step metadata H2D and the sampled
// ids D2H go through this kernel instead of hipMemcpyAsync, so every per-step transfer is a plain
// kernel dispatch on the compute stream (no copy-engine / runtime blit path, no per-step pinning).
__global__ __launch_bounds__(256) void copy_mapped_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                          int64_t n16, const unsigned char* __restrict__ src_tail,
                                                          unsigned char* __restrict__ dst_tail, int tail) {
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int64_t i = i0; i < n16; i += (int64_t)gridDim.x * blockDim.x) dst[i] = src[i];
  if (i0 < tail) dst_tail[i0] = src_tail[i0];
}

OME_API int ome_copy_mapped(const void* src, void* dst, int64_t nbytes, hipStream_t stream) {
  if (nbytes <= 0) return 0;
  // 16-B vectors when both ends are 16-B aligned, bytes otherwise
  const bool vec = ((uintptr_t)src % 16 == 0) && ((uintptr_t)dst % 16 == 0);
  const int64_t n16 = vec ? nbytes / 16 : 0;
  const int64_t tail = nbytes - n16 * 16;
  if (tail > (1 << 20)) return -2;  // unaligned bulk copies are not this kernel's job
  const int64_t work = n16 > tail ? n16 : tail;
  int grid = (int)((work + 255) / 256);
  grid = grid < 1 ? 1 : (grid > 1024 ? 1024 : grid);
  if (tail > (int64_t)grid * 256) grid = (int)((tail + 255) / 256);
  copy_mapped_kernel<<<grid, 256, 0, stream>>>((const uint4*)src, (uint4*)dst, n16,
                                               (const unsigned char*)src + n16 * 16, (unsigned char*)dst + n16 * 16,
                                               (int)tail);
  OME_CHECK_LAUNCH();
  return 0;
}

// Device address of a pinned host allocation (identity on ROCm for hipHostMalloc memory).
OME_API int ome_host_device_ptr(void* host, void** dev) {
  return hipHostGetDevicePointer(dev, host, 0) == hipSuccess ? 0 : -1;
}
