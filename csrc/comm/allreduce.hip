// Custom tensor-parallel all-reduce over xGMI peer mappings.
//
// An 8x MI355X node is a full mesh: every GPU has a direct xGMI link to every other one, so a
// small all-reduce is fastest as ONE kernel in which each GPU reads all peers' inputs directly
// (no ring, no RCCL proxy), and a large one as reduce-scatter + all-gather over the same
// mappings, which moves (N-1)/N of the bytes per link instead of the ring's 2(N-1)/N hops.
//
// Memory per rank (shared with the peers through hipIpc handles):
//   signal  (hipDeviceMallocUncached): start/end flags [kMaxBlocks][kMaxRanks] + per-block epoch
//           counters — uncached so spinning never reads a stale line;
//   data    (coarse-grained): the rank's staged input (one-shot) or reduced chunk (two-shot).
// Synchronisation is per workgroup: block b of every rank bumps its epoch (kept in device memory,
// so captured HIP graphs replay correctly), stores it into flag[b][rank] of every peer with a
// system-scope release, and waits (system-scope acquire, bounded spin) until all peers' flags
// reached the epoch.  A bounded spin that expires records an error word instead of hanging the
// GPU.  Accumulation is in fp32.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>

#define OME_API extern "C" __attribute__((visibility("default")))

namespace {

constexpr int kMaxRanks = 8;
constexpr int kMaxBlocks = 128;
constexpr int kThreads = 512;
constexpr uint64_t kSpinLimitDefault = 1ull << 26;

struct Signal {
  uint32_t start[kMaxBlocks][kMaxRanks];
  uint32_t end[kMaxBlocks][kMaxRanks];
  uint32_t epoch[kMaxBlocks];
  uint32_t error;
};

struct Peers {
  Signal* sig[kMaxRanks];
  char* data[kMaxRanks];
  // fault handling (kernel arguments, so the normal path pays one scalar compare):
  //   spin_limit  bounded flag waits (OME_COMM_SPIN_LIMIT, s_sleep(1) iterations);
  //   host_err    host-mapped word that an expired wait also sets, so a host watchdog sees the
  //               failure without a HIP call (a blocking copy could queue behind the hung work);
  //   fault       host-mapped {stall iterations} word, non-null only when OME_COMM_FAULT is set:
  //               the flag lanes sleep that long before publishing (a stalled rank)
  uint64_t spin_limit;
  uint32_t* host_err;
  const uint32_t* fault;
};

typedef __bf16 bf16;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void st_release(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ uint32_t ld_acquire(uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// all ranks' block b meet here; `which` 0 = start flags, 1 = end flags.
// Publish order (MI355X_MICROARCH.md, inter-workgroup visibility): every wave drains its stores
// (`s_waitcnt vmcnt(0)`), workgroup barrier, then the flag lanes release at system scope and wait
// once more before the flag store (ROCm 7.2 may drop the fence's own wait).
__device__ __forceinline__ void block_barrier(const Peers& P, int rank, int world, uint32_t epoch, int which) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x < world) {
    if (P.fault) {   // fault injection: stall before the publish
      const uint32_t n = __hip_atomic_load(P.fault, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      for (uint32_t i = 0; i < n; ++i) __builtin_amdgcn_s_sleep(127);
    }
    __threadfence_system();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    Signal* peer = P.sig[threadIdx.x];
    st_release(which ? &peer->end[blockIdx.x][rank] : &peer->start[blockIdx.x][rank], epoch);
    Signal* self = P.sig[rank];
    uint32_t* f = which ? &self->end[blockIdx.x][threadIdx.x] : &self->start[blockIdx.x][threadIdx.x];
    uint64_t spins = 0;
    while (ld_acquire(f) < epoch) {
      if (++spins > P.spin_limit) {
        atomicOr(&self->error, 1u);
        if (P.host_err) __hip_atomic_store(P.host_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // make the peers' released data visible to plain loads
}

__device__ __forceinline__ void add8(float* acc, u32x4 v) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t w = v[i];
    acc[2 * i] += __uint_as_float(w << 16);
    acc[2 * i + 1] += __uint_as_float(w & 0xffff0000u);
  }
}

__device__ __forceinline__ u32x4 pack8(const float* a) {
  u32x4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const bf16 lo = (bf16)a[2 * i], hi = (bf16)a[2 * i + 1];
    r[i] = (uint32_t)__builtin_bit_cast(uint16_t, lo) | ((uint32_t)__builtin_bit_cast(uint16_t, hi) << 16);
  }
  return r;
}

template <int W>
__global__ __launch_bounds__(kThreads) void ar_one_shot(Peers P, int rank, int64_t n_vec, const u32x4* __restrict__ in,
                                                        u32x4* __restrict__ out) {
  __shared__ uint32_t s_epoch;
  Signal* self = P.sig[rank];
  if (threadIdx.x == 0) s_epoch = self->epoch[blockIdx.x] + 1;
  // in-kernel staging (no D2D copy node): block b stages exactly the vectors block b of every
  // rank reads below; the start barrier publishes them
  if (in != nullptr) {
    u32x4* mine = reinterpret_cast<u32x4*>(P.data[rank]);
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n_vec; i += (int64_t)gridDim.x * kThreads)
      mine[i] = in[i];
  }
  __syncthreads();
  const uint32_t epoch = s_epoch;
  block_barrier(P, rank, W, epoch, 0);
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n_vec; i += (int64_t)gridDim.x * kThreads) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    u32x4 v[W];
#pragma unroll
    for (int r = 0; r < W; ++r) v[r] = reinterpret_cast<const u32x4*>(P.data[(rank + r) % W])[i];
#pragma unroll
    for (int r = 0; r < W; ++r) add8(acc, v[r]);
    out[i] = pack8(acc);
  }
  block_barrier(P, rank, W, epoch, 1);  // nobody may restage its buffer while a peer still reads it
  if (threadIdx.x == 0) self->epoch[blockIdx.x] = epoch;
}

// reduce-scatter into the own buffer's chunk, then all-gather the peers' reduced chunks
// `red_vec` = offset (in 16-B vectors) of the reduced-chunk half of every rank's buffer.  It is
// the registered capacity, NOT the message size: a next call of a different size restages its
// input into [0, n') only, which can never overlap the reduced chunk a slower peer is still
// gathering from this call.
template <int W>
__global__ __launch_bounds__(kThreads) void ar_two_shot(Peers P, int rank, int64_t n_vec, int64_t red_vec,
                                                        const u32x4* __restrict__ in, u32x4* __restrict__ out) {
  __shared__ uint32_t s_epoch;
  Signal* self = P.sig[rank];
  if (threadIdx.x == 0) s_epoch = self->epoch[blockIdx.x] + 1;
  const int64_t chunk = (n_vec + W - 1) / W;
  if (in != nullptr) {   // stage what block b of every rank reduces from us: its slice of each chunk
    u32x4* mine = reinterpret_cast<u32x4*>(P.data[rank]);
    for (int c = 0; c < W; ++c) {
      const int64_t lo = c * chunk, hi = lo + chunk < n_vec ? lo + chunk : n_vec;
      for (int64_t i = lo + (int64_t)blockIdx.x * kThreads + threadIdx.x; i < hi; i += (int64_t)gridDim.x * kThreads)
        mine[i] = in[i];
    }
  }
  __syncthreads();
  const uint32_t epoch = s_epoch;
  block_barrier(P, rank, W, epoch, 0);
  const int64_t c0 = rank * chunk, c1 = c0 + chunk < n_vec ? c0 + chunk : n_vec;
  u32x4* mine = reinterpret_cast<u32x4*>(P.data[rank]);
  for (int64_t i = c0 + (int64_t)blockIdx.x * kThreads + threadIdx.x; i < c1; i += (int64_t)gridDim.x * kThreads) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    u32x4 v[W];
#pragma unroll
    for (int r = 0; r < W; ++r) v[r] = reinterpret_cast<const u32x4*>(P.data[(rank + r) % W])[i];
#pragma unroll
    for (int r = 0; r < W; ++r) add8(acc, v[r]);
    const u32x4 s = pack8(acc);
    out[i] = s;
    mine[red_vec + i] = s;  // peers gather it from the reduced half of our buffer
  }
  block_barrier(P, rank, W, epoch, 1);
  for (int r = 1; r < W; ++r) {
    const int src = (rank + r) % W;
    const int64_t s0 = src * chunk, s1 = s0 + chunk < n_vec ? s0 + chunk : n_vec;
    const u32x4* theirs = reinterpret_cast<const u32x4*>(P.data[src]) + red_vec;
    for (int64_t i = s0 + (int64_t)blockIdx.x * kThreads + threadIdx.x; i < s1; i += (int64_t)gridDim.x * kThreads)
      out[i] = theirs[i];
  }
  // No closing meeting is needed.  (1) A peer restages its input half only after its own kernel
  // ended, i.e. after every one of its blocks passed the barrier above, which every reader of its
  // input passed too; the restage covers [0, n') of the input half and never the reduced half.
  // (2) A peer's block b' writes its next reduced chunk only after the next call's start barrier
  // for b', which needs this rank's next kernel to be running, i.e. this kernel (all of its
  // gathering) to have ended: launches on one stream do not overlap.
  if (threadIdx.x == 0) self->epoch[blockIdx.x] = epoch;
}


// One-shot all-reduce fused with the residual add + RMSNorm that follows every row-parallel
// projection in a decoder layer: per token row,
//   a = bf16(sum over ranks of the staged inputs)        (what ar_one_shot would write)
//   res <- bf16(a + res) ; x <- bf16(rmsnorm(res) * w)    (ops.fused_add_rmsnorm semantics)
// Block b of every rank handles rows b, b + grid, ... (the per-block barrier pairs them), one
// 512-lane pass per row with VPT 16-byte vectors per lane (H <= 512 * 8 * VPT).
template <int W, int VPT>
__global__ __launch_bounds__(kThreads) void ar_one_shot_add_rmsnorm(Peers P, int rank, int rows, int H,
                                                                    const u32x4* __restrict__ src,
                                                                    u32x4* __restrict__ x, u32x4* __restrict__ res,
                                                                    const u32x4* __restrict__ w, float eps) {
  __shared__ uint32_t s_epoch;
  __shared__ float red[kThreads / 64];
  Signal* self = P.sig[rank];
  if (threadIdx.x == 0) s_epoch = self->epoch[blockIdx.x] + 1;
  const int hv = H >> 3;
  if (src != nullptr) {   // stage this block's rows (the rows block b of every rank reduces)
    u32x4* mine = reinterpret_cast<u32x4*>(P.data[rank]);
    for (int row = blockIdx.x; row < rows; row += gridDim.x)
      for (int i = threadIdx.x; i < hv; i += kThreads) mine[(int64_t)row * hv + i] = src[(int64_t)row * hv + i];
  }
  __syncthreads();
  const uint32_t epoch = s_epoch;
  block_barrier(P, rank, W, epoch, 0);
  for (int row = blockIdx.x; row < rows; row += gridDim.x) {
    float v[VPT][8];
    float ss = 0.f;
#pragma unroll
    for (int c = 0; c < VPT; ++c) {
      const int i = threadIdx.x + c * kThreads;
      if (i < hv) {
        const int64_t e = (int64_t)row * hv + i;
        float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        u32x4 in[W];
#pragma unroll
        for (int r = 0; r < W; ++r) in[r] = reinterpret_cast<const u32x4*>(P.data[(rank + r) % W])[e];
#pragma unroll
        for (int r = 0; r < W; ++r) add8(acc, in[r]);
        const u32x4 a = pack8(acc);   // the all-reduce result, rounded to bf16
        float fa[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        add8(fa, a);
        add8(fa, res[e]);
        const u32x4 sres = pack8(fa);  // residual stream stays bf16
        res[e] = sres;
        float fs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        add8(fs, sres);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          v[c][j] = fs[j];
          ss += fs[j] * fs[j];
        }
      }
    }
    // block reduction of the row's sum of squares
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
    __syncthreads();
    float tot = 0.f;
#pragma unroll
    for (int k = 0; k < kThreads / 64; ++k) tot += red[k];
    __syncthreads();
    const float rs = rsqrtf(tot / (float)H + eps);
#pragma unroll
    for (int c = 0; c < VPT; ++c) {
      const int i = threadIdx.x + c * kThreads;
      if (i < hv) {
        float fw[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        add8(fw, w[i]);
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = v[c][j] * rs * fw[j];
        x[(int64_t)row * hv + i] = pack8(o);
      }
    }
  }
  block_barrier(P, rank, W, epoch, 1);  // nobody may restage its buffer while a peer still reads it
  if (threadIdx.x == 0) self->epoch[blockIdx.x] = epoch;
}

// All-gather along the last dim: every rank stages in[rows][cols] (its own slice, written into its
// IPC buffer by this kernel), out[rows][W * cols] = concat over ranks (rank-major per row), the
// layout of torch.cat(parts, dim=-1) for vocab-parallel logits.  Block b stages and gathers the
// same vector indices on every rank, so the per-block barrier orders each hand-off.
template <int W>
__global__ __launch_bounds__(kThreads) void ag_one_shot(Peers P, int rank, const u32x4* __restrict__ in,
                                                       int64_t rows, int64_t cvec, u32x4* __restrict__ out) {
  __shared__ uint32_t s_epoch;
  Signal* self = P.sig[rank];
  if (threadIdx.x == 0) s_epoch = self->epoch[blockIdx.x] + 1;
  __syncthreads();
  const uint32_t epoch = s_epoch;
  const int64_t n = rows * cvec;
  u32x4* mine = reinterpret_cast<u32x4*>(P.data[rank]);
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads) {
    const u32x4 v = in[i];
    mine[i] = v;
    const int64_t r = i / cvec, c = i - r * cvec;
    out[r * (W * cvec) + rank * cvec + c] = v;
  }
  block_barrier(P, rank, W, epoch, 0);
  for (int q = 1; q < W; ++q) {
    const int src = (rank + q) % W;
    const u32x4* theirs = reinterpret_cast<const u32x4*>(P.data[src]);
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads) {
      const int64_t r = i / cvec, c = i - r * cvec;
      out[r * (W * cvec) + src * cvec + c] = theirs[i];
    }
  }
  block_barrier(P, rank, W, epoch, 1);
  if (threadIdx.x == 0) self->epoch[blockIdx.x] = epoch;
}

struct Ctx {
  int rank, world;
  size_t data_bytes;
  Signal* sig;
  char* data;
  Peers peers;
  bool opened[kMaxRanks];
  uint32_t* host_ctl;   // host-mapped: [0] error mirror, [1] fault stall iterations
};

}  // namespace

// allocate this rank's signal + data buffers; returns the two IPC handles (64 bytes each)
// OME_COMM_FINEGRAINED=1: IPC-shared data buffers allocated fine-grained (docs/COHERENCE.md)
static bool comm_finegrained() {
  static const bool f = getenv("OME_COMM_FINEGRAINED") && atoi(getenv("OME_COMM_FINEGRAINED")) != 0;
  return f;
}

OME_API int ome_comm_create(int rank, int world, size_t data_bytes, void** ctx_out, void* sig_handle,
                            void* data_handle) {
  if (world < 2 || world > kMaxRanks || rank < 0 || rank >= world) return -2;
  Ctx* c = new Ctx();
  memset(c, 0, sizeof(Ctx));
  c->rank = rank;
  c->world = world;
  c->data_bytes = data_bytes;
  hipError_t e = hipExtMallocWithFlags((void**)&c->sig, sizeof(Signal), hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  e = hipMemset(c->sig, 0, sizeof(Signal));
  if (e != hipSuccess) return (int)e;
  data_bytes = (data_bytes + 15) & ~(size_t)15;
  c->data_bytes = data_bytes;
  // input half + reduced-chunk half at +data_bytes; OME_COMM_FINEGRAINED=1: fine-grained (coherent
  // peer access without relying on the system-scope write-back / invalidate, docs/COHERENCE.md)
  e = comm_finegrained() ? hipExtMallocWithFlags((void**)&c->data, 2 * data_bytes, hipDeviceMallocFinegrained)
                         : hipMalloc((void**)&c->data, 2 * data_bytes);
  if (e != hipSuccess) return (int)e;
  e = hipIpcGetMemHandle((hipIpcMemHandle_t*)sig_handle, c->sig);
  if (e != hipSuccess) return (int)e;
  e = hipIpcGetMemHandle((hipIpcMemHandle_t*)data_handle, c->data);
  if (e != hipSuccess) return (int)e;
  c->peers.sig[rank] = c->sig;
  c->peers.data[rank] = c->data;
  const char* sl = getenv("OME_COMM_SPIN_LIMIT");
  c->peers.spin_limit = sl && atoll(sl) > 0 ? (uint64_t)atoll(sl) : kSpinLimitDefault;
  e = hipHostMalloc((void**)&c->host_ctl, 64, hipHostMallocMapped | hipHostMallocCoherent);
  if (e != hipSuccess) return (int)e;
  memset(c->host_ctl, 0, 64);
  uint32_t* dctl = nullptr;
  e = hipHostGetDevicePointer((void**)&dctl, c->host_ctl, 0);
  if (e != hipSuccess) return (int)e;
  c->peers.host_err = dctl;
  c->peers.fault = getenv("OME_COMM_FAULT") ? dctl + 1 : nullptr;
  *ctx_out = c;
  return 0;
}

// host-side error word (set by the kernels when a bounded wait expires): no HIP call, safe to poll
// from a watchdog thread while the GPU is busy
OME_API int ome_comm_host_error(void* ctx) {
  Ctx* c = (Ctx*)ctx;
  return (int)__atomic_load_n(&c->host_ctl[0], __ATOMIC_ACQUIRE);
}

// fault injection (OME_COMM_FAULT set at create time): the flag lanes of every following barrier
// sleep `stall` x s_sleep(127) before publishing (0 = off); -1 when injection is not enabled
OME_API int ome_comm_set_fault(void* ctx, uint32_t stall) {
  Ctx* c = (Ctx*)ctx;
  if (!c->peers.fault) return -1;
  __atomic_store_n(&c->host_ctl[1], stall, __ATOMIC_RELEASE);
  return 0;
}

OME_API int ome_comm_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }

// map every peer's buffers (handles: world x handle_size bytes each, own entries ignored)
OME_API int ome_comm_open(void* ctx, const void* sig_handles, const void* data_handles) {
  Ctx* c = (Ctx*)ctx;
  const size_t hs = sizeof(hipIpcMemHandle_t);
  for (int r = 0; r < c->world; ++r) {
    if (r == c->rank) continue;
    hipIpcMemHandle_t hsig, hdat;
    memcpy(&hsig, (const char*)sig_handles + r * hs, hs);
    memcpy(&hdat, (const char*)data_handles + r * hs, hs);
    void* p = nullptr;
    hipError_t e = hipIpcOpenMemHandle(&p, hsig, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) return (int)e;
    c->peers.sig[r] = (Signal*)p;
    e = hipIpcOpenMemHandle(&p, hdat, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) return (int)e;
    c->peers.data[r] = (char*)p;
    c->opened[r] = true;
  }
  return 0;
}

// in-place-safe bf16 sum: out = sum over ranks of `in` (n elements, n % 8 == 0)
OME_API int ome_comm_all_reduce(void* ctx, const void* in, void* out, int64_t n, int two_shot, int blocks,
                                hipStream_t stream) {
  Ctx* c = (Ctx*)ctx;
  if (n % 8) return -2;
  const size_t bytes = (size_t)n * 2;
  if (bytes > c->data_bytes) return -3;
  if (blocks <= 0 || blocks > kMaxBlocks) blocks = kMaxBlocks;
  hipError_t e = hipSuccess;
  // callers that produced the input straight into the IPC buffer skip the staging pass
  const u32x4* src = in != c->data ? (const u32x4*)in : nullptr;
  // one-shot: peers read every index of this rank's IPC buffer while the kernel writes `out`;
  // an output inside that buffer could be re-read (already reduced) by a slower peer
  if (!two_shot && (const char*)out < (const char*)c->data + c->data_bytes &&
      (const char*)out + bytes > (const char*)c->data)
    return -4;
  const int64_t n_vec = n / 8;
  const int64_t red_vec = (int64_t)(c->data_bytes / 16);
  dim3 grid(blocks), block(kThreads);
#define OME_AR_CASE(W)                                                                               \
  case W:                                                                                            \
    if (two_shot)                                                                                    \
      ar_two_shot<W><<<grid, block, 0, stream>>>(c->peers, c->rank, n_vec, red_vec, src, (u32x4*)out); \
    else                                                                                               \
      ar_one_shot<W><<<grid, block, 0, stream>>>(c->peers, c->rank, n_vec, src, (u32x4*)out);          \
    break;
  switch (c->world) {
    OME_AR_CASE(2)
    OME_AR_CASE(4)
    OME_AR_CASE(8)
    default:
      return -2;
  }
#undef OME_AR_CASE
  e = hipGetLastError();
  return (int)e;
}

// base address of this rank's IPC input buffer (callers may produce an all-reduce input into it)
OME_API void* ome_comm_buffer(void* ctx) { return ((Ctx*)ctx)->data; }

// x, res: [rows][H] bf16 (contiguous); the reduced input is the staged buffer (`in`, copied into
// the IPC buffer unless it already is it).  res <- bf16(allreduce(in) + res); x <- rmsnorm(res) * w
OME_API int ome_comm_all_reduce_add_rmsnorm(void* ctx, const void* in, void* x, void* res, const void* w,
                                            int rows, int H, float eps, int blocks, hipStream_t stream) {
  Ctx* c = (Ctx*)ctx;
  if (H % 8 || rows <= 0) return rows == 0 ? 0 : -2;
  const size_t bytes = (size_t)rows * H * 2;
  if (bytes > c->data_bytes) return -3;
  const int vpt = (H / 8 + kThreads - 1) / kThreads;
  if (vpt > 4) return -2;
  if (blocks <= 0 || blocks > kMaxBlocks) blocks = kMaxBlocks;
  if (blocks > rows) blocks = rows;
  const u32x4* src = in != c->data ? (const u32x4*)in : nullptr;   // staged in-kernel unless produced there
  dim3 grid(blocks), block(kThreads);
#define OME_ARN_CASE(W, V)                                                                                 \
  if (c->world == W && vpt <= V && vpt > V / 2) {                                                         \
    ar_one_shot_add_rmsnorm<W, V><<<grid, block, 0, stream>>>(c->peers, c->rank, rows, H, src, (u32x4*)x,  \
                                                              (u32x4*)res, (const u32x4*)w, eps);         \
    return (int)hipGetLastError();                                                                         \
  }
#define OME_ARN_W(W) OME_ARN_CASE(W, 1) OME_ARN_CASE(W, 2) OME_ARN_CASE(W, 4)
  OME_ARN_W(2)
  OME_ARN_W(4)
  OME_ARN_W(8)
#undef OME_ARN_W
#undef OME_ARN_CASE
  return -2;
}

// out[rows][world * cols] = concat over ranks of in[rows][cols] (bf16/fp16, cols * 2 % 16 == 0)
OME_API int ome_comm_all_gather(void* ctx, const void* in, void* out, int64_t rows, int64_t cols, int blocks,
                                hipStream_t stream) {
  Ctx* c = (Ctx*)ctx;
  if ((cols * 2) % 16 || rows < 0) return -2;
  if ((size_t)rows * cols * 2 > c->data_bytes) return -3;
  if (rows == 0) return 0;
  if (blocks <= 0 || blocks > kMaxBlocks) blocks = kMaxBlocks;
  const int64_t cvec = cols * 2 / 16;
  dim3 grid(blocks), block(kThreads);
  switch (c->world) {
    case 2: ag_one_shot<2><<<grid, block, 0, stream>>>(c->peers, c->rank, (const u32x4*)in, rows, cvec, (u32x4*)out); break;
    case 4: ag_one_shot<4><<<grid, block, 0, stream>>>(c->peers, c->rank, (const u32x4*)in, rows, cvec, (u32x4*)out); break;
    case 8: ag_one_shot<8><<<grid, block, 0, stream>>>(c->peers, c->rank, (const u32x4*)in, rows, cvec, (u32x4*)out); break;
    default: return -2;
  }
  return (int)hipGetLastError();
}

OME_API int ome_comm_error(void* ctx) {
  Ctx* c = (Ctx*)ctx;
  uint32_t err = 0;
  if (hipMemcpy(&err, &c->sig->error, sizeof(err), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return (int)err;
}

OME_API void ome_comm_destroy(void* ctx) {
  Ctx* c = (Ctx*)ctx;
  if (!c) return;
  if (c->host_ctl) (void)hipHostFree(c->host_ctl);
  for (int r = 0; r < c->world; ++r) {
    if (c->opened[r]) {
      (void)hipIpcCloseMemHandle(c->peers.sig[r]);
      (void)hipIpcCloseMemHandle(c->peers.data[r]);
    }
  }
  (void)hipFree(c->sig);
  (void)hipFree(c->data);
  delete c;
}
