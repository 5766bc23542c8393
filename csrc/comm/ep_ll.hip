// Low-latency expert-parallel dispatch / combine over xGMI peer mappings (SURVEY.md §2.9 K17,
// the DeepEP `low_latency` mode of the reference's DeepSeek runtimes,
// config/runtimes/srt/deepseek-rdma-pd-rt.yaml:83-126).  Everything stays on the device -- no
// per-layer split counts travel to the host -- so a decode step's MoE layers can be captured in a
// HIP graph.
//
// Pull protocol (every buffer is written only by its owner; peers read it over xGMI after a
// system-scope release / acquire on a flag, the pattern of csrc/comm/allreduce.hip):
//   begin    : epoch += 1 (device counter; parity p = epoch & 1 selects one of two buffer sets,
//              so the next layer's writes never touch what a slow peer may still be reading);
//   plan     : each (token, k-slot) assignment -> (owner rank, slot in the owner's bucket);
//   pack     : rows into MY send buffer S[p][dst][slot] (+ local expert id, bucket counts);
//              every storing workgroup writes its XCD's L2 back (system release);
//   signal/wait (dispatch flags);
//   pull     : rows the peers packed for me -> my receive buffer R[src][slot] (remote reads);
//   (experts run on R with the grouped GEMM, rows of empty slots carry the null expert id);
//   comb_pack: expert outputs -> MY combine buffer C[p][src][slot], released;
//   signal/wait (combine flags);
//   comb_pull: out[t] = scale * sum_j w[t, j] * C_of_owner(t, j)[p][me][slot(t, j)]  (fp32).
// Bounded spins record an error word instead of hanging the GPU.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define OME_API extern "C" __attribute__((visibility("default")))

namespace {

constexpr int kMaxRanks = 8;
constexpr uint64_t kSpinLimitDefault = 1ull << 26;
typedef __bf16 bf16;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct EpSig {
  uint32_t ready[2][kMaxRanks];  // [dispatch / combine][peer] = last epoch that peer published
  uint32_t epoch;
  uint32_t error;
  uint32_t done[2];              // fused kernels: finished workgroups of the current send / comb_send
  int scnt[kMaxRanks];           // fused send: rows bucketed per owner so far (reset by the last block)
};

struct EpPeers {
  EpSig* sig[kMaxRanks];
  char* buf[kMaxRanks];  // each rank's shared buffer (layout below)
  // fault handling, as in allreduce.hip: bounded waits (OME_COMM_SPIN_LIMIT), host-mapped error
  // mirror, optional stall-before-publish word (OME_COMM_FAULT)
  uint64_t spin_limit;
  uint32_t* host_err;
  const uint32_t* fault;
};

__device__ __forceinline__ void ep_fault_stall(const EpPeers& P) {
  if (P.fault) {
    const uint32_t n = __hip_atomic_load(P.fault, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    for (uint32_t i = 0; i < n; ++i) __builtin_amdgcn_s_sleep(127);
  }
}

// shared buffer layout (bytes), per parity p:  S rows [W][cap][H] bf16 | S ids [W][cap] i32 |
// S counts [W] i32 (padded to 256 B) | C rows [W][cap][H] bf16
struct Layout {
  int64_t rows, ids, counts, comb, per_parity;
  __host__ __device__ Layout(int W, int cap, int H) {
    rows = (int64_t)W * cap * H * 2;
    ids = (int64_t)W * cap * 4;
    counts = 256;
    comb = rows;
    per_parity = rows + ids + counts + comb;
  }
};

__device__ __forceinline__ void st_release_sys(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint32_t ld_acquire_sys(uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// the storing workgroup publishes its writes past its XCD's L2 (peers read HBM over xGMI)
__device__ __forceinline__ void block_release() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_system();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

__global__ void ep_begin_kernel(EpSig* self) {
  if (threadIdx.x == 0) self->epoch = self->epoch + 1;
}

// one workgroup: assignment a = t * k + j -> (owner, slot, owner-local expert slot); counts per
// owner in MY S[p] counts.  Without EPLB tables rank r owns experts [r * e_local, (r+1) * e_local);
// with them (rep_rank / rep_slot [E][rmax], n_rep [E], ome_amd.parallel.eplb) the assignment goes
// to replica (a mod n_rep[e]) of its expert, as in the normal-mode all-to-all.
__global__ __launch_bounds__(1024) void ep_plan_kernel(const int* __restrict__ topk_ids, int n, int e_local, int W,
                                                       int n_experts, int cap, int* __restrict__ a_dst,
                                                       int* __restrict__ a_slot,
                                                       int* __restrict__ a_local, const int64_t* __restrict__ rep_rank,
                                                       const int64_t* __restrict__ rep_slot,
                                                       const int64_t* __restrict__ n_rep, int rmax, EpSig* self,
                                                       char* mybuf, Layout L) {
  __shared__ int cnt[kMaxRanks];
  if (threadIdx.x < kMaxRanks) cnt[threadIdx.x] = 0;
  __syncthreads();
  for (int a = threadIdx.x; a < n; a += blockDim.x) {
    int id = topk_ids[a];
    id = id < 0 ? 0 : (id < n_experts ? id : n_experts - 1);   // never index tables / peers out of range
    int dst, loc;
    if (rep_rank != nullptr) {
      const int nr = (int)n_rep[id];
      const int j = nr > 0 ? a % nr : 0;
      dst = (int)rep_rank[(int64_t)id * rmax + j];
      loc = (int)rep_slot[(int64_t)id * rmax + j];
    } else {
      dst = id / e_local;
      loc = id - dst * e_local;
    }
    dst = dst < 0 ? 0 : (dst < W ? dst : W - 1);
    loc = loc < 0 ? 0 : (loc < e_local ? loc : e_local - 1);
    const int slot = atomicAdd(&cnt[dst], 1);
    a_dst[a] = dst;
    a_local[a] = loc;
    a_slot[a] = slot < cap ? slot : -1;  // over capacity: dropped (recorded below)
  }
  __syncthreads();
  const int par = self->epoch & 1;
  int* counts = (int*)(mybuf + par * L.per_parity + L.rows + L.ids);
  if (threadIdx.x < W) {
    const int c = cnt[threadIdx.x];
    counts[threadIdx.x] = c < cap ? c : cap;
    if (c > cap) atomicOr(&self->error, 2u);
  }
}

// grid = assignments; row x[a / k] -> S[p][dst][slot], id -> S ids
__global__ __launch_bounds__(256) void ep_pack_kernel(const bf16* __restrict__ x, int64_t ldx, int H, int k,
                                                      const int* __restrict__ a_local,
                                                      const int* __restrict__ a_dst, const int* __restrict__ a_slot,
                                                      int cap, const EpSig* self, char* mybuf, Layout L) {
  const int a = blockIdx.x;
  const int slot = a_slot[a], dst = a_dst[a];
  const int par = self->epoch & 1;
  if (slot >= 0) {
    char* base = mybuf + par * L.per_parity;
    const u32x4* src = reinterpret_cast<const u32x4*>(x + (int64_t)(a / k) * ldx);
    u32x4* dstp = reinterpret_cast<u32x4*>(base + ((int64_t)dst * cap + slot) * H * 2);
    for (int v = threadIdx.x; v < H / 8; v += blockDim.x) dstp[v] = src[v];
    if (threadIdx.x == 0) reinterpret_cast<int*>(base + L.rows)[dst * cap + slot] = a_local[a];
  }
  block_release();
}

// thread p < W: publish the current epoch on peer p's flag `which` for me
__global__ void ep_signal_kernel(EpPeers P, int me, int W, int which, EpSig* self) {
  const uint32_t e = self->epoch;
  if ((int)threadIdx.x < W) {
    ep_fault_stall(P);
    __threadfence_system();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    st_release_sys(&P.sig[threadIdx.x]->ready[which][me], e);
  }
}

__global__ void ep_wait_kernel(EpPeers P, EpSig* self, int W, int which) {
  const uint32_t e = self->epoch;
  if ((int)threadIdx.x < W) {
    uint64_t spins = 0;
    while (ld_acquire_sys(&self->ready[which][threadIdx.x]) < e) {
      if (++spins > P.spin_limit) {
        atomicOr(&self->error, 1u);
        if (P.host_err) __hip_atomic_store(P.host_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

// grid (cap, W): row (src, slot) of my receive buffer R [W][cap][H] <- peer src's S[p][me][slot];
// rids[src * cap + slot] = its local expert id, or e_local (the null expert) past the count
__global__ __launch_bounds__(256) void ep_pull_kernel(EpPeers P, int me, int H, int cap, int e_local, Layout L,
                                                      const EpSig* self, bf16* __restrict__ R, int* __restrict__ rids,
                                                      int* __restrict__ rcount) {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  const int slot = blockIdx.x, src = blockIdx.y;
  const int par = self->epoch & 1;
  const char* base = P.buf[src] + par * L.per_parity;
  const int count = reinterpret_cast<const int*>(base + L.rows + L.ids)[me];
  if (slot == 0 && threadIdx.x == 0) rcount[src] = count;
  if (slot >= count) {
    if (threadIdx.x == 0) rids[src * cap + slot] = e_local;
    return;
  }
  const u32x4* s = reinterpret_cast<const u32x4*>(base + ((int64_t)me * cap + slot) * H * 2);
  u32x4* d = reinterpret_cast<u32x4*>(R + ((int64_t)src * cap + slot) * H);
  for (int v = threadIdx.x; v < H / 8; v += blockDim.x) d[v] = s[v];
  if (threadIdx.x == 0) rids[src * cap + slot] = reinterpret_cast<const int*>(base + L.rows)[me * cap + slot];
}

// grid (cap, W): expert output of received row (src, slot) -- y_sorted[inv[src * cap + slot]] --
// into MY combine buffer C[p][src][slot]; released for the pulling sources
__global__ __launch_bounds__(256) void ep_comb_pack_kernel(const bf16* __restrict__ y_sorted, const int* __restrict__ inv,
                                                           const int* __restrict__ rcount, int H, int cap, Layout L,
                                                           const EpSig* self, char* mybuf) {
  const int slot = blockIdx.x, src = blockIdx.y;
  if (slot < rcount[src]) {
    const int par = self->epoch & 1;
    char* base = mybuf + par * L.per_parity + L.rows + L.ids + L.counts;
    const u32x4* s = reinterpret_cast<const u32x4*>(y_sorted + (int64_t)inv[src * cap + slot] * H);
    u32x4* d = reinterpret_cast<u32x4*>(base + ((int64_t)src * cap + slot) * H * 2);
    for (int v = threadIdx.x; v < H / 8; v += blockDim.x) d[v] = s[v];
  }
  block_release();
}

__device__ __forceinline__ void add8(float* acc, u32x4 v, float w) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    acc[2 * i] += w * __uint_as_float(v[i] << 16);
    acc[2 * i + 1] += w * __uint_as_float(v[i] & 0xffff0000u);
  }
}

// grid = tokens: out[t] = scale * sum_j w[t, j] * (owner(t, j)'s C[p][me][slot(t, j)])
__global__ __launch_bounds__(256) void ep_comb_pull_kernel(EpPeers P, int me, int H, int k, int cap, Layout L,
                                                           const EpSig* self, const float* __restrict__ topk_w,
                                                           const int* __restrict__ a_dst,
                                                           const int* __restrict__ a_slot, float scale,
                                                           bf16* __restrict__ out, int64_t ldo) {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  const int t = blockIdx.x;
  const int par = self->epoch & 1;
  for (int v = threadIdx.x; v < H / 8; v += blockDim.x) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < k; ++j) {
      const int a = t * k + j, slot = a_slot[a];
      if (slot < 0) continue;
      const char* base = P.buf[a_dst[a]] + par * L.per_parity + L.rows + L.ids + L.counts;
      add8(acc, reinterpret_cast<const u32x4*>(base + ((int64_t)me * cap + slot) * H * 2)[v], topk_w[a]);
    }
    u32x4 r;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bf16 lo = (bf16)(acc[2 * i] * scale), hi = (bf16)(acc[2 * i + 1] * scale);
      r[i] = (uint32_t)__builtin_bit_cast(uint16_t, lo) | ((uint32_t)__builtin_bit_cast(uint16_t, hi) << 16);
    }
    reinterpret_cast<u32x4*>(out + (int64_t)t * ldo)[v] = r;
  }
}

// ------------------------------------------------------------------------------------------
// Fused path (default): 4 launches per MoE layer instead of 10.
//   send      (grid = assignments): plan + pack in one pass -- each workgroup buckets its
//             assignment with an atomic on MY per-owner counter, packs the row into S[p][dst][slot],
//             releases; the LAST workgroup (done counter) publishes the counts, resets the
//             counters, advances the epoch and raises my dispatch flag on every peer.
//   recv      (grid G x W): per source, wait for its flag, then copy only the rows it actually
//             sent (slot loop bounded by its count, not the capacity) and mark the rest empty.
//   comb_send (grid G x W): expert outputs of the received rows -> MY C[p][src][slot]; the last
//             workgroup raises my combine flag on every peer.
//   comb_recv (grid = tokens): wait for every owner's combine flag, weighted sum (fp32).
// The counters / done words live in the uncached signal page; the data buffers keep the
// owner-writes / peers-read protocol of the unfused kernels above.
// ------------------------------------------------------------------------------------------
constexpr int kRecvBlocks = 32;
// largest grid whose every workgroup may spin on the peer flags itself (decode-sized token
// counts: saves the separate wait launch); larger grids wait in one 64-thread ep_wait_kernel
constexpr int kSpinMaxBlocks = 64;

__device__ __forceinline__ bool last_block(uint32_t* done) {
  __shared__ int last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_system();   // this block's stores are visible system-wide before it counts
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = atomicAdd(done, 1u) == gridDim.x * gridDim.y - 1;
  }
  __syncthreads();
  return last != 0;
}

__device__ __forceinline__ void spin_flag(const EpPeers& P, EpSig* self, int which, int src, uint32_t e) {
  uint64_t spins = 0;
  while (ld_acquire_sys(&self->ready[which][src]) < e) {
    if (++spins > P.spin_limit) {
      atomicOr(&self->error, 1u);
      if (P.host_err) __hip_atomic_store(P.host_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

__global__ __launch_bounds__(256) void ep_send_kernel(EpPeers P, int me, int W, const bf16* __restrict__ x,
                                                      int64_t ldx, int H, int k, const int* __restrict__ topk_ids,
                                                      int n, int e_local, int n_experts, int cap,
                                                      int* __restrict__ a_dst, int* __restrict__ a_slot,
                                                      int* __restrict__ a_local, const int64_t* __restrict__ rep_rank,
                                                      const int64_t* __restrict__ rep_slot,
                                                      const int64_t* __restrict__ n_rep, int rmax, EpSig* self,
                                                      char* mybuf, Layout L) {
  const uint32_t cur = self->epoch + 1;
  const int par = cur & 1;
  const int a = blockIdx.x;
  __shared__ int s_dst, s_slot, s_loc;
  if (a < n && threadIdx.x == 0) {
    int id = topk_ids[a];
    id = id < 0 ? 0 : (id < n_experts ? id : n_experts - 1);
    int dst, loc;
    if (rep_rank != nullptr) {
      const int nr = (int)n_rep[id];
      const int j = nr > 0 ? a % nr : 0;
      dst = (int)rep_rank[(int64_t)id * rmax + j];
      loc = (int)rep_slot[(int64_t)id * rmax + j];
    } else {
      dst = id / e_local;
      loc = id - dst * e_local;
    }
    dst = dst < 0 ? 0 : (dst < W ? dst : W - 1);
    loc = loc < 0 ? 0 : (loc < e_local ? loc : e_local - 1);
    const int slot = atomicAdd(&self->scnt[dst], 1);
    a_dst[a] = dst;
    a_local[a] = loc;
    a_slot[a] = slot < cap ? slot : -1;
    s_dst = dst;
    s_slot = slot < cap ? slot : -1;
    s_loc = loc;
  }
  __syncthreads();
  if (a < n && s_slot >= 0) {
    char* base = mybuf + par * L.per_parity;
    const u32x4* src = reinterpret_cast<const u32x4*>(x + (int64_t)(a / k) * ldx);
    u32x4* dstp = reinterpret_cast<u32x4*>(base + ((int64_t)s_dst * cap + s_slot) * H * 2);
    for (int v = threadIdx.x; v < H / 8; v += blockDim.x) dstp[v] = src[v];
    if (threadIdx.x == 0) reinterpret_cast<int*>(base + L.rows)[s_dst * cap + s_slot] = s_loc;
  }
  if (!last_block(&self->done[0])) return;
  // last workgroup: every row of this epoch is packed and released
  int* counts = (int*)(mybuf + par * L.per_parity + L.rows + L.ids);
  if ((int)threadIdx.x < W) {
    const int c = atomicExch(&self->scnt[threadIdx.x], 0);
    counts[threadIdx.x] = c < cap ? c : cap;
    if (c > cap) atomicOr(&self->error, 2u);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    self->done[0] = 0;
    self->epoch = cur;
    __threadfence_system();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if ((int)threadIdx.x < W) {
    ep_fault_stall(P);
    st_release_sys(&P.sig[threadIdx.x]->ready[0][me], cur);
  }
}

// grid (kRecvBlocks, W): rows source `src` sent me, R [W][cap][H]; rids past the count = e_local
__global__ __launch_bounds__(256) void ep_recv_kernel(EpPeers P, int me, int H, int cap, int e_local, Layout L,
                                                      EpSig* self, bf16* __restrict__ R, int* __restrict__ rids,
                                                      int* __restrict__ rcount, int spin) {
  const int g = blockIdx.x, src = blockIdx.y;
  const uint32_t cur = self->epoch;
  if (spin && threadIdx.x == 0) spin_flag(P, self, 0, src, cur);
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  const int par = cur & 1;
  const char* base = P.buf[src] + par * L.per_parity;
  const int count = reinterpret_cast<const int*>(base + L.rows + L.ids)[me];
  if (g == 0 && threadIdx.x == 0) rcount[src] = count;
  for (int slot = g; slot < cap; slot += gridDim.x) {
    if (slot >= count) {   // empty slots: ids only (the grouped GEMM skips the null expert)
      for (int s2 = slot + (int)threadIdx.x * gridDim.x; s2 < cap; s2 += blockDim.x * gridDim.x)
        rids[src * cap + s2] = e_local;
      break;
    }
    const u32x4* s = reinterpret_cast<const u32x4*>(base + ((int64_t)me * cap + slot) * H * 2);
    u32x4* d = reinterpret_cast<u32x4*>(R + ((int64_t)src * cap + slot) * H);
    for (int v = threadIdx.x; v < H / 8; v += blockDim.x) d[v] = s[v];
    if (threadIdx.x == 0) rids[src * cap + slot] = reinterpret_cast<const int*>(base + L.rows)[me * cap + slot];
  }
}

// grid (kRecvBlocks, W): expert outputs of the rows src sent me -> MY C[p][src][slot]; the last
// workgroup raises my combine flag on every peer
__global__ __launch_bounds__(256) void ep_comb_send_kernel(EpPeers P, int me, int W, const bf16* __restrict__ y_sorted,
                                                           const int* __restrict__ inv,
                                                           const int* __restrict__ rcount, int H, int cap, Layout L,
                                                           EpSig* self, char* mybuf) {
  const int g = blockIdx.x, src = blockIdx.y;
  const uint32_t cur = self->epoch;
  const int par = cur & 1;
  char* base = mybuf + par * L.per_parity + L.rows + L.ids + L.counts;
  const int count = rcount[src];
  for (int slot = g; slot < count; slot += gridDim.x) {
    const u32x4* s = reinterpret_cast<const u32x4*>(y_sorted + (int64_t)inv[src * cap + slot] * H);
    u32x4* d = reinterpret_cast<u32x4*>(base + ((int64_t)src * cap + slot) * H * 2);
    for (int v = threadIdx.x; v < H / 8; v += blockDim.x) d[v] = s[v];
  }
  if (!last_block(&self->done[1])) return;
  if (threadIdx.x == 0) {
    self->done[1] = 0;
    __threadfence_system();
  }
  __syncthreads();
  if ((int)threadIdx.x < W) {
    ep_fault_stall(P);
    st_release_sys(&P.sig[threadIdx.x]->ready[1][me], cur);
  }
}

// grid = tokens: wait for every owner's combine flag, then the weighted sum of ep_comb_pull_kernel
// spin = 0: the flags were already waited for by ep_wait_kernel on the same stream (grids larger
// than kSpinMaxBlocks: thousands of resident spinning workgroups -- one per token of a prefill
// chunk -- would hold the CUs that the co-scheduled work, e.g. the other two-batch-overlap half or
// a peer process sharing the GPU, needs to make progress; profiles/r06_tbo_trace.md)
__global__ __launch_bounds__(256) void ep_comb_recv_kernel(EpPeers P, int me, int W, int H, int k, int cap, Layout L,
                                                           EpSig* self, const float* __restrict__ topk_w,
                                                           const int* __restrict__ a_dst,
                                                           const int* __restrict__ a_slot, float scale,
                                                           bf16* __restrict__ out, int64_t ldo, int spin) {
  const uint32_t cur = self->epoch;
  if (spin && (int)threadIdx.x < W) spin_flag(P, self, 1, threadIdx.x, cur);
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  const int t = blockIdx.x;
  const int par = cur & 1;
  for (int v = threadIdx.x; v < H / 8; v += blockDim.x) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < k; ++j) {
      const int a = t * k + j, slot = a_slot[a];
      if (slot < 0) continue;
      const char* base = P.buf[a_dst[a]] + par * L.per_parity + L.rows + L.ids + L.counts;
      add8(acc, reinterpret_cast<const u32x4*>(base + ((int64_t)me * cap + slot) * H * 2)[v], topk_w[a]);
    }
    u32x4 r;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bf16 lo = (bf16)(acc[2 * i] * scale), hi = (bf16)(acc[2 * i + 1] * scale);
      r[i] = (uint32_t)__builtin_bit_cast(uint16_t, lo) | ((uint32_t)__builtin_bit_cast(uint16_t, hi) << 16);
    }
    reinterpret_cast<u32x4*>(out + (int64_t)t * ldo)[v] = r;
  }
}

// OME_EP_LL_FUSED=0 selects the 10-launch kernels (A/B timing)
// OME_EP_WAIT_KERNEL=1: every receive waits in one 64-thread kernel (no spinning workgroups in
// the copy kernels; one extra launch per exchange) -- the two-batch-overlap experiment
static bool wait_kernel() {
  static const bool w = [] {
    const char* e = getenv("OME_EP_WAIT_KERNEL");
    return e && atoi(e) == 1;
  }();
  return w;
}

static bool fused() {
  static const bool f = !getenv("OME_EP_LL_FUSED") || atoi(getenv("OME_EP_LL_FUSED")) != 0;
  return f;
}

struct EpCtx {
  int rank, world, cap, H;
  EpSig* sig;
  char* buf;
  Layout L;
  EpPeers peers;
  bool opened[kMaxRanks];
  uint32_t* host_ctl;   // host-mapped: [0] error mirror, [1] fault stall iterations
};

}  // namespace

// OME_COMM_FINEGRAINED=1: IPC-shared data buffers allocated fine-grained (docs/COHERENCE.md)
static bool comm_finegrained() {
  static const bool f = getenv("OME_COMM_FINEGRAINED") && atoi(getenv("OME_COMM_FINEGRAINED")) != 0;
  return f;
}

OME_API int ome_ep_create(int rank, int world, int cap, int H, void** ctx_out, void* sig_handle, void* buf_handle) {
  if (world < 2 || world > kMaxRanks || rank < 0 || rank >= world || H % 8 || cap <= 0) return -2;
  EpCtx* c = new EpCtx{rank, world, cap, H, nullptr, nullptr, Layout(world, cap, H), {}, {}, nullptr};
  hipError_t e = hipExtMallocWithFlags((void**)&c->sig, sizeof(EpSig), hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  if ((e = hipMemset(c->sig, 0, sizeof(EpSig))) != hipSuccess) return (int)e;
  e = comm_finegrained() ? hipExtMallocWithFlags((void**)&c->buf, 2 * c->L.per_parity, hipDeviceMallocFinegrained)
                         : hipMalloc((void**)&c->buf, 2 * c->L.per_parity);   // docs/COHERENCE.md
  if (e != hipSuccess) return (int)e;
  if ((e = hipMemset(c->buf, 0, 2 * c->L.per_parity)) != hipSuccess) return (int)e;
  if ((e = hipIpcGetMemHandle((hipIpcMemHandle_t*)sig_handle, c->sig)) != hipSuccess) return (int)e;
  if ((e = hipIpcGetMemHandle((hipIpcMemHandle_t*)buf_handle, c->buf)) != hipSuccess) return (int)e;
  c->peers.sig[rank] = c->sig;
  c->peers.buf[rank] = c->buf;
  const char* sl = getenv("OME_COMM_SPIN_LIMIT");
  c->peers.spin_limit = sl && atoll(sl) > 0 ? (uint64_t)atoll(sl) : kSpinLimitDefault;
  if ((e = hipHostMalloc((void**)&c->host_ctl, 64, hipHostMallocMapped | hipHostMallocCoherent)) != hipSuccess)
    return (int)e;
  memset(c->host_ctl, 0, 64);
  uint32_t* dctl = nullptr;
  if ((e = hipHostGetDevicePointer((void**)&dctl, c->host_ctl, 0)) != hipSuccess) return (int)e;
  c->peers.host_err = dctl;
  c->peers.fault = getenv("OME_COMM_FAULT") ? dctl + 1 : nullptr;
  *ctx_out = c;
  return 0;
}

OME_API int ome_ep_host_error(void* ctx) {
  EpCtx* c = (EpCtx*)ctx;
  return (int)__atomic_load_n(&c->host_ctl[0], __ATOMIC_ACQUIRE);
}

OME_API int ome_ep_set_fault(void* ctx, uint32_t stall) {
  EpCtx* c = (EpCtx*)ctx;
  if (!c->peers.fault) return -1;
  __atomic_store_n(&c->host_ctl[1], stall, __ATOMIC_RELEASE);
  return 0;
}

OME_API int ome_ep_open(void* ctx, const void* sig_handles, const void* buf_handles) {
  EpCtx* c = (EpCtx*)ctx;
  const size_t hs = sizeof(hipIpcMemHandle_t);
  for (int r = 0; r < c->world; ++r) {
    if (r == c->rank) continue;
    hipIpcMemHandle_t hsig, hbuf;
    memcpy(&hsig, (const char*)sig_handles + r * hs, hs);
    memcpy(&hbuf, (const char*)buf_handles + r * hs, hs);
    void* p = nullptr;
    hipError_t e = hipIpcOpenMemHandle(&p, hsig, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) return (int)e;
    c->peers.sig[r] = (EpSig*)p;
    if ((e = hipIpcOpenMemHandle(&p, hbuf, hipIpcMemLazyEnablePeerAccess)) != hipSuccess) return (int)e;
    c->peers.buf[r] = (char*)p;
    c->opened[r] = true;
  }
  return 0;
}

// dispatch: plan + pack + signal + wait + pull.  Outputs (device, caller-allocated): a_dst, a_slot
// [T*k]; R [W*cap][H] received rows, rids [W*cap] local expert ids (e_local = empty slot), rcount [W].
// a_local [T*k] scratch; rep_rank / rep_slot / n_rep: optional EPLB tables (int64, [E][rmax], [E]).
OME_API int ome_ep_dispatch(void* ctx, const void* x, int64_t ldx, const int* topk_ids, int T, int k, int e_local,
                            int n_experts, int* a_dst, int* a_slot, int* a_local, const int64_t* rep_rank,
                            const int64_t* rep_slot, const int64_t* n_rep, int rmax, void* R, int* rids, int* rcount,
                            hipStream_t stream) {
  EpCtx* c = (EpCtx*)ctx;
  const int n = T * k;
  if (e_local <= 0 || n_experts <= 0) return -2;
  if (fused()) {
    ep_send_kernel<<<n > 0 ? n : 1, 256, 0, stream>>>(c->peers, c->rank, c->world, (const bf16*)x, ldx, c->H, k,
                                                      topk_ids, n, e_local, n_experts, c->cap, a_dst, a_slot, a_local,
                                                      rep_rank, rep_slot, n_rep, rmax, c->sig, c->buf, c->L);
    const int spin = !wait_kernel();
    if (!spin) ep_wait_kernel<<<1, 64, 0, stream>>>(c->peers, c->sig, c->world, 0);
    ep_recv_kernel<<<dim3(kRecvBlocks, c->world), 256, 0, stream>>>(c->peers, c->rank, c->H, c->cap, e_local, c->L,
                                                                   c->sig, (bf16*)R, rids, rcount, spin);
    return (int)hipGetLastError();
  }
  ep_begin_kernel<<<1, 64, 0, stream>>>(c->sig);
  ep_plan_kernel<<<1, 1024, 0, stream>>>(topk_ids, n, e_local, c->world, n_experts, c->cap, a_dst, a_slot, a_local,
                                         rep_rank,
                                         rep_slot, n_rep, rmax, c->sig, c->buf, c->L);
  if (n > 0)
    ep_pack_kernel<<<n, 256, 0, stream>>>((const bf16*)x, ldx, c->H, k, a_local, a_dst, a_slot, c->cap, c->sig,
                                          c->buf, c->L);
  ep_signal_kernel<<<1, 64, 0, stream>>>(c->peers, c->rank, c->world, 0, c->sig);
  ep_wait_kernel<<<1, 64, 0, stream>>>(c->peers, c->sig, c->world, 0);
  ep_pull_kernel<<<dim3(c->cap, c->world), 256, 0, stream>>>(c->peers, c->rank, c->H, c->cap, e_local, c->L, c->sig,
                                                            (bf16*)R, rids, rcount);
  return (int)hipGetLastError();
}

// combine: y_sorted [rows][H] expert outputs in the grouped GEMM's sorted order, inv [W*cap] the
// position of received row i in it; out [T][H] = scale * sum_j w * (row of assignment (t, j)).
OME_API int ome_ep_combine(void* ctx, const void* y_sorted, const int* inv, const int* rcount, const float* topk_w,
                           const int* a_dst, const int* a_slot, int T, int k, float scale, void* out, int64_t ldo,
                           hipStream_t stream) {
  EpCtx* c = (EpCtx*)ctx;
  if (fused()) {
    ep_comb_send_kernel<<<dim3(kRecvBlocks, c->world), 256, 0, stream>>>(
        c->peers, c->rank, c->world, (const bf16*)y_sorted, inv, rcount, c->H, c->cap, c->L, c->sig, c->buf);
    if (T > 0) {
      const int spin = T <= kSpinMaxBlocks && !wait_kernel();
      if (!spin) ep_wait_kernel<<<1, 64, 0, stream>>>(c->peers, c->sig, c->world, 1);
      ep_comb_recv_kernel<<<T, 256, 0, stream>>>(c->peers, c->rank, c->world, c->H, k, c->cap, c->L, c->sig, topk_w,
                                                 a_dst, a_slot, scale, (bf16*)out, ldo, spin);
    }
    return (int)hipGetLastError();
  }
  ep_comb_pack_kernel<<<dim3(c->cap, c->world), 256, 0, stream>>>((const bf16*)y_sorted, inv, rcount, c->H, c->cap,
                                                                 c->L, c->sig, c->buf);
  ep_signal_kernel<<<1, 64, 0, stream>>>(c->peers, c->rank, c->world, 1, c->sig);
  ep_wait_kernel<<<1, 64, 0, stream>>>(c->peers, c->sig, c->world, 1);
  if (T > 0)
    ep_comb_pull_kernel<<<T, 256, 0, stream>>>(c->peers, c->rank, c->H, k, c->cap, c->L, c->sig, topk_w, a_dst,
                                               a_slot, scale, (bf16*)out, ldo);
  return (int)hipGetLastError();
}

OME_API int ome_ep_error(void* ctx) {
  EpCtx* c = (EpCtx*)ctx;
  uint32_t err = 0;
  if (hipMemcpy(&err, &c->sig->error, sizeof(err), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return (int)err;
}

OME_API void ome_ep_destroy(void* ctx) {
  EpCtx* c = (EpCtx*)ctx;
  if (!c) return;
  if (c->host_ctl) (void)hipHostFree(c->host_ctl);
  for (int r = 0; r < c->world; ++r)
    if (c->opened[r]) {
      (void)hipIpcCloseMemHandle(c->peers.sig[r]);
      (void)hipIpcCloseMemHandle(c->peers.buf[r]);
    }
  (void)hipFree(c->sig);
  (void)hipFree(c->buf);
  delete c;
}
