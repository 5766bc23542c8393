// Gated DeltaNet (Qwen3-Next linear-attention layers; reference catalog
// ``config/runtimes/srt/Qwen/qwen3-next-80b-a3b-instruct-rt.yaml``) for gfx950.
//
// Per value head h of a sequence, with k-head h / (Hv / Hk), L2-normalised q, k (q also scaled
// by 1/sqrt(dk)), g = -exp(A_log[h]) * softplus(a + dt_bias[h]), beta = sigmoid(b):
//   S <- exp(g) * S
//   S <- S + k (beta * (v - S^T k))^T          (the delta rule: a rank-1 correction)
//   o  = S^T q
// S is fp32 per (slot, head), stored TRANSPOSED as [dv, dk] (each state column contiguous),
// continued across prefill chunks and decode steps (the runner's per-request state slots;
// ``reset`` starts a sequence's first chunk from zero).
//
// One workgroup = (sequence, v-head), dv threads; thread j keeps column S[:, j] (dk fp32 values)
// in VGPRs for the whole sequence, so S^T k and S^T q are in-lane dot products and the update is
// in-lane FMAs -- no cross-lane reduction in the time loop.  Per row the block normalises q and k
// (one wave, shuffle reduction) into a double-buffered LDS slot that every lane then reads as a
// broadcast; one barrier per row.  Recurrent form: the chunked (WY) form for long prefills is a
// later optimisation; decode rows are the same launch with one row per sequence.
#include "common.h"

#include <cstdlib>

namespace {

__device__ __forceinline__ float gdn_softplus(float x) { return x > 20.f ? x : log1pf(__expf(x)); }

template <int DK>
__global__ __launch_bounds__(128) void gdn_scan_kernel(
    const bf16* __restrict__ q, const bf16* __restrict__ k, const bf16* __restrict__ v, int64_t qkv_stride,
    const bf16* __restrict__ a, const bf16* __restrict__ b, int64_t ab_stride, const float* __restrict__ A_log,
    const float* __restrict__ dt_bias, float* __restrict__ state, bf16* __restrict__ out, int64_t out_stride,
    const int* __restrict__ cu, const int* __restrict__ slot, const int* __restrict__ reset, int Hv, int Hk,
    int dv) {
  __shared__ float s_qk[2][2][DK];   // [buffer][q | k][DK]
  __shared__ float s_gb[2][2];       // [buffer][decay | beta]
  const int s = blockIdx.x, h = blockIdx.y, j = threadIdx.x;
  const int r0 = cu[s], r1 = cu[s + 1];
  if (r1 <= r0) return;   // uniform per block
  const int hk = h / (Hv / Hk);
  float* st = state + ((int64_t)slot[s] * Hv + h) * DK * dv;
  const bool fresh = reset[s] != 0;
  float S[DK];
#pragma unroll
  for (int i = 0; i < DK; ++i) S[i] = (fresh || j >= dv) ? 0.f : st[(int64_t)j * DK + i];
  const float negA = -__expf(A_log[h]), dtb = dt_bias[h];
  const float qscale = rsqrtf((float)DK);

  // stage row r into buffer p: L2-normalised q (scaled) and k, decay and beta (wave 0)
  auto stage = [&](int r, int p) {
    if (j < 64) {
      constexpr int PER = DK / 64;
      float qv[PER], kv[PER], sq = 0.f, sk = 0.f;
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int d = j * PER + u;
        qv[u] = (float)q[(int64_t)r * qkv_stride + (int64_t)hk * DK + d];
        kv[u] = (float)k[(int64_t)r * qkv_stride + (int64_t)hk * DK + d];
        sq += qv[u] * qv[u];
        sk += kv[u] * kv[u];
      }
      sq = wave_sum(sq);
      sk = wave_sum(sk);
      const float iq = rsqrtf(sq + 1e-6f) * qscale, ik = rsqrtf(sk + 1e-6f);
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        s_qk[p][0][j * PER + u] = qv[u] * iq;
        s_qk[p][1][j * PER + u] = kv[u] * ik;
      }
      if (j == 0) {
        const float av = (float)a[(int64_t)r * ab_stride + h], bv = (float)b[(int64_t)r * ab_stride + h];
        s_gb[p][0] = __expf(negA * gdn_softplus(av + dtb));
        s_gb[p][1] = 1.f / (1.f + __expf(-bv));
      }
    }
  };

  stage(r0, 0);
  __syncthreads();
  int p = 0;
  for (int r = r0; r < r1; ++r) {
    if (r + 1 < r1) stage(r + 1, p ^ 1);   // the other buffer was last read before the previous barrier
    const float decay = s_gb[p][0], beta = s_gb[p][1];
    const float vj = j < dv ? (float)v[(int64_t)r * qkv_stride + (int64_t)h * dv + j] : 0.f;
    float kvm = 0.f;
#pragma unroll
    for (int i = 0; i < DK; ++i) {
      S[i] *= decay;
      kvm += S[i] * s_qk[p][1][i];
    }
    const float delta = (vj - kvm) * beta;
    float o = 0.f;
#pragma unroll
    for (int i = 0; i < DK; ++i) {
      S[i] += s_qk[p][1][i] * delta;
      o += S[i] * s_qk[p][0][i];
    }
    if (j < dv) out[(int64_t)r * out_stride + (int64_t)h * dv + j] = (bf16)o;
    __syncthreads();
    p ^= 1;
  }
  if (j < dv) {
#pragma unroll
    for (int i = 0; i < DK; ++i) st[(int64_t)j * DK + i] = S[i];
  }
}

// ---------------------------------------------------------------------------------------------
// v3 (default) = prep + scan.
// prep: one wave per (row, k-head) L2-normalises q (also / sqrt(dk)) and k into fp32 workspaces,
//   forms q^.k^, and per v-head the decay exp(g) and beta -- fully parallel over rows, so the
//   sequential scan below does no normalisation work at all.
// scan: state column j of head h is split over L = dk / 8 lanes of one DPP row (8 fp32 entries
//   per lane: the [dv, dk] state gives every lane 32 contiguous bytes and a wave 2 KiB), a wave
//   covers 64 / L columns, the grid is (sequence, v-head, dv / (4 * 64 / L)).  Per row: two
//   in-lane 8-entry dot products (S^T k^, S^T q^), an L-lane all-reduce with DPP (quad_perm
//   xor 1 / xor 2, row_half_mirror, row_mirror: no LDS, no barrier), then
//     delta = (v - decay * S^T k^) * beta,  o = decay * S^T q^ + delta * (k^.q^),
//     S <- decay * S + k^ delta^T
//   i.e. one pass over the state per row, with the next row's q^ / k^ slices prefetched.
template <int DK>
__global__ __launch_bounds__(256) void gdn_prep_kernel(
    const bf16* __restrict__ q, const bf16* __restrict__ k, int64_t qkv_stride, const bf16* __restrict__ a,
    const bf16* __restrict__ b, int64_t ab_stride, const float* __restrict__ A_log, const float* __restrict__ dt_bias,
    float* __restrict__ qn, float* __restrict__ kn, float* __restrict__ qk, float* __restrict__ gb, int T, int Hk,
    int Hv) {
  constexpr int PER = DK / 64;
  const int lane = threadIdx.x & 63;
  const int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int r = wid / Hk, hk = wid - r * Hk;
  if (r >= T) return;   // whole wave
  float qv[PER], kv[PER], sq = 0.f, sk = 0.f, sqk = 0.f;
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int d = lane * PER + u;
    qv[u] = (float)q[(int64_t)r * qkv_stride + (int64_t)hk * DK + d];
    kv[u] = (float)k[(int64_t)r * qkv_stride + (int64_t)hk * DK + d];
    sq += qv[u] * qv[u];
    sk += kv[u] * kv[u];
    sqk += qv[u] * kv[u];
  }
  sq = wave_sum(sq);
  sk = wave_sum(sk);
  sqk = wave_sum(sqk);
  const float iq = rsqrtf(sq + 1e-6f) * rsqrtf((float)DK), ik = rsqrtf(sk + 1e-6f);
  float* qo = qn + ((int64_t)r * Hk + hk) * DK + lane * PER;
  float* ko = kn + ((int64_t)r * Hk + hk) * DK + lane * PER;
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    qo[u] = qv[u] * iq;
    ko[u] = kv[u] * ik;
  }
  if (lane == 0) qk[(int64_t)r * Hk + hk] = sqk * iq * ik;
  const int ratio = Hv / Hk;
  for (int e = lane; e < ratio; e += 64) {
    const int h = hk * ratio + e;
    const float av = (float)a[(int64_t)r * ab_stride + h], bv = (float)b[(int64_t)r * ab_stride + h];
    gb[((int64_t)r * Hv + h) * 2] = __expf(-__expf(A_log[h]) * gdn_softplus(av + dt_bias[h]));
    gb[((int64_t)r * Hv + h) * 2 + 1] = 1.f / (1.f + __expf(-bv));
  }
}

template <int L>
__device__ __forceinline__ float row_allreduce(float v) {   // sum over aligned groups of L lanes (DPP)
  if constexpr (L >= 2)
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  if constexpr (L >= 4)
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  if constexpr (L >= 8)   // row_half_mirror
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false));
  if constexpr (L >= 16)  // row_mirror
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false));
  if constexpr (L >= 32)  // across the two DPP rows of a half-wave (dk = 256)
    v += __shfl_xor(v, 16);
  return v;
}

template <int DK, int NC>
__global__ __launch_bounds__(256) void gdn_scan_v3_kernel(
    const float* __restrict__ qn, const float* __restrict__ kn, const float* __restrict__ qk,
    const float* __restrict__ gb, const bf16* __restrict__ v, int64_t v_stride, float* __restrict__ state,
    bf16* __restrict__ out, int64_t out_stride, const int* __restrict__ cu, const int* __restrict__ slot,
    const int* __restrict__ reset, int Hv, int Hk, int dv) {
  constexpr int L = DK / 8, GPW = 64 / L, CPB = 4 * GPW * NC;   // lanes per column group, groups / wave
  const int s = blockIdx.x, h = blockIdx.y;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int j0 = blockIdx.z * CPB + (w * GPW + lane / L) * NC;   // this lane's NC state columns
  const int i0 = (lane % L) * 8;                                 // and 8 state rows
  const int r0 = cu[s], r1 = cu[s + 1];
  if (r1 <= r0) return;   // uniform per block
  const int hk = h / (Hv / Hk);
  float* st = state + (((int64_t)slot[s] * Hv + h) * dv) * DK + i0;   // [dv, dk]: 32 contiguous bytes / column
  const bool fresh = reset[s] != 0;
  f32x4 S0[NC], S1[NC];
  bool ok[NC];
  int jc[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    ok[c] = j0 + c < dv;
    jc[c] = ok[c] ? j0 + c : 0;
    if (fresh || !ok[c]) {
      S0[c] = f32x4{0.f, 0.f, 0.f, 0.f};
      S1[c] = S0[c];
    } else {
      S0[c] = reinterpret_cast<const f32x4*>(st + (int64_t)jc[c] * DK)[0];
      S1[c] = reinterpret_cast<const f32x4*>(st + (int64_t)jc[c] * DK)[1];
    }
  }
  const bf16* vp = v + (int64_t)h * dv;
  auto qrow = [&](int r) { return reinterpret_cast<const f32x4*>(qn + ((int64_t)r * Hk + hk) * DK + i0); };
  auto krow = [&](int r) { return reinterpret_cast<const f32x4*>(kn + ((int64_t)r * Hk + hk) * DK + i0); };
  f32x4 q0 = qrow(r0)[0], q1 = qrow(r0)[1], k0 = krow(r0)[0], k1 = krow(r0)[1];
  float2 gbn = *reinterpret_cast<const float2*>(gb + ((int64_t)r0 * Hv + h) * 2);
  float kqn = qk[(int64_t)r0 * Hk + hk];
  bf16 vn[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) vn[c] = vp[(int64_t)r0 * v_stride + jc[c]];
  for (int r = r0; r < r1; ++r) {
    const f32x4 qa = q0, qb = q1, ka = k0, kb = k1;
    const float decay = gbn.x, beta = gbn.y, kq = kqn;
    float vj[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) vj[c] = (float)vn[c];
    if (r + 1 < r1) {   // prefetch everything the next row reads
      q0 = qrow(r + 1)[0];
      q1 = qrow(r + 1)[1];
      k0 = krow(r + 1)[0];
      k1 = krow(r + 1)[1];
      gbn = *reinterpret_cast<const float2*>(gb + ((int64_t)(r + 1) * Hv + h) * 2);
      kqn = qk[(int64_t)(r + 1) * Hk + hk];
#pragma unroll
      for (int c = 0; c < NC; ++c) vn[c] = vp[(int64_t)(r + 1) * v_stride + jc[c]];
    }
    float sk[NC], sq[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      sk[c] = 0.f;
      sq[c] = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        sk[c] += S0[c][e] * ka[e] + S1[c][e] * kb[e];
        sq[c] += S0[c][e] * qa[e] + S1[c][e] * qb[e];
      }
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      sk[c] = row_allreduce<L>(sk[c]);
      sq[c] = row_allreduce<L>(sq[c]);
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const float delta = (vj[c] - decay * sk[c]) * beta;
      const float o = decay * sq[c] + delta * kq;
      S0[c] = S0[c] * decay + ka * delta;
      S1[c] = S1[c] * decay + kb * delta;
      if (ok[c] && (lane % L) == 0) out[(int64_t)r * out_stride + (int64_t)h * dv + j0 + c] = (bf16)o;
    }
  }
#pragma unroll
  for (int c = 0; c < NC; ++c)
    if (ok[c]) {
      reinterpret_cast<f32x4*>(st + (int64_t)jc[c] * DK)[0] = S0[c];
      reinterpret_cast<f32x4*>(st + (int64_t)jc[c] * DK)[1] = S1[c];
    }
}

}  // namespace

// q / k / v: row-major views (shared row stride qkv_stride, in elements) of the conv output,
// q and k [T, Hk * dk], v [T, Hv * dv]; a / b: [T, Hv] views (row stride ab_stride); state fp32
// [slots, Hv, dv, dk] (transposed); out [T, Hv * dv].  dk in {64, 128, 256} (v1: 64 / 128, dv <= 128).  ws: fp32 workspace of
// T * (2 * Hk * dk + Hk + 2 * Hv) floats for v3 (null -> the v1 kernel: one lane per state
// column, q / k staged through LDS; kept as the numerics cross-check and for comparison).
OME_API int ome_gdn_scan(const void* q, const void* k, const void* v, int64_t qkv_stride, const void* a,
                         const void* b, int64_t ab_stride, const float* A_log, const float* dt_bias, float* state,
                         void* out, int64_t out_stride, const int* cu, const int* slot, const int* reset, int S,
                         int T, int Hv, int Hk, int dk, int dv, float* ws, hipStream_t stream) {
  if (S <= 0) return 0;
  if (dv <= 0 || Hk <= 0 || Hv % Hk != 0) return -2;
  static const int nc_env = getenv("OME_GDN_NC") ? atoi(getenv("OME_GDN_NC")) : 0;   // bench override
  if (ws) {   // v3: prep (parallel over rows) + scan; any dv (grid z tiles the state columns)
    if (dk != 256 && dk != 128 && dk != 64) return -3;
    float* qn = ws;
    float* kn = qn + (int64_t)T * Hk * dk;
    float* qk = kn + (int64_t)T * Hk * dk;
    float* gb = qk + (int64_t)T * Hk;
    const int waves = T * Hk;
    if (waves > 0) {
      if (dk == 256)
        gdn_prep_kernel<256><<<(waves + 3) / 4, 256, 0, stream>>>((const bf16*)q, (const bf16*)k, qkv_stride,
                                                                  (const bf16*)a, (const bf16*)b, ab_stride, A_log,
                                                                  dt_bias, qn, kn, qk, gb, T, Hk, Hv);
      else if (dk == 128)
        gdn_prep_kernel<128><<<(waves + 3) / 4, 256, 0, stream>>>((const bf16*)q, (const bf16*)k, qkv_stride,
                                                                  (const bf16*)a, (const bf16*)b, ab_stride, A_log,
                                                                  dt_bias, qn, kn, qk, gb, T, Hk, Hv);
      else
        gdn_prep_kernel<64><<<(waves + 3) / 4, 256, 0, stream>>>((const bf16*)q, (const bf16*)k, qkv_stride,
                                                                 (const bf16*)a, (const bf16*)b, ab_stride, A_log,
                                                                 dt_bias, qn, kn, qk, gb, T, Hk, Hv);
      OME_CHECK_LAUNCH();
    }
    // columns per lane: 1 for one or two long prefills (latency-bound: 0.41 us / row at the 80B
    // shape), 2 / 4 as sequences multiply (each lane reuses its q / k slice for more columns,
    // cutting the broadcast traffic that bounds many-sequence batches); profiles/r02_gdn_bench.txt
    const int nc = nc_env > 0 ? nc_env : T == S ? 2 : S * Hv <= 64 ? 1 : S * Hv <= 512 ? 2 : 4;
    const int cpb = 4 * (64 / (dk / 8)) * nc;
    dim3 grid3(S, Hv, (dv + cpb - 1) / cpb);
#define GDN3(DKV, NCV)                                                                                      \
  gdn_scan_v3_kernel<DKV, NCV><<<grid3, 256, 0, stream>>>(qn, kn, qk, gb, (const bf16*)v, qkv_stride, state, \
                                                           (bf16*)out, out_stride, cu, slot, reset, Hv, Hk, dv)
    if (dk == 256) {
      if (nc == 1) GDN3(256, 1);
      else if (nc == 2) GDN3(256, 2);
      else GDN3(256, 4);
    } else if (dk == 128) {
      if (nc == 1) GDN3(128, 1);
      else if (nc == 2) GDN3(128, 2);
      else GDN3(128, 4);
    } else {
      if (nc == 1) GDN3(64, 1);
      else if (nc == 2) GDN3(64, 2);
      else GDN3(64, 4);
    }
#undef GDN3
    OME_CHECK_LAUNCH();
    return 0;
  }
  if (dv > 128) return -2;   // v1: one 128-thread workgroup per (sequence, head)
  dim3 grid(S, Hv);
#define GDN_ARGS                                                                                                \
  (const bf16*)q, (const bf16*)k, (const bf16*)v, qkv_stride, (const bf16*)a, (const bf16*)b, ab_stride, A_log, \
      dt_bias, state, (bf16*)out, out_stride, cu, slot, reset, Hv, Hk, dv
  if (dk == 128) gdn_scan_kernel<128><<<grid, 128, 0, stream>>>(GDN_ARGS);
  else if (dk == 64) gdn_scan_kernel<64><<<grid, 128, 0, stream>>>(GDN_ARGS);
  else return -3;
#undef GDN_ARGS
  OME_CHECK_LAUNCH();
  return 0;
}
