// Gated DeltaNet (Qwen3-Next linear-attention layers; reference catalog
// ``config/runtimes/srt/Qwen/qwen3-next-80b-a3b-instruct-rt.yaml``) for gfx950.
//
// Per value head h of a sequence, with k-head h / (Hv / Hk), L2-normalised q, k (q also scaled
// by 1/sqrt(dk)), g = -exp(A_log[h]) * softplus(a + dt_bias[h]), beta = sigmoid(b):
//   S <- exp(g) * S
//   S <- S + k (beta * (v - S^T k))^T          (the delta rule: a rank-1 correction)
//   o  = S^T q
// S is [dk, dv] fp32 per (slot, head), continued across prefill chunks and decode steps (the
// runner's per-request state slots; ``reset`` starts a sequence's first chunk from zero).
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
  for (int i = 0; i < DK; ++i) S[i] = (fresh || j >= dv) ? 0.f : st[(int64_t)i * dv + j];
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
    for (int i = 0; i < DK; ++i) st[(int64_t)i * dv + j] = S[i];
  }
}

// ---------------------------------------------------------------------------------------------
// v2 (default): no LDS, no barriers.  Each state column j is split over L = DK / 8 lanes of one
// DPP row (8 fp32 entries per lane), so a wave covers 64 / L columns and the grid is
// (sequence, v-head, dv / (4 * 64 / L)) -- 8x more workgroups than v1 and an 8-deep FMA chain
// per dot product instead of DK.  Per row every lane loads its 8-element slices of raw q and k
// (one 16-byte load each, the next row's loads issued before the current row's math), forms five
// partial sums (|q|^2, |k|^2, q.k, S^T k, S^T q) and all-reduces them over its L lanes with DPP
// (quad_perm xor 1 / xor 2, row_half_mirror, row_mirror).  Normalisation is applied to the
// reduced scalars instead of the vectors:
//   kv = decay * |k|^-1 * (S^T k),   delta = (v - kv) * beta,
//   o  = decay * iq * (S^T q) + delta * iq * |k|^-1 * (q.k),   S <- decay * S + (|k|^-1 delta) k
// with iq = |q|^-1 / sqrt(dk) -- the same function as v1 with one pass over S per row.
template <int L>
__device__ __forceinline__ float dpp_allreduce(float v) {
  if constexpr (L >= 2)
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  if constexpr (L >= 4)
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  if constexpr (L >= 8)
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false));
  if constexpr (L >= 16)
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false));
  return v;
}

template <int DK>
__global__ __launch_bounds__(256) void gdn_scan_v2_kernel(
    const bf16* __restrict__ q, const bf16* __restrict__ k, const bf16* __restrict__ v, int64_t qkv_stride,
    const bf16* __restrict__ a, const bf16* __restrict__ b, int64_t ab_stride, const float* __restrict__ A_log,
    const float* __restrict__ dt_bias, float* __restrict__ state, bf16* __restrict__ out, int64_t out_stride,
    const int* __restrict__ cu, const int* __restrict__ slot, const int* __restrict__ reset, int Hv, int Hk,
    int dv) {
  constexpr int L = DK / 8, CPW = 64 / L, CPB = 4 * CPW;
  const int s = blockIdx.x, h = blockIdx.y;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int j = blockIdx.z * CPB + w * CPW + lane / L;   // state column
  const int e0 = (lane % L) * 8;                         // first of this lane's 8 state rows
  const int r0 = cu[s], r1 = cu[s + 1];
  if (r1 <= r0) return;   // uniform per block
  const bool col = j < dv;
  const int jc = col ? j : 0;
  const int hk = h / (Hv / Hk);
  float* st = state + ((int64_t)slot[s] * Hv + h) * DK * dv + jc;
  float S[8];
  const bool fresh = reset[s] != 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) S[i] = (fresh || !col) ? 0.f : st[(int64_t)(e0 + i) * dv];
  const float negA = -__expf(A_log[h]), dtb = dt_bias[h];
  const float qscale = rsqrtf((float)DK);
  const bf16* qp = q + (int64_t)hk * DK + e0;
  const bf16* kp = k + (int64_t)hk * DK + e0;
  const bf16* vp = v + (int64_t)h * dv + jc;

  bf16x8 qn = ld8(qp + (int64_t)r0 * qkv_stride), kn = ld8(kp + (int64_t)r0 * qkv_stride);
  bf16 vn = vp[(int64_t)r0 * qkv_stride];
  bf16 an = a[(int64_t)r0 * ab_stride + h], bn = b[(int64_t)r0 * ab_stride + h];
  for (int r = r0; r < r1; ++r) {
    const bf16x8 qc = qn, kc = kn;
    const float vj = (float)vn, av = (float)an, bv = (float)bn;
    if (r + 1 < r1) {   // prefetch the next row
      const int64_t o = (int64_t)(r + 1) * qkv_stride;
      qn = ld8(qp + o);
      kn = ld8(kp + o);
      vn = vp[o];
      an = a[(int64_t)(r + 1) * ab_stride + h];
      bn = b[(int64_t)(r + 1) * ab_stride + h];
    }
    float qq = 0.f, kk = 0.f, qk = 0.f, sk = 0.f, sq = 0.f, kf[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float qi = (float)qc[i], ki = (float)kc[i];
      kf[i] = ki;
      qq += qi * qi;
      kk += ki * ki;
      qk += qi * ki;
      sk += S[i] * ki;
      sq += S[i] * qi;
    }
    qq = dpp_allreduce<L>(qq);
    kk = dpp_allreduce<L>(kk);
    qk = dpp_allreduce<L>(qk);
    sk = dpp_allreduce<L>(sk);
    sq = dpp_allreduce<L>(sq);
    const float decay = __expf(negA * gdn_softplus(av + dtb)), beta = 1.f / (1.f + __expf(-bv));
    const float ik = rsqrtf(kk + 1e-6f), iq = rsqrtf(qq + 1e-6f) * qscale;
    const float delta = (vj - decay * ik * sk) * beta;
    const float o = decay * iq * sq + delta * iq * ik * qk;
    const float dk_ = ik * delta;
#pragma unroll
    for (int i = 0; i < 8; ++i) S[i] = S[i] * decay + kf[i] * dk_;
    if (col && (lane % L) == 0) out[(int64_t)r * out_stride + (int64_t)h * dv + j] = (bf16)o;
  }
  if (col) {
#pragma unroll
    for (int i = 0; i < 8; ++i) st[(int64_t)(e0 + i) * dv] = S[i];
  }
}

}  // namespace

// q / k / v: row-major views (shared row stride qkv_stride, in elements) of the conv output,
// q and k [T, Hk * dk], v [T, Hv * dv]; a / b: [T, Hv] views (row stride ab_stride); state fp32
// [slots, Hv, dk, dv]; out [T, Hv * dv].  dk in {64, 128}, dv <= 128.
OME_API int ome_gdn_scan(const void* q, const void* k, const void* v, int64_t qkv_stride, const void* a,
                         const void* b, int64_t ab_stride, const float* A_log, const float* dt_bias, float* state,
                         void* out, int64_t out_stride, const int* cu, const int* slot, const int* reset, int S,
                         int Hv, int Hk, int dk, int dv, hipStream_t stream) {
  if (S <= 0) return 0;
  if (dv <= 0 || dv > 128 || Hk <= 0 || Hv % Hk != 0) return -2;
  static const bool v1 = getenv("OME_GDN_V1") && getenv("OME_GDN_V1")[0] == '1';
  // v2 reads q / k slices with 16-byte loads; unaligned views take v1
  if (!v1 && qkv_stride % 8 == 0 && !((uintptr_t)q & 15) && !((uintptr_t)k & 15)) {
    const int cpb = 4 * 64 / (dk / 8);
    dim3 grid2(S, Hv, (dv + cpb - 1) / cpb);
#define GDN2_ARGS                                                                                               \
  (const bf16*)q, (const bf16*)k, (const bf16*)v, qkv_stride, (const bf16*)a, (const bf16*)b, ab_stride, A_log, \
      dt_bias, state, (bf16*)out, out_stride, cu, slot, reset, Hv, Hk, dv
    if (dk == 128) gdn_scan_v2_kernel<128><<<grid2, 256, 0, stream>>>(GDN2_ARGS);
    else if (dk == 64) gdn_scan_v2_kernel<64><<<grid2, 256, 0, stream>>>(GDN2_ARGS);
    else return -3;
#undef GDN2_ARGS
    OME_CHECK_LAUNCH();
    return 0;
  }
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
