// Paged attention on MFMA for gfx950: decode (split-K "flash-decoding", K5) and
// varlen causal prefill with prefix / chunked-prefill support (K4).  SURVEY.md §2.9.
//
// Both kernels use v_mfma_f32_16x16x32_bf16 and need NO LDS transposes: the paged cache
// layouts (rope_cache.hip) put every MFMA operand in lane-contiguous 8/16-byte runs.
//
// Fragment maps (16x16x32 bf16, cdna_hip_programming.md §3):
//   A: lane l holds A[row = l&15][k = 8*(l>>4) + j]   j = 0..7
//   B: lane l holds B[k = 8*(l>>4) + j][col = l&15]
//   C: lane l reg i  = C[row = 4*(l>>4) + i][col = l&15]
//
// Scores are computed transposed, S^T = K * Q^T (keys on MFMA rows, queries on lanes), so
// each lane owns one query column: the softmax row statistics stay lane-local up to a
// 4-lane-group xor-shuffle.  The output is accumulated transposed too, O^T = V^T * P^T,
// with the 32 keys of two pages assigned to the K slots in the permuted order
//   k-slot (g, j) = page (j >> 2), key 4g + (j & 3)
// which is exactly the order the S^T accumulators already sit in, so P feeds the second
// MFMA from registers with no lane movement (the "accumulator as next operand" idiom).
//
// KV-cache formats (K15): every kernel except decode v1 is templated on the cache element
// format F (common.h KVFmt).  fp8 caches are read at half the bytes and converted to bf16 in
// registers just before the MFMA; the host folds k_scale into the softmax scale and the
// kernels multiply the normalised output by v_scale.
#include "common.h"

#include <cstdlib>

#ifndef OME_NEG_INF
#define OME_NEG_INF (-__builtin_inff())
#endif

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// First key a query at position ``qpos`` may see.  ``window`` > 0: sliding window of that many keys
// (Mistral / Gemma / GPT-OSS); ``window`` < -1: chunked attention with chunks of -window tokens
// (Llama-4 RoPE layers: keys in the query's own chunk only); otherwise full causal.
__device__ __forceinline__ int attn_lo(int qpos, int window) {
  return window > 0 ? max(0, qpos - window + 1) : (window < -1 ? qpos - qpos % (-window) : 0);
}

// raw score -> log2-domain logit: s * scale * log2(e), or with logit soft-capping (Gemma-2:
// cap * tanh(s * scale / cap)) cap * log2(e) * tanh(s * scale / cap)
struct Scaler {
  float mul;      // scale * log2(e) (cap_inv == 0)
  float cap_inv;  // scale / cap, 0 = no soft-capping
  float cap_l2;   // cap * log2(e)
  const float* alibi;  // ALiBi slopes per query head (Bloom / MPT / Falcon-RW), nullptr = off: the
                       // logit gains slope * (key_pos - query_pos), i.e. alibi_l2(head) * (k - q)
  const int* row_lo;   // decode only: per-row first visible key (nullptr = 0) -- Mllama cross
                       // attention reads one [lo, seq_len) range of a request's vision-token cache
  // Block-sparse causal attention (Phi-3-small): keys and queries in blocks of 1 << bs_shift
  // tokens; query block qb sees key block kb <= qb when qb - kb < bs_local (the local band) or
  // (kb + bs_h0 + head * bs_step + 1) % bs_vert == 0 (per-head vertical stripes).  bs_shift == 0:
  // dense.  Applied as a -inf mask on the scores; the v2 prefill kernel also skips key stages no
  // head of its kv group sees (bs_stage_needed) before loading them.
  int bs_shift, bs_local, bs_vert, bs_step, bs_h0;
  int bs_skip;   // prefill skips invisible stages (OME_BS_SKIP=0: mask only, the r05 behaviour)
  __device__ __forceinline__ float alibi_l2(int head) const {
    return alibi != nullptr ? alibi[head] * 1.4426950408889634f : 0.f;
  }
  __device__ __forceinline__ bool bs_visible(int qpos, int key, int head) const {
    if (bs_shift == 0) return true;
    const int qb = qpos >> bs_shift, kb = key >> bs_shift;
    return qb - kb < bs_local || bs_stripe(kb, head);
  }
  // block kb is a vertical stripe of `head`
  __device__ __forceinline__ bool bs_stripe(int kb, int head) const {
    return (kb + bs_h0 + head * bs_step + 1) % bs_vert == 0;
  }
  // Does any (query, head) of query blocks >= qb_lo (up to the causal limit) and heads h0 ..
  // h0 + nh - 1 see a key of [k0, k0 + n)?  The local band is widest for the EARLIEST query
  // block, so qb_lo decides it.  Block-sparse kernels skip stages nobody sees, before loading.
  __device__ __forceinline__ bool bs_stage_needed(int k0, int n, int qb_lo, int h0, int nh) const {
    if (bs_shift == 0) return true;
    const int b0 = k0 >> bs_shift, b1 = (k0 + n - 1) >> bs_shift;
    if (qb_lo - b1 < bs_local) return true;   // the last block is in the first row's local band
    for (int b = b0; b <= b1; ++b) {
      if (qb_lo - b < bs_local) return true;
      for (int h = 0; h < nh; ++h)
        if (bs_stripe(b, h0 + h)) return true;
    }
    return false;
  }
  // Every query block in [qb_lo, qb_hi] of `head` sees every key of [k0, k0 + n)?
  __device__ __forceinline__ bool bs_stage_full(int k0, int n, int qb_hi, int head) const {
    if (bs_shift == 0) return true;
    const int b0 = k0 >> bs_shift, b1 = (k0 + n - 1) >> bs_shift;
    if (qb_hi - b0 < bs_local) return true;
    for (int b = b0; b <= b1; ++b)
      if (qb_hi - b >= bs_local && !bs_stripe(b, head)) return false;
    return true;
  }
  __device__ __forceinline__ float operator()(float s) const {
    if (cap_inv > 0.f) {
      const float e = fast_exp2(2.8853900817779268f * s * cap_inv);  // exp(2x)
      return cap_l2 * (1.f - 2.f / (e + 1.f));                        // tanh(x), saturating at +-1
    }
    return s * mul;
  }
};

// packed block-sparse parameters (ops.blocksparse_pack): [0:4) log2 block, [4:20) local blocks,
// [20:32) vertical stride, [32:40) head step, [40:52) global index of this rank's first head
static inline void set_blocksparse(Scaler& r, int64_t bs) {
  r.bs_shift = (int)(bs & 15);
  r.bs_local = (int)((bs >> 4) & 0xffff);
  r.bs_vert = (int)((bs >> 20) & 0xfff);
  r.bs_step = (int)((bs >> 32) & 0xff);
  r.bs_h0 = (int)((bs >> 40) & 0xfff);
  if (r.bs_vert <= 0) r.bs_shift = 0;
  static const int skip = getenv("OME_BS_SKIP") ? atoi(getenv("OME_BS_SKIP")) : 1;
  r.bs_skip = skip;
}

static inline Scaler make_scaler(float scale, float softcap, const float* alibi = nullptr, int64_t bs = 0) {
  const float l2e = 1.4426950408889634f;
  Scaler r;
  r.alibi = alibi;
  r.row_lo = nullptr;
  set_blocksparse(r, bs);
  r.mul = scale * l2e;
  r.cap_inv = softcap > 0.f ? scale / softcap : 0.f;
  r.cap_l2 = softcap > 0.f ? softcap * l2e : 0.f;
  return r;
}

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8 cat44(bf16x4 a, bf16x4 b) {
  bf16x8 r;
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; r[3] = a[3];
  r[4] = b[0]; r[5] = b[1]; r[6] = b[2]; r[7] = b[3];
  return r;
}

// raw cache fragments (8 consecutive elements / 4 consecutive elements) and their bf16 views
template <int F> struct KVRaw {
  typedef uint2 K8;
  typedef uint32_t V4;
};
template <> struct KVRaw<KV_BF16> {
  typedef bf16x8 K8;
  typedef bf16x4 V4;
};

template <int F>
__device__ __forceinline__ bf16x8 k8_bf16(const typename KVRaw<F>::K8& x) {
  if constexpr (F == KV_BF16) return x;
  else return fp8x8_to_bf16<F>(x);
}
template <int F>
__device__ __forceinline__ bf16x4 v4_bf16(const typename KVRaw<F>::V4& x) {
  if constexpr (F == KV_BF16) return x;
  else return fp8x4_to_bf16<F>(x);
}
template <int F>
__device__ __forceinline__ typename KVRaw<F>::K8 k8_load(const typename KVStore<F>::T* p) {
  return *reinterpret_cast<const typename KVRaw<F>::K8*>(p);
}
template <int F>
__device__ __forceinline__ typename KVRaw<F>::V4 v4_load(const typename KVStore<F>::T* p) {
  return *reinterpret_cast<const typename KVRaw<F>::V4*>(p);
}

// ------------------------------------------------------------------------------------------
// Decode: one workgroup = (partition, kv head, sequence); 4 waves split the partition's
// 32-key tiles round-robin, each with its own online-softmax state, merged through LDS.
// The G = Hq/Hkv query heads of the kv head share every K/V byte loaded (GQA-aware).
// ------------------------------------------------------------------------------------------
template <int D, int P>
__global__ __launch_bounds__(256) void paged_decode_kernel(
    const bf16* __restrict__ q, int64_t q_stride, const bf16* __restrict__ k_cache,
    const bf16* __restrict__ v_cache, const int* __restrict__ block_tables, int bt_stride,
    const int* __restrict__ seq_lens, bf16* __restrict__ out, int64_t out_stride, float* __restrict__ part_o,
    float* __restrict__ part_ml, int Hq, int Hkv, int part_size, int max_parts, float scale_log2, int window) {
  static_assert(P == 16, "decode kernel assumes 16-token pages");
  constexpr int NB = D / 16;  // 16-dim output blocks
  constexpr int KS = D / 32;  // 32-dim k-steps for QK
  const int part = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  const int seq_len = seq_lens[b];
  const int p_start = part * part_size;
  if (p_start >= seq_len) return;
  const int p_end = min(seq_len, p_start + part_size);
  const int G = Hq / Hkv;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n = lane & 15, g = lane >> 4;
  const int lo = attn_lo(seq_len - 1, window);

  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sm_m = smem;              // [4][16]
  float* sm_l = smem + 64;         // [4][16]
  float* sm_o = smem + 128;        // [4][16][D]

  // Q^T fragments (B operand): head n, dims 32ks + 8g .. +7
  bf16x8 qf[KS];
  {
    const bf16* qh = q + (int64_t)b * q_stride + (int64_t)(kvh * G + n) * D;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (n < G) qf[ks] = ld8(qh + 32 * ks + 8 * g);
      else qf[ks] = bf16x8{};
    }
  }
  float m_i = OME_NEG_INF, l_i = 0.f;
  f32x4 o[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) o[nb] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int* bt = block_tables + (int64_t)b * bt_stride;
  const int64_t kpage = (int64_t)Hkv * P * D;  // elements per page (all heads)
  for (int kb = p_start + wave * 32; kb < p_end; kb += 128) {
    if (kb + 32 <= lo) continue;
    const int pA = bt[kb / P];
    const int pB = (kb + P < seq_len) ? bt[kb / P + 1] : pA;
    const bf16* kA = k_cache + pA * kpage + (int64_t)kvh * P * D;
    const bf16* kB = k_cache + pB * kpage + (int64_t)kvh * P * D;
    f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8 a0 = ld8(kA + n * D + 32 * ks + 8 * g);
      bf16x8 a1 = ld8(kB + n * D + 32 * ks + 8 * g);
      s0 = mfma16(a0, qf[ks], s0);
      s1 = mfma16(a1, qf[ks], s1);
    }
    float mt = OME_NEG_INF;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k0 = kb + 4 * g + i, k1 = k0 + 16;
      s0[i] = (k0 < p_end && k0 >= lo) ? s0[i] * scale_log2 : OME_NEG_INF;
      s1[i] = (k1 < p_end && k1 >= lo) ? s1[i] * scale_log2 : OME_NEG_INF;
      mt = fmaxf(mt, fmaxf(s0[i], s1[i]));
    }
    mt = group4_max(mt);
    const float m_new = fmaxf(m_i, mt);
    const float m_use = (m_new == OME_NEG_INF) ? 0.f : m_new;
    const float alpha = fast_exp2(m_i - m_use);
    bf16x8 pb;
    float rs = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float p0 = fast_exp2(s0[i] - m_use), p1 = fast_exp2(s1[i] - m_use);
      pb[i] = (bf16)p0;
      pb[4 + i] = (bf16)p1;
      rs += p0 + p1;
    }
    rs = group4_sum(rs);
    l_i = l_i * alpha + rs;
    m_i = m_new;
    const bf16* vA = v_cache + pA * kpage + (int64_t)kvh * D * P;
    const bf16* vB = v_cache + pB * kpage + (int64_t)kvh * D * P;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const int dim = 16 * nb + n;
      bf16x8 a = cat44(ld4(vA + dim * P + 4 * g), ld4(vB + dim * P + 4 * g));
      o[nb] = o[nb] * alpha;
      o[nb] = mfma16(a, pb, o[nb]);
    }
  }
  // ---- merge the 4 waves' states ----
  if (g == 0) {
    sm_m[wave * 16 + n] = m_i;
    sm_l[wave * 16 + n] = l_i;
  }
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int i = 0; i < 4; ++i) sm_o[(wave * 16 + n) * D + 16 * nb + 4 * g + i] = o[nb][i];
  __syncthreads();
  const int nparts = (seq_len + part_size - 1) / part_size;
  for (int idx = threadIdx.x; idx < G * D; idx += 256) {
    const int h = idx / D, d = idx % D;
    float M = OME_NEG_INF;
#pragma unroll
    for (int w = 0; w < 4; ++w) M = fmaxf(M, sm_m[w * 16 + h]);
    const float Mu = (M == OME_NEG_INF) ? 0.f : M;
    float L = 0.f, acc = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float f = fast_exp2(sm_m[w * 16 + h] - Mu);
      L += sm_l[w * 16 + h] * f;
      acc += sm_o[(w * 16 + h) * D + d] * f;
    }
    const int head = kvh * G + h;
    const float res = L > 0.f ? acc / L : 0.f;
    if (nparts == 1) {
      out[(int64_t)b * out_stride + (int64_t)head * D + d] = (bf16)res;
    } else {
      const int64_t pidx = ((int64_t)b * Hq + head) * max_parts + part;
      part_o[pidx * D + d] = res;
      if (d == 0) {
        part_ml[pidx * 2 + 0] = M;
        part_ml[pidx * 2 + 1] = L;
      }
    }
  }
}

// Split-K partition span of a sequence: a fixed ``part_size`` (multiple of 128), or with
// part_size == 0 the sequence's own length spread over ``max_parts`` partitions (128-key granules),
// so short contexts still fill every partition instead of leaving all but the first idle.
__device__ __forceinline__ int decode_part_span(int part_size, int seq_len, int max_parts) {
  if (part_size > 0) return part_size;
  return max(128, (((seq_len + max_parts - 1) / max_parts) + 127) & ~127);
}

template <int D>
__global__ __launch_bounds__(D) void paged_decode_reduce_kernel(const int* __restrict__ seq_lens,
                                                                 const float* __restrict__ part_o,
                                                                 const float* __restrict__ part_ml,
                                                                 bf16* __restrict__ out, int64_t out_stride, int Hq,
                                                                 int part_size, int max_parts,
                                                                 const float* __restrict__ sinks = nullptr) {
  const int b = blockIdx.y, head = blockIdx.x, d = threadIdx.x;
  const int seq_len = seq_lens[b];
  const int psz = decode_part_span(part_size, seq_len, max_parts);
  const int nparts = (seq_len + psz - 1) / psz;
  if (nparts <= 1) return;
  const int64_t base = ((int64_t)b * Hq + head) * max_parts;
  float M = OME_NEG_INF;
  for (int p = 0; p < nparts; ++p) M = fmaxf(M, part_ml[(base + p) * 2]);
  const float Mu = (M == OME_NEG_INF) ? 0.f : M;
  float L = 0.f, acc = 0.f;
  for (int p = 0; p < nparts; ++p) {
    const float w = part_ml[(base + p) * 2 + 1] * fast_exp2(part_ml[(base + p) * 2] - Mu);
    L += w;
    acc += w * part_o[(base + p) * D + d];
  }
  if (sinks != nullptr) L += fast_exp2(sinks[head] * 1.4426950408889634f - Mu);
  out[(int64_t)b * out_stride + (int64_t)head * D + d] = (bf16)(L > 0.f ? acc / L : 0.f);
}

// ------------------------------------------------------------------------------------------
// Decode v2 (default): same math and layouts as v1, re-scheduled for HBM streaming.
//  * a tile's K AND V fragments are issued together (one memory round trip per 32-key tile,
//    not two), and the next tile of the wave is issued before the current one is consumed
//    (2-deep register ring, counted vmcnt by the compiler): ~32 KB in flight per wave;
//  * the LDS merge stores only the G live query heads (8.5 KB for G=4 instead of 33 KB), so
//    occupancy is set by VGPRs, not LDS;
//  * fp8 caches keep the raw bytes in the tile (half the VGPRs) and convert at consume time.
// ------------------------------------------------------------------------------------------
template <int D, int F>
struct KVTile {
  typename KVRaw<F>::K8 ka[D / 32], kb[D / 32];
  typename KVRaw<F>::V4 va[D / 16], vb[D / 16];
};

template <int D, int P, int F>
__device__ __forceinline__ void kv_tile_load(KVTile<D, F>& t, const typename KVStore<F>::T* __restrict__ k_cache,
                                             const typename KVStore<F>::T* __restrict__ v_cache,
                                             const int* __restrict__ bt, int kb, int seq_len, int64_t kpage, int kvh,
                                             int n, int g) {
  const int pA = bt[kb / P];
  const int pB = (kb + P < seq_len) ? bt[kb / P + 1] : pA;
  const typename KVStore<F>::T* kA = k_cache + pA * kpage + (int64_t)kvh * P * D;
  const typename KVStore<F>::T* kB = k_cache + pB * kpage + (int64_t)kvh * P * D;
  const typename KVStore<F>::T* vA = v_cache + pA * kpage + (int64_t)kvh * D * P;
  const typename KVStore<F>::T* vB = v_cache + pB * kpage + (int64_t)kvh * D * P;
#pragma unroll
  for (int ks = 0; ks < D / 32; ++ks) {
    t.ka[ks] = k8_load<F>(kA + n * D + 32 * ks + 8 * g);
    t.kb[ks] = k8_load<F>(kB + n * D + 32 * ks + 8 * g);
  }
#pragma unroll
  for (int nb = 0; nb < D / 16; ++nb) {
    const int dim = 16 * nb + n;
    t.va[nb] = v4_load<F>(vA + dim * P + 4 * g);
    t.vb[nb] = v4_load<F>(vB + dim * P + 4 * g);
  }
}

template <int D, int F, bool AL = false>
__device__ __forceinline__ void kv_tile_compute(const KVTile<D, F>& t, const bf16x8 (&qf)[D / 32],
                                                f32x4 (&o)[D / 16], float& m_i, float& l_i, int kb, int p_end,
                                                int lo, Scaler scl, int g, float al, int qpos, int head = 0) {
  f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < D / 32; ++ks) {
    s0 = mfma16(k8_bf16<F>(t.ka[ks]), qf[ks], s0);
    s1 = mfma16(k8_bf16<F>(t.kb[ks]), qf[ks], s1);
  }
  float mt = OME_NEG_INF;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int k0 = kb + 4 * g + i, k1 = k0 + 16;
    // AL instantiation: ALiBi bias and / or the block-sparse mask (both per query head)
    const bool v0 = k0 < p_end && k0 >= lo && (!AL || scl.bs_visible(qpos, k0, head));
    const bool v1 = k1 < p_end && k1 >= lo && (!AL || scl.bs_visible(qpos, k1, head));
    s0[i] = v0 ? (AL ? scl(s0[i]) + al * (float)(k0 - qpos) : scl(s0[i])) : OME_NEG_INF;
    s1[i] = v1 ? (AL ? scl(s1[i]) + al * (float)(k1 - qpos) : scl(s1[i])) : OME_NEG_INF;
    mt = fmaxf(mt, fmaxf(s0[i], s1[i]));
  }
  mt = group4_max(mt);
  const float m_new = fmaxf(m_i, mt);
  const float m_use = (m_new == OME_NEG_INF) ? 0.f : m_new;
  const float alpha = fast_exp2(m_i - m_use);
  bf16x8 pb;
  float rs = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float p0 = fast_exp2(s0[i] - m_use), p1 = fast_exp2(s1[i] - m_use);
    pb[i] = (bf16)p0;
    pb[4 + i] = (bf16)p1;
    rs += p0 + p1;
  }
  rs = group4_sum(rs);
  l_i = l_i * alpha + rs;
  m_i = m_new;
#pragma unroll
  for (int nb = 0; nb < D / 16; ++nb) {
    o[nb] = o[nb] * alpha;
    o[nb] = mfma16(cat44(v4_bf16<F>(t.va[nb]), v4_bf16<F>(t.vb[nb])), pb, o[nb]);
  }
}

// ---- key-permuted tile (decode v4): MFMA row n of S^T tile s0 holds key 8*((n>>2)&1) + (n&3) of page
// (n>>3), tile s1 the key 4 later.  The S^T accumulators of lane group g then hold keys
// 8*(g&1) .. +7 of page g>>1, so the V^T operand of a lane is 8 CONSECUTIVE keys of one page:
// one 16-B load per 16 dims (bf16) instead of two 8-B loads from two pages.
template <int D, int F>
struct KVTileP {
  typename KVRaw<F>::K8 ka[D / 32], kb[D / 32];
  typename KVRaw<F>::K8 v[D / 16];
};

template <int D, int P, int F>
__device__ __forceinline__ void kv_tilep_load(KVTileP<D, F>& t, const typename KVStore<F>::T* __restrict__ k_cache,
                                              const typename KVStore<F>::T* __restrict__ v_cache,
                                              const int* __restrict__ bt, int kb, int seq_len, int64_t kpage, int kvh,
                                              int n, int g) {
  const int pA = bt[kb / P];
  const int pB = (kb + P < seq_len) ? bt[kb / P + 1] : pA;
  const int prow = (n >> 3) ? pB : pA, krow = 8 * ((n >> 2) & 1) + (n & 3);
  const typename KVStore<F>::T* k0 = k_cache + prow * kpage + (int64_t)kvh * P * D + krow * D;
  const typename KVStore<F>::T* k1 = k0 + 4 * D;
  const typename KVStore<F>::T* vp = v_cache + ((g >> 1) ? pB : pA) * kpage + (int64_t)kvh * D * P + 8 * (g & 1);
#pragma unroll
  for (int ks = 0; ks < D / 32; ++ks) {
    t.ka[ks] = k8_load<F>(k0 + 32 * ks + 8 * g);
    t.kb[ks] = k8_load<F>(k1 + 32 * ks + 8 * g);
  }
#pragma unroll
  for (int nb = 0; nb < D / 16; ++nb) t.v[nb] = k8_load<F>(vp + (16 * nb + n) * P);
}

template <int D, int F, bool AL = false>
__device__ __forceinline__ void kv_tilep_compute(const KVTileP<D, F>& t, const bf16x8 (&qf)[D / 32],
                                                 f32x4 (&o)[D / 16], float& m_i, float& l_i, int kb, int p_end,
                                                 int lo, Scaler scl, int g, float al, int qpos, int head = 0) {
  f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < D / 32; ++ks) {
    s0 = mfma16(k8_bf16<F>(t.ka[ks]), qf[ks], s0);
    s1 = mfma16(k8_bf16<F>(t.kb[ks]), qf[ks], s1);
  }
  const int base = kb + 16 * (g >> 1) + 8 * (g & 1);
  float mt = OME_NEG_INF;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int k0 = base + i, k1 = k0 + 4;
    // AL instantiation: ALiBi bias and / or the block-sparse mask (both per query head)
    const bool v0 = k0 < p_end && k0 >= lo && (!AL || scl.bs_visible(qpos, k0, head));
    const bool v1 = k1 < p_end && k1 >= lo && (!AL || scl.bs_visible(qpos, k1, head));
    s0[i] = v0 ? (AL ? scl(s0[i]) + al * (float)(k0 - qpos) : scl(s0[i])) : OME_NEG_INF;
    s1[i] = v1 ? (AL ? scl(s1[i]) + al * (float)(k1 - qpos) : scl(s1[i])) : OME_NEG_INF;
    mt = fmaxf(mt, fmaxf(s0[i], s1[i]));
  }
  mt = group4_max(mt);
  const float m_new = fmaxf(m_i, mt);
  const float m_use = (m_new == OME_NEG_INF) ? 0.f : m_new;
  const float alpha = fast_exp2(m_i - m_use);
  bf16x8 pb;
  float rs = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float p0 = fast_exp2(s0[i] - m_use), p1 = fast_exp2(s1[i] - m_use);
    pb[i] = (bf16)p0;
    pb[4 + i] = (bf16)p1;
    rs += p0 + p1;
  }
  rs = group4_sum(rs);
  l_i = l_i * alpha + rs;
  m_i = m_new;
#pragma unroll
  for (int nb = 0; nb < D / 16; ++nb) {
    o[nb] = o[nb] * alpha;
    o[nb] = mfma16(k8_bf16<F>(t.v[nb]), pb, o[nb]);
  }
}

template <int D, int P, int MODE, int F, bool AL = false>
__global__ __launch_bounds__(256) void paged_decode_v2_kernel(
    const bf16* __restrict__ q, int64_t q_stride, const typename KVStore<F>::T* __restrict__ k_cache,
    const typename KVStore<F>::T* __restrict__ v_cache, const int* __restrict__ block_tables, int bt_stride,
    const int* __restrict__ seq_lens, bf16* __restrict__ out, int64_t out_stride, float* __restrict__ part_o,
    float* __restrict__ part_ml, int Hq, int Hkv, int part_size, int max_parts, Scaler scl, int window,
    const int* __restrict__ order, float v_scale, const float* __restrict__ sinks) {
  static_assert(P == 16, "decode kernel assumes 16-token pages");
  constexpr int NB = D / 16, KS = D / 32;
  // blockIdx.z walks sequences longest-first when the host provides ``order`` (the dispatcher
  // hands out workgroups in grid order, so the long tail starts first instead of last)
  const int part = blockIdx.x, kvh = blockIdx.y, b = order ? order[blockIdx.z] : blockIdx.z;
  const int seq_len = seq_lens[b];
  const int psz = decode_part_span(part_size, seq_len, max_parts);
  const int p_start = part * psz;
  if (p_start >= seq_len) return;
  const int p_end = min(seq_len, p_start + psz);
  const int G = Hq / Hkv;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n = lane & 15, g = lane >> 4;
  const int lo = scl.row_lo != nullptr ? max(attn_lo(seq_len - 1, window), scl.row_lo[b]) : attn_lo(seq_len - 1, window);
  const float al = n < G ? scl.alibi_l2(kvh * G + n) : 0.f;  // this lane's query head (S^T column n)
  const int qpos = seq_len - 1;

  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sm_m = smem;              // [4][G]
  float* sm_l = smem + 4 * G;      // [4][G]
  float* sm_o = smem + 8 * G;      // [4][G][D]

  bf16x8 qf[KS];
  {
    const bf16* qh = q + (int64_t)b * q_stride + (int64_t)(kvh * G + n) * D;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[ks] = (n < G) ? ld8(qh + 32 * ks + 8 * g) : bf16x8{};
  }
  float m_i = OME_NEG_INF, l_i = 0.f;
  f32x4 o[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) o[nb] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int* bt = block_tables + (int64_t)b * bt_stride;
  const int64_t kpage = (int64_t)Hkv * P * D;
  int kb = p_start + wave * 32;
  if (lo > 0) {  // sliding window: skip whole tiles before the window
    while (kb + 32 <= lo && kb < p_end) kb += 128;
  }
  if (MODE == 2) {
    const int qb = AL && scl.bs_shift ? qpos >> scl.bs_shift : 0;
    for (; kb < p_end; kb += 128) {
      // block-sparse: a 32-key tile no head of the group sees is not loaded at all
      if (AL && scl.bs_shift && scl.bs_skip && !scl.bs_stage_needed(kb, 32, qb, kvh * G, G)) continue;
      KVTileP<D, F> t;
      kv_tilep_load<D, P, F>(t, k_cache, v_cache, bt, kb, seq_len, kpage, kvh, n, g);
      kv_tilep_compute<D, F, AL>(t, qf, o, m_i, l_i, kb, p_end, lo, scl, g, al, qpos, kvh * G + n);
    }
  } else if (MODE == 0) {
    for (; kb < p_end; kb += 128) {
      KVTile<D, F> t;
      kv_tile_load<D, P, F>(t, k_cache, v_cache, bt, kb, seq_len, kpage, kvh, n, g);
      kv_tile_compute<D, F, AL>(t, qf, o, m_i, l_i, kb, p_end, lo, scl, g, al, qpos, kvh * G + n);
    }
  } else if (kb < p_end) {
    KVTile<D, F> t0, t1;
    kv_tile_load<D, P, F>(t0, k_cache, v_cache, bt, kb, seq_len, kpage, kvh, n, g);
    for (;;) {
      const int kn = kb + 128;
      const bool more = kn < p_end;
      if (more) kv_tile_load<D, P, F>(t1, k_cache, v_cache, bt, kn, seq_len, kpage, kvh, n, g);
      kv_tile_compute<D, F, AL>(t0, qf, o, m_i, l_i, kb, p_end, lo, scl, g, al, qpos, kvh * G + n);
      if (!more) break;
      const int kn2 = kn + 128;
      const bool more2 = kn2 < p_end;
      if (more2) kv_tile_load<D, P, F>(t0, k_cache, v_cache, bt, kn2, seq_len, kpage, kvh, n, g);
      kv_tile_compute<D, F, AL>(t1, qf, o, m_i, l_i, kn, p_end, lo, scl, g, al, qpos, kvh * G + n);
      if (!more2) break;
      kb = kn2;
    }
  }
  // ---- merge the 4 waves' states (only the G live heads) ----
  if (g == 0 && n < G) {
    sm_m[wave * G + n] = m_i;
    sm_l[wave * G + n] = l_i;
  }
  if (n < G) {
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int i = 0; i < 4; ++i) sm_o[(wave * G + n) * D + 16 * nb + 4 * g + i] = o[nb][i];
  }
  __syncthreads();
  const int nparts = (seq_len + psz - 1) / psz;
  for (int idx = threadIdx.x; idx < G * D; idx += 256) {
    const int h = idx / D, d = idx % D;
    float M = OME_NEG_INF;
#pragma unroll
    for (int w = 0; w < 4; ++w) M = fmaxf(M, sm_m[w * G + h]);
    const float Mu = (M == OME_NEG_INF) ? 0.f : M;
    float L = 0.f, acc = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float f = fast_exp2(sm_m[w * G + h] - Mu);
      L += sm_l[w * G + h] * f;
      acc += sm_o[(w * G + h) * D + d] * f;
    }
    const int head = kvh * G + h;
    // attention sink (GPT-OSS): an extra softmax column with logit sinks[head] and no value
    if (sinks != nullptr && nparts == 1) L += fast_exp2(sinks[head] * 1.4426950408889634f - Mu);
    const float res = L > 0.f ? acc / L * v_scale : 0.f;
    if (nparts == 1) {
      out[(int64_t)b * out_stride + (int64_t)head * D + d] = (bf16)res;
    } else {
      const int64_t pidx = ((int64_t)b * Hq + head) * max_parts + part;
      part_o[pidx * D + d] = res;
      if (d == 0) {
        part_ml[pidx * 2 + 0] = M;
        part_ml[pidx * 2 + 1] = L;
      }
    }
  }
}

template <int D, int F>
static void launch_decode_v2(int variant, dim3 grid, size_t smem, hipStream_t stream, const void* q,
                             int64_t q_stride, const void* k_cache, const void* v_cache, const int* block_tables,
                             int bt_stride, const int* seq_lens, void* out, int64_t out_stride, void* part_o,
                             void* part_ml, int Hq, int Hkv, int part_size, int max_parts, Scaler scl,
                             int window, const int* order, float v_scale, const float* sinks) {
  // ALiBi (Bloom / MPT) runs the key-permuted variant only, compiled with the bias term; the
  // other instantiations carry no trace of it
  auto kern = (scl.alibi != nullptr || scl.bs_shift != 0) ? paged_decode_v2_kernel<D, 16, 2, F, true>
              : variant == 2       ? paged_decode_v2_kernel<D, 16, 1, F>
              : variant == 4       ? paged_decode_v2_kernel<D, 16, 2, F>
                                   : paged_decode_v2_kernel<D, 16, 0, F>;
  kern<<<grid, 256, smem, stream>>>((const bf16*)q, q_stride, (const typename KVStore<F>::T*)k_cache,
                                    (const typename KVStore<F>::T*)v_cache, block_tables, bt_stride, seq_lens,
                                    (bf16*)out, out_stride, (float*)part_o, (float*)part_ml, Hq, Hkv, part_size,
                                    max_parts, scl, window, order, v_scale, sinks);
}

// kv_fmt: KVFmt of the cache; k_scale / v_scale: per-layer dequantisation scales (1 for bf16);
// softcap: attention-logit soft-capping (Gemma-2), 0 = off.  Head dims 64 / 128 / 256.
template <int D>
static int decode_dispatch(int variant, int kv_fmt, dim3 grid, int B, hipStream_t stream, const void* q,
                           int64_t q_stride, const void* k_cache, const void* v_cache, const int* block_tables,
                           int bt_stride, const int* seq_lens, void* out, int64_t out_stride, void* part_o,
                           void* part_ml, int Hq, int Hkv, int part_size, int max_parts, Scaler scl, int window,
                           const int* order, float v_scale, const float* sinks) {
  const int G = Hq / Hkv;
  const size_t smem = (8 * G + 4 * G * D) * sizeof(float);
#define ARGS                                                                                                     \
  variant, grid, smem, stream, q, q_stride, k_cache, v_cache, block_tables, bt_stride, seq_lens, out, out_stride, \
      part_o, part_ml, Hq, Hkv, part_size, max_parts, scl, window, order, v_scale, sinks
  if (kv_fmt == KV_BF16) launch_decode_v2<D, KV_BF16>(ARGS);
  else if (kv_fmt == KV_E4M3) launch_decode_v2<D, KV_E4M3>(ARGS);
  else launch_decode_v2<D, KV_E5M2>(ARGS);
#undef ARGS
  OME_CHECK_LAUNCH();
  if (max_parts > 1) {
    paged_decode_reduce_kernel<D><<<dim3(Hq, B), D, 0, stream>>>(seq_lens, (const float*)part_o,
                                                                  (const float*)part_ml, (bf16*)out, out_stride, Hq,
                                                                  part_size, max_parts, sinks);
    OME_CHECK_LAUNCH();
  }
  return 0;
}

OME_API int ome_paged_decode(const void* q, int64_t q_stride, const void* k_cache, const void* v_cache,
                             const int* block_tables, int bt_stride, const int* seq_lens, void* out,
                             int64_t out_stride, void* part_o, void* part_ml, int B, int Hq, int Hkv, int D, int P,
                             int part_size, int max_parts, float scale, int window, const int* order, int kv_fmt,
                             float k_scale, float v_scale, float softcap, const float* sinks, const float* alibi,
                             const int* row_lo, int64_t bsparse, hipStream_t stream) {
  if (B <= 0) return 0;
  if ((D != 64 && D != 128 && D != 256) || P != 16) return -2;
  if (Hq % Hkv != 0 || Hq / Hkv > 16) return -3;
  if (part_size < 0 || part_size % 128 != 0 || max_parts <= 0) return -4;   // 0: per-sequence span
  if (kv_fmt < 0 || kv_fmt > 2) return -5;
  Scaler scl = make_scaler(scale * k_scale, softcap, alibi, bsparse);
  scl.row_lo = row_lo;
  dim3 grid(max_parts, Hkv, B);
  // A/B switch for benchmarking: 1 = v1, 2 = v2 (register ring), 3 = v2 without ring, 4 = v3 with
  // key-permuted tiles (16-B V loads; default: 5.38 vs 5.24 TB/s on the bench's context mix)
  const char* ve = getenv("OME_DECODE_ATTN");
  int variant = ve ? atoi(ve) : 4;
  if (variant == 1 && (kv_fmt != KV_BF16 || D != 128 || softcap > 0.f || sinks || alibi || row_lo || part_size == 0 ||
                       scl.bs_shift != 0))
    variant = 4;  // v1: plain bf16 D=128, fixed partitions
  if (variant == 1) {
    const size_t smem = (128 + 4 * 16 * D) * sizeof(float);
    paged_decode_kernel<128, 16><<<grid, 256, smem, stream>>>(
        (const bf16*)q, q_stride, (const bf16*)k_cache, (const bf16*)v_cache, block_tables, bt_stride, seq_lens,
        (bf16*)out, out_stride, (float*)part_o, (float*)part_ml, Hq, Hkv, part_size, max_parts, scl.mul, window);
    OME_CHECK_LAUNCH();
    if (max_parts > 1) {
      paged_decode_reduce_kernel<128><<<dim3(Hq, B), 128, 0, stream>>>(seq_lens, (const float*)part_o,
                                                                        (const float*)part_ml, (bf16*)out,
                                                                        out_stride, Hq, part_size, max_parts);
      OME_CHECK_LAUNCH();
    }
    return 0;
  }
#define ARGS                                                                                                      \
  variant, kv_fmt, grid, B, stream, q, q_stride, k_cache, v_cache, block_tables, bt_stride, seq_lens, out,         \
      out_stride, part_o, part_ml, Hq, Hkv, part_size, max_parts, scl, window, order, v_scale, sinks
  if (D == 64) return decode_dispatch<64>(ARGS);
  if (D == 256) return decode_dispatch<256>(ARGS);
  return decode_dispatch<128>(ARGS);
#undef ARGS
}

// ------------------------------------------------------------------------------------------
// Prefill: one workgroup = (work item, kv head).  A work item is 32 consecutive query rows of
// one sequence.  Each wave takes one query head of the kv group (wave w: heads w, w+8, ...),
// so the G waves of the workgroup stream the same K/V tiles (L1/L2 reuse across GQA heads).
// Queries at local row r sit at absolute position (kv_len - q_len + r): this covers fresh
// prompts (kv_len == q_len), chunked prefill and prefix-cache hits uniformly.
// ------------------------------------------------------------------------------------------
template <int D, int P, int F>
__global__ __launch_bounds__(512) void paged_prefill_kernel(
    const bf16* __restrict__ q, int64_t q_stride, const typename KVStore<F>::T* __restrict__ k_cache,
    const typename KVStore<F>::T* __restrict__ v_cache, const int* __restrict__ block_tables, int bt_stride,
    const int* __restrict__ cu_q, const int* __restrict__ kv_lens, const int2* __restrict__ items,
    bf16* __restrict__ out, int64_t out_stride, int Hq, int Hkv, Scaler scl, int window, float v_scale,
    const float* __restrict__ sinks, const int* __restrict__ row_hi) {
  static_assert(P == 16, "prefill kernel assumes 16-token pages");
  constexpr int NB = D / 16, KS = D / 32;
  const int2 it = items[blockIdx.x];
  const int s = it.x, r0 = it.y;
  const int kvh = blockIdx.y;
  const int q0 = cu_q[s];
  const int q_len = cu_q[s + 1] - q0;
  const int kv_len = kv_lens[s];
  const int prefix = kv_len - q_len;
  const int G = Hq / Hkv;
  const int nwaves = blockDim.x >> 6;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n = lane & 15, g = lane >> 4;
  const int r_hi = min(r0 + 32, q_len);
  // row_hi (optional, per query row): last visible key beyond the causal one (Gemma 3 image
  // blocks attend bidirectionally); keys up to the sequence end may then be visible
  const int kv_end = row_hi ? kv_len : min(kv_len, prefix + r_hi);
  int kv_lo = 0;
  kv_lo = attn_lo(prefix + r0, window) & ~31;
  const int* bt = block_tables + (int64_t)s * bt_stride;
  const int64_t kpage = (int64_t)Hkv * P * D;

  for (int hl = wave; hl < G; hl += nwaves) {
    const int head = kvh * G + hl;
    bf16x8 qf[2][KS];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      const int r = r0 + 16 * rb + n;
      const bf16* qr = q + (int64_t)(q0 + r) * q_stride + (int64_t)head * D;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) qf[rb][ks] = (r < q_len) ? ld8(qr + 32 * ks + 8 * g) : bf16x8{};
    }
    float m_i[2] = {OME_NEG_INF, OME_NEG_INF}, l_i[2] = {0.f, 0.f};
    const float al = scl.alibi_l2(head);
    f32x4 o[2][NB];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) o[rb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int kb = kv_lo; kb < kv_end; kb += 32) {
      const int pA = bt[kb / P];
      const int pB = (kb + P < kv_len) ? bt[kb / P + 1] : pA;
      const typename KVStore<F>::T* kA = k_cache + pA * kpage + (int64_t)kvh * P * D;
      const typename KVStore<F>::T* kB = k_cache + pB * kpage + (int64_t)kvh * P * D;
      f32x4 sc[2][2];
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) sc[rb][0] = sc[rb][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        bf16x8 a0 = kv_ld8<F>(kA + n * D + 32 * ks + 8 * g);
        bf16x8 a1 = kv_ld8<F>(kB + n * D + 32 * ks + 8 * g);
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
          sc[rb][0] = mfma16(a0, qf[rb][ks], sc[rb][0]);
          sc[rb][1] = mfma16(a1, qf[rb][ks], sc[rb][1]);
        }
      }
      const bool need_mask = (kb + 32 > prefix + r0 + 1) || (kb + 32 > kv_len) || (window > 0 || window < -1) ||
                             scl.bs_shift != 0;
      bf16x8 pb[2];
      float alpha[2];
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
        const int qpos = prefix + r0 + 16 * rb + n;
        const int qlim = row_hi ? max(qpos, row_hi[q0 + min(r0 + 16 * rb + n, q_len - 1)]) : qpos;
        float mt = OME_NEG_INF;
#pragma unroll
        for (int X = 0; X < 2; ++X)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float v = scl(sc[rb][X][i]);
            const int key = kb + 16 * X + 4 * g + i;
            if (al != 0.f) v += al * (float)(key - qpos);
            if (need_mask) {
              const bool ok = key <= qlim && key < kv_len && key >= attn_lo(qpos, window) &&
                               scl.bs_visible(qpos, key, head);
              v = ok ? v : OME_NEG_INF;
            }
            sc[rb][X][i] = v;
            mt = fmaxf(mt, v);
          }
        mt = group4_max(mt);
        const float m_new = fmaxf(m_i[rb], mt);
        const float m_use = (m_new == OME_NEG_INF) ? 0.f : m_new;
        alpha[rb] = fast_exp2(m_i[rb] - m_use);
        float rs = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float p0 = fast_exp2(sc[rb][0][i] - m_use), p1 = fast_exp2(sc[rb][1][i] - m_use);
          pb[rb][i] = (bf16)p0;
          pb[rb][4 + i] = (bf16)p1;
          rs += p0 + p1;
        }
        rs = group4_sum(rs);
        l_i[rb] = l_i[rb] * alpha[rb] + rs;
        m_i[rb] = m_new;
      }
      const typename KVStore<F>::T* vA = v_cache + pA * kpage + (int64_t)kvh * D * P;
      const typename KVStore<F>::T* vB = v_cache + pB * kpage + (int64_t)kvh * D * P;
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        const int dim = 16 * nb + n;
        bf16x8 a = cat44(kv_ld4<F>(vA + dim * P + 4 * g), kv_ld4<F>(vB + dim * P + 4 * g));
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
          o[rb][nb] = o[rb][nb] * alpha[rb];
          o[rb][nb] = mfma16(a, pb[rb], o[rb][nb]);
        }
      }
    }
    // ---- epilogue: normalise, store O[row][dims 16nb+4g .. +3] as bf16x4 ----
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      const int r = r0 + 16 * rb + n;
      if (r < q_len) {
        const float lt = sinks ? l_i[rb] + fast_exp2(sinks[head] * 1.4426950408889634f - m_i[rb]) : l_i[rb];
        const float inv = lt > 0.f ? v_scale / lt : 0.f;
        bf16* orow = out + (int64_t)(q0 + r) * out_stride + (int64_t)head * D;
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
          bf16x4 v;
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = (bf16)(o[rb][nb][i] * inv);
          *reinterpret_cast<bf16x4*>(orow + 16 * nb + 4 * g) = v;
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// Prefill v2 (G == 4): the workgroup's 4 waves share each 32-key K/V tile through LDS instead
// of each wave streaming it from L1/L2 (v1 was load-path bound: 4 waves x 16 KB per tile).
// Wave w takes head (w % G) of the kv group and row block (w / G): an item is 32*(4/G) query
// rows.  Tiles are double-buffered: the next tile's global loads are in flight while the
// current one is consumed from LDS.  LDS images (conflict-free for ds_read_b128):
//   K: [32 keys][128 dims + 8 pad]         (row = 272 B: 16 rows start on distinct bank quads)
//   V: [128 dims][32 keys + 8 pad], keys stored in the MFMA k-slot order of the S^T
//      accumulators (slot 8g+j: j<4 -> page A key 4g+j, j>=4 -> page B key 4g+j-4), so a
//      lane's A fragment of O^T = V^T P^T is one 16-B read.
// fp8 caches are staged raw in registers (8 B per chunk) and converted to bf16 on the LDS
// write, so the LDS images and the MFMA loop are identical for every cache format.
// ------------------------------------------------------------------------------------------
constexpr int PF_KLD = 128 + 8, PF_VLD = 32 + 8;

// SPLIT: the item's key range is cut into chunks of `chunk` keys run by separate workgroups
// (items4 = {seq, row0, chunk start, part}; part < 0 = the only chunk, written as final output).
// A short prefill (a few hundred keys per row) otherwise leaves most CUs idle and every
// workgroup latency-bound on its serial chain of K/V tile loads; partial (O, m, l) per part go
// to fp32 workspaces and prefill_combine_kernel merges them.
//
// FAST: plain causal attention (no soft-capping, ALiBi, window or row_hi) -- the Llama / Qwen /
// Mixtral prefill.  The generic per-score code (soft-cap select, ALiBi term, window and row_hi
// bounds, each a per-element branch) made the loop VALU-issue bound at ~3.3 us per 64-key step
// (8x the MFMA time, profiles/r03_prefill_attn_fast.txt).  The fast body keeps raw scores, masks
// only diagonal stages (key <= qpos also bounds kv_len), folds the scale into the exp2 FMA,
// keeps per-lane partial row sums (reduced across the row's 4 lanes once, at the end) and
// rescales O / l lazily (only when some row's max grew by more than 2^8).
// NW = waves per workgroup: 4 (one 32-row block per head of the kv group) or 8 (two row blocks:
// 64-row items, every K/V stage staged once for twice the query rows, one chunk per thread).
// PROBE (timing diagnostics, wrong results by design; OME_PREFILL_PROBE): 1 = no V image stores,
// 2 = no K/V global loads, 3 = identity pages (no block-table loads before the K/V loads).
// BS (FAST only): block-sparse layer -- skip the key stages no head of the kv group sees and mask
// this head's invisible keys (a separate instantiation: the dense kernels keep their registers).
template <int SUB, int F, bool SPLIT, bool FAST = false, int NW = 4, int PROBE = 0, bool BS = false>
__global__ __launch_bounds__(64 * NW, 8 / NW) void paged_prefill_v2_kernel(
    const bf16* __restrict__ q, int64_t q_stride, const typename KVStore<F>::T* __restrict__ k_cache,
    const typename KVStore<F>::T* __restrict__ v_cache, const int* __restrict__ block_tables, int bt_stride,
    const int* __restrict__ cu_q, const int* __restrict__ kv_lens, const int2* __restrict__ items,
    bf16* __restrict__ out, int64_t out_stride, int Hq, int Hkv, Scaler scl, int window, float v_scale,
    const float* __restrict__ sinks, const int* __restrict__ row_hi, int chunk, float* __restrict__ part_o,
    float* __restrict__ part_ml) {
  constexpr int D = 128, P = 16, NB = D / 16, KS = D / 32;
  typedef typename KVRaw<F>::K8 Raw8;  // 8 consecutive cache elements
  __shared__ __attribute__((aligned(16))) bf16 sK[2][SUB][32 * PF_KLD];
  __shared__ __attribute__((aligned(16))) bf16 sV[2][SUB][D * PF_VLD];
  int s, r0_item, c_lo = 0, part = -1;
  if constexpr (SPLIT) {
    const int4 it4 = reinterpret_cast<const int4*>(items)[blockIdx.x];
    s = it4.x, r0_item = it4.y, c_lo = it4.z, part = it4.w;
  } else {
    const int2 it = items[blockIdx.x];
    s = it.x, r0_item = it.y;
  }
  const int kvh = blockIdx.y;
  const int q0 = cu_q[s];
  const int q_len = cu_q[s + 1] - q0;
  const int kv_len = kv_lens[s];
  const int prefix = kv_len - q_len;
  const int G = Hq / Hkv;
  static_assert(NW == 4 || NW == 8, "NW");
  static_assert(!SPLIT || NW == 4, "split partials are laid out for 4 waves");
  constexpr int PT = 2 * 4 / NW;   // K (and V) chunks of 8 elements per thread per 32-key subtile
  const int rows_per_item = 32 * (NW / G);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int n = lane & 15, g = lane >> 4;
  const int hl = wave % G, rblk = wave / G;
  const int head = kvh * G + hl;
  const int r0 = r0_item + 32 * rblk;
  const int item_hi = min(r0_item + rows_per_item, q_len);
  int kv_end = row_hi ? kv_len : min(kv_len, prefix + item_hi);
  int kv_lo = 0;
  kv_lo = attn_lo(prefix + r0_item, window) & ~31;
  if constexpr (SPLIT) {   // chunk starts are multiples of 64 keys: kv_lo stays 32-aligned
    kv_lo = max(kv_lo, c_lo);
    kv_end = min(kv_end, c_lo + chunk);
  }
  const int* bt = block_tables + (int64_t)s * bt_stride;
  const int64_t kpage = (int64_t)Hkv * P * D;

  // ---- per-wave query fragments (rows r0 .. r0+31 of `head`) ----
  bf16x8 qf[2][KS];
#pragma unroll
  for (int rb = 0; rb < 2; ++rb) {
    const int r = r0 + 16 * rb + n;
    const bf16* qr = q + (int64_t)(q0 + r) * q_stride + (int64_t)head * D;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[rb][ks] = (r < q_len) ? ld8(qr + 32 * ks + 8 * g) : bf16x8{};
  }
  float m_i[2] = {OME_NEG_INF, OME_NEG_INF}, l_i[2] = {0.f, 0.f};
  const float al = scl.alibi_l2(head);
  f32x4 o[2][NB];
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) o[rb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- cooperative tile staging: per 32-key subtile, 2 x 8 elements of K and 2 x 8 of V per
  // thread; a pipeline stage is SUB subtiles (32*SUB keys), so SUB x more bytes are in flight ----
  // Two register stages (A, B) in flight: a tile's global loads are issued two compute phases
  // before its LDS write, so each load has ~2 x (64 MFMA + softmax) per wave to land.  With one
  // stage the loop was latency-bound at ~3.9 us per 64-key step (profiles/r03_prefill_*).
  Raw8 rkA[SUB][PT], rvA[SUB][PT], rkB[SUB][PT], rvB[SUB][PT];
  auto load_tile = [&](Raw8 (&rk)[SUB][PT], Raw8 (&rv)[SUB][PT], int kb0) {
    if constexpr (PROBE == 2) {
#pragma unroll
      for (int u = 0; u < SUB; ++u)
#pragma unroll
        for (int i = 0; i < PT; ++i) asm volatile("" : "+v"(rk[u][i]), "+v"(rv[u][i]));
      return;
    }
#pragma unroll
    for (int u = 0; u < SUB; ++u) {
      const int kb = kb0 + 32 * u;
      const int pi = kb / P;
      const int pA = PROBE == 3 ? pi : (kb < kv_len) ? bt[pi] : bt[0];  // out-of-range subtiles: any valid page (masked)
      const int pB = PROBE == 3 ? pi + 1 : (kb + P < kv_len) ? bt[pi + 1] : pA;
#pragma unroll
      for (int i = 0; i < PT; ++i) {
        const int c = tid + 64 * NW * i;
        const int key = c >> 4, dc = c & 15;
        const typename KVStore<F>::T* kp = k_cache + (key < 16 ? pA : pB) * kpage + (int64_t)kvh * P * D;
        rk[u][i] = k8_load<F>(kp + (key & 15) * D + dc * 8);
        const int page = c >> 8, dim = (c & 255) >> 1, half = c & 1;
        const typename KVStore<F>::T* vp = v_cache + (page ? pB : pA) * kpage + (int64_t)kvh * D * P;
        rv[u][i] = k8_load<F>(vp + dim * P + half * 8);
      }
    }
  };
  auto store_tile = [&](const Raw8 (&rk)[SUB][PT], const Raw8 (&rv)[SUB][PT], int buf) {
#pragma unroll
    for (int u = 0; u < SUB; ++u)
#pragma unroll
      for (int i = 0; i < PT; ++i) {
        const int c = tid + 64 * NW * i;
        const int key = c >> 4, dc = c & 15;
        *reinterpret_cast<bf16x8*>(&sK[buf][u][key * PF_KLD + dc * 8]) = k8_bf16<F>(rk[u][i]);
        if constexpr (PROBE == 1) {
          asm volatile("" ::"v"(rv[u][i]));
          continue;
        }
        const int page = c >> 8, dim = (c & 255) >> 1, half = c & 1;
        bf16* vrow = &sV[buf][u][dim * PF_VLD];
        const bf16x8 vv = k8_bf16<F>(rv[u][i]);
        bf16x4 lo4 = {vv[0], vv[1], vv[2], vv[3]};
        bf16x4 hi4 = {vv[4], vv[5], vv[6], vv[7]};
        *reinterpret_cast<bf16x4*>(vrow + (2 * half) * 8 + page * 4) = lo4;      // keys 8h..8h+3
        *reinterpret_cast<bf16x4*>(vrow + (2 * half + 1) * 8 + page * 4) = hi4;  // keys 8h+4..8h+7
      }
  };

  const bool active = r0 < q_len;  // a wave whose rows are all past q_len still stages tiles
  auto compute = [&](int buf, int kb) {
    if (!active) return;
#pragma unroll
    for (int u = 0; u < SUB; ++u) {
      const int kbu = kb + 32 * u;
      if (kbu < kv_end) {
        f32x4 sc[2][2];
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) sc[rb][0] = sc[rb][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(&sK[buf][u][n * PF_KLD + 32 * ks + 8 * g]);
          const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(&sK[buf][u][(16 + n) * PF_KLD + 32 * ks + 8 * g]);
#pragma unroll
          for (int rb = 0; rb < 2; ++rb) {
            sc[rb][0] = mfma16(a0, qf[rb][ks], sc[rb][0]);
            sc[rb][1] = mfma16(a1, qf[rb][ks], sc[rb][1]);
          }
        }
        bf16x8 pb[2];
        float alpha[2];
        const bool need_mask =
            (kbu + 32 > prefix + r0 + 1) || (kbu + 32 > kv_len) || (window > 0 || window < -1) ||
            scl.bs_shift != 0;
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
          const int qpos = prefix + r0 + 16 * rb + n;
          const int qlim = row_hi ? max(qpos, row_hi[q0 + min(r0 + 16 * rb + n, q_len - 1)]) : qpos;
          float mt = OME_NEG_INF;
#pragma unroll
          for (int X = 0; X < 2; ++X)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              float v = scl(sc[rb][X][i]);
              const int key = kbu + 16 * X + 4 * g + i;
              if (al != 0.f) v += al * (float)(key - qpos);
              if (need_mask) {
                const bool ok = key <= qlim && key < kv_len && key >= attn_lo(qpos, window) &&
                               scl.bs_visible(qpos, key, head);
                v = ok ? v : OME_NEG_INF;
              }
              sc[rb][X][i] = v;
              mt = fmaxf(mt, v);
            }
          mt = group4_max(mt);
          const float m_new = fmaxf(m_i[rb], mt);
          const float m_use = (m_new == OME_NEG_INF) ? 0.f : m_new;
          alpha[rb] = fast_exp2(m_i[rb] - m_use);
          float rs = 0.f;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float p0 = fast_exp2(sc[rb][0][i] - m_use), p1 = fast_exp2(sc[rb][1][i] - m_use);
            pb[rb][i] = (bf16)p0;
            pb[rb][4 + i] = (bf16)p1;
            rs += p0 + p1;
          }
          rs = group4_sum(rs);
          l_i[rb] = l_i[rb] * alpha[rb] + rs;
          m_i[rb] = m_new;
        }
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
          const bf16x8 a = *reinterpret_cast<const bf16x8*>(&sV[buf][u][(16 * nb + n) * PF_VLD + 8 * g]);
#pragma unroll
          for (int rb = 0; rb < 2; ++rb) {
            o[rb][nb] = o[rb][nb] * alpha[rb];
            o[rb][nb] = mfma16(a, pb[rb], o[rb][nb]);
          }
        }
      }
    }
  };

  // FAST body: one online-softmax update per 32*SUB-key stage (one max reduction, one O
  // rescale) instead of per 32-key subtile.  Subtiles past kv_end are skipped in both MFMA
  // passes and their scores set to -inf here, so they never enter l whatever the alignment of
  // kv_lo / the split chunk start (the diagonal mask alone covers them only while stages are
  // 64-aligned to the causal limit).
  auto compute_fast = [&](int buf, int kb) __attribute__((always_inline)) {
    if (!active) return;
    f32x4 sc[SUB][2][2];
#pragma unroll
    for (int u = 0; u < SUB; ++u) {
      const float s0 = kb + 32 * u < kv_end ? 0.f : OME_NEG_INF;
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) sc[u][rb][0] = sc[u][rb][1] = f32x4{s0, s0, s0, s0};
      if (kb + 32 * u < kv_end) {
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(&sK[buf][u][n * PF_KLD + 32 * ks + 8 * g]);
          const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(&sK[buf][u][(16 + n) * PF_KLD + 32 * ks + 8 * g]);
#pragma unroll
          for (int rb = 0; rb < 2; ++rb) {
            sc[u][rb][0] = mfma16(a0, qf[rb][ks], sc[u][rb][0]);
            sc[u][rb][1] = mfma16(a1, qf[rb][ks], sc[u][rb][1]);
          }
        }
      }
    }
    if (BS && !scl.bs_stage_full(kb, 32 * SUB, (prefix + r0 + 31) >> scl.bs_shift, head)) {
      // block-sparse: this head's invisible keys of the stage.  Blocks are >= 32 * SUB keys (host
      // check), so the stage spans blocks b0 and at most b1 = b0 + 1, split at key offset `cut`;
      // visibility is per (row, block): local band or this head's stripe
      asm volatile("" ::: "memory");
      const int b0 = kb >> scl.bs_shift, b1 = (kb + 32 * SUB - 1) >> scl.bs_shift;
      const int cut = (b1 << scl.bs_shift) - kb;   // first key offset in b1 (b1 == b0: >= stage)
      const bool st0 = scl.bs_stripe(b0, head), st1 = scl.bs_stripe(b1, head);
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
        const int qb = (prefix + r0 + 16 * rb + n) >> scl.bs_shift;
        const bool v0 = st0 || qb - b0 < scl.bs_local, v1 = st1 || qb - b1 < scl.bs_local;
#pragma unroll
        for (int u = 0; u < SUB; ++u)
#pragma unroll
          for (int X = 0; X < 2; ++X)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int off = 32 * u + 16 * X + 4 * g + i;
              if (!((off < cut || b1 == b0) ? v0 : v1)) sc[u][rb][X][i] = OME_NEG_INF;
            }
      }
    }
    const bool diag = kb + 32 * SUB > prefix + r0 + 1;   // wave-uniform
    if (diag) {   // only the diagonal stage masks (a real branch: the asm keeps it from being speculated)
      asm volatile("" ::: "memory");
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
        const int lim = prefix + r0 + 16 * rb + n - kb;   // last visible key offset of this row
#pragma unroll
        for (int u = 0; u < SUB; ++u)
#pragma unroll
          for (int X = 0; X < 2; ++X)
#pragma unroll
            for (int i = 0; i < 4; ++i)
              if (32 * u + 16 * X + 4 * g + i > lim) sc[u][rb][X][i] = OME_NEG_INF;
      }
    }
    float mt[2];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      float v = OME_NEG_INF;
#pragma unroll
      for (int u = 0; u < SUB; ++u)
#pragma unroll
        for (int X = 0; X < 2; ++X)
#pragma unroll
          for (int i = 0; i < 4; ++i) v = fmaxf(v, sc[u][rb][X][i]);
      mt[rb] = group4_max(v) * scl.mul;   // log2 domain
    }
    // lazy rescale (FA-3 style): keep the running max while no row of the wave grew it by more
    // than 8 (p <= 2^8 then, exact in fp32 and bf16's range); O and l are rescaled only on the
    // stages where some row did -- the first stage always, afterwards rarely
    const bool grow = __ballot(mt[0] > m_i[0] + 8.f || mt[1] > m_i[1] + 8.f) != 0;
    if (grow) {
      asm volatile("" ::: "memory");
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
        const float m_new = fmaxf(m_i[rb], mt[rb]);
        const float m_use = (m_new == OME_NEG_INF) ? 0.f : m_new;
        const float alpha = fast_exp2(m_i[rb] - m_use);
        l_i[rb] *= alpha;
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) o[rb][nb] = o[rb][nb] * alpha;
        m_i[rb] = m_new;
      }
    }
    bf16x8 pb[SUB][2];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      const float m_use = (m_i[rb] == OME_NEG_INF) ? 0.f : m_i[rb];
      float rs = 0.f;
#pragma unroll
      for (int u = 0; u < SUB; ++u)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float p0 = fast_exp2(__builtin_fmaf(sc[u][rb][0][i], scl.mul, -m_use));
          const float p1 = fast_exp2(__builtin_fmaf(sc[u][rb][1][i], scl.mul, -m_use));
          pb[u][rb][i] = (bf16)p0;
          pb[u][rb][4 + i] = (bf16)p1;
          rs += p0 + p1;
        }
      l_i[rb] += rs;   // this lane's partial row sum
    }
#pragma unroll
    for (int u = 0; u < SUB; ++u) {
      if (kb + 32 * u < kv_end) {
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
          const bf16x8 a = *reinterpret_cast<const bf16x8*>(&sV[buf][u][(16 * nb + n) * PF_VLD + 8 * g]);
#pragma unroll
          for (int rb = 0; rb < 2; ++rb) o[rb][nb] = mfma16(a, pb[u][rb], o[rb][nb]);
        }
      }
    }
  };
  auto step = [&](int buf, int kb) __attribute__((always_inline)) {
    if constexpr (FAST) compute_fast(buf, kb);
    else compute(buf, kb);
  };

  constexpr int STEP = 32 * SUB;
  // the stages this workgroup runs: every STEP-key stage from kv_lo, except (block-sparse) stages
  // that no query row of the item and no head of the kv group sees -- skipped before their loads,
  // so a sparse layer costs its visible tiles only.  Dense: nxt(k) == k.
  auto nxt = [&](int k) __attribute__((always_inline)) {
    if constexpr (BS) {
      const int qb_lo = (prefix + r0_item) >> scl.bs_shift;   // the item's first query row
      if (scl.bs_skip)
        while (k < kv_end && !scl.bs_stage_needed(k, STEP, qb_lo, kvh * G, G)) k += STEP;
    }
    return k;
  };
  int kb = nxt(kv_lo);
  int kB = kb < kv_end ? nxt(kb + STEP) : kv_end;
  if (kb < kv_end) {
    load_tile(rkA, rvA, kb);
    if (kB < kv_end) load_tile(rkB, rvB, kB);
    store_tile(rkA, rvA, 0);
  }
  __syncthreads();
  int kC = kB < kv_end ? nxt(kB + STEP) : kv_end;
  if (kC < kv_end) load_tile(rkA, rvA, kC);
  // invariant at the top: LDS buf 0 = stage kb, registers B = stage kB, A = stage kC (the next
  // needed stages in order; dense: kb + STEP, kb + 2 STEP)
  while (kb < kv_end) {
    step(0, kb);
    if (kB < kv_end) store_tile(rkB, rvB, 1);
    __syncthreads();
    if (kB >= kv_end) break;
    const int kD = kC < kv_end ? nxt(kC + STEP) : kv_end;
    if (kD < kv_end) load_tile(rkB, rvB, kD);
    step(1, kB);
    if (kC < kv_end) store_tile(rkA, rvA, 0);
    __syncthreads();
    const int kE = kD < kv_end ? nxt(kD + STEP) : kv_end;
    if (kE < kv_end) load_tile(rkA, rvA, kE);
    kb = kC;
    kB = kD;
    kC = kE;
  }
  if (!active) return;
  if constexpr (FAST) {   // per-lane partial row sums -> the row's total (its 4 lane groups)
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      l_i[rb] = group4_sum(l_i[rb]);
    }
  }
  if (SPLIT && part >= 0) {   // unnormalised partial: O^T rows of this wave + (m, l) per row
    const int64_t pw = ((int64_t)part * Hkv + kvh) * 4 + wave;
    float* po = part_o + pw * 32 * D;
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      const int row = 16 * rb + n;
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) *reinterpret_cast<f32x4*>(po + row * D + 16 * nb + 4 * g) = o[rb][nb];
      if (g == 0) *reinterpret_cast<float2*>(part_ml + (pw * 32 + row) * 2) = make_float2(m_i[rb], l_i[rb]);
    }
    return;
  }
#pragma unroll
  for (int rb = 0; rb < 2; ++rb) {
    const int r = r0 + 16 * rb + n;
    if (r < q_len) {
      const float lt = sinks ? l_i[rb] + fast_exp2(sinks[head] * 1.4426950408889634f - m_i[rb]) : l_i[rb];
      const float inv = lt > 0.f ? v_scale / lt : 0.f;
      bf16* orow = out + (int64_t)(q0 + r) * out_stride + (int64_t)head * D;
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        bf16x4 v;
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = (bf16)(o[rb][nb][i] * inv);
        *reinterpret_cast<bf16x4*>(orow + 16 * nb + 4 * g) = v;
      }
    }
  }
}

// Merge the split-KV partials of paged_prefill_v2_kernel<SPLIT>: comb = {seq, row0, first part,
// parts}.  grid (4 x combine items, Hq): block = 8 query rows x 32 lanes of 4 dims for one head,
// every thread independent (no serial row loop), part loop unrolled so loads overlap.
__global__ __launch_bounds__(256) void prefill_combine_kernel(const int4* __restrict__ comb,
                                                              const int* __restrict__ cu_q,
                                                              const float* __restrict__ part_o,
                                                              const float* __restrict__ part_ml,
                                                              bf16* __restrict__ out, int64_t out_stride, int Hkv,
                                                              float v_scale, const float* __restrict__ sinks) {
  constexpr int D = 128;
  const int4 c = comb[blockIdx.x >> 2];
  const int s = c.x, p0 = c.z, np = c.w;
  const int head = blockIdx.y, kvh = head >> 2, w = head & 3;
  const int r = 8 * (blockIdx.x & 3) + (threadIdx.x >> 5), quad = threadIdx.x & 31;
  const int q0 = cu_q[s], q_len = cu_q[s + 1] - q0;
  const int row = c.y + r;
  if (row >= q_len) return;
  const float sink = sinks ? sinks[head] * 1.4426950408889634f : OME_NEG_INF;
  auto pw_of = [&](int p) -> int64_t { return ((int64_t)(p0 + p) * Hkv + kvh) * 4 + w; };
  float M = sink;
#pragma unroll 4
  for (int p = 0; p < np; ++p) M = fmaxf(M, part_ml[(pw_of(p) * 32 + r) * 2]);
  const float Mu = M == OME_NEG_INF ? 0.f : M;
  float L = sinks ? fast_exp2(sink - Mu) : 0.f;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int p = 0; p < np; ++p) {
    const int64_t pw = pw_of(p);
    const float2 ml = *reinterpret_cast<const float2*>(part_ml + (pw * 32 + r) * 2);
    const f32x4 ov = *reinterpret_cast<const f32x4*>(part_o + (pw * 32 + r) * D + 4 * quad);
    const float wt = fast_exp2(ml.x - Mu);
    L += wt * ml.y;
    acc += wt * ov;
  }
  const float inv = L > 0.f ? v_scale / L : 0.f;
  bf16x4 v;
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = (bf16)(acc[i] * inv);
  *reinterpret_cast<bf16x4*>(out + (int64_t)(q0 + row) * out_stride + (int64_t)head * D + 4 * quad) = v;
}

// the FAST body of paged_prefill_v2_kernel applies: causal (block-sparse included: its per-head
// mask runs on the stages a head does not fully see) -- OME_PREFILL_FAST=0 forces the generic
// body, for A/B runs
static bool prefill_fast(const Scaler& scl, int window, const int* row_hi) {
  static const bool off = [] {
    const char* e = getenv("OME_PREFILL_FAST");
    return e && atoi(e) == 0;
  }();
  return !off && scl.cap_inv == 0.f && scl.alibi == nullptr && row_hi == nullptr &&
         (window == -1 || window == 0);
}

template <int D, int F>
static void launch_prefill(int variant, int rows, int G, dim3 grid, hipStream_t stream, const void* q, int64_t q_stride,
                           const void* k_cache, const void* v_cache, const int* block_tables, int bt_stride,
                           const int* cu_q, const int* kv_lens, const int* items, void* out, int64_t out_stride,
                           int Hq, int Hkv, Scaler scl, int window, float v_scale, const float* sinks,
                           const int* row_hi) {
  typedef typename KVStore<F>::T T;
  if constexpr (D == 128) {
    if (variant == 2 && G == 4) {  // one head per wave over 32-row items (GQA-4: Llama-3, Qwen3, Mixtral)
#define OME_PF2B(FAST, NW, BS)                                                                                    \
  paged_prefill_v2_kernel<2, F, false, FAST, NW, 0, BS><<<grid, 64 * NW, 0, stream>>>(                            \
      (const bf16*)q, q_stride, (const T*)k_cache, (const T*)v_cache, block_tables, bt_stride, cu_q, kv_lens,      \
      (const int2*)items, (bf16*)out, out_stride, Hq, Hkv, scl, window, v_scale, sinks, row_hi, 0, nullptr, nullptr)
#define OME_PF2(FAST, NW) OME_PF2B(FAST, NW, false)
      const bool bs = scl.bs_shift != 0;   // BS kernels need blocks >= 64 keys (else: generic body, mask only)
      const bool bs_fast = bs && scl.bs_shift >= 6 && prefill_fast(scl, window, row_hi);
      if (rows == 64) {   // 8 waves over 64-row items
        if (bs_fast) OME_PF2B(true, 8, true);
        else if (!bs && prefill_fast(scl, window, row_hi)) OME_PF2(true, 8);
        else OME_PF2(false, 8);
      } else if (bs_fast) {
        OME_PF2B(true, 4, true);
      } else {
        static const int probe = getenv("OME_PREFILL_PROBE") ? atoi(getenv("OME_PREFILL_PROBE")) : 0;
        if (!bs && prefill_fast(scl, window, row_hi)) {
#define OME_PF2P(PR)                                                                                              \
  paged_prefill_v2_kernel<2, F, false, true, 4, PR><<<grid, 256, 0, stream>>>(                                    \
      (const bf16*)q, q_stride, (const T*)k_cache, (const T*)v_cache, block_tables, bt_stride, cu_q, kv_lens,      \
      (const int2*)items, (bf16*)out, out_stride, Hq, Hkv, scl, window, v_scale, sinks, row_hi, 0, nullptr, nullptr)
          bool done = false;
          if constexpr (F == KV_BF16) {   // diagnostic instantiations for the bf16 cache only
            done = probe >= 1 && probe <= 3;
            if (probe == 1) OME_PF2P(1);
            else if (probe == 2) OME_PF2P(2);
            else if (probe == 3) OME_PF2P(3);
          }
          if (!done) OME_PF2(true, 4);
#undef OME_PF2P
        } else {
          OME_PF2(false, 4);
        }
      }
#undef OME_PF2
#undef OME_PF2B
      return;
    }
  }
  const int nw = G < 8 ? G : 8;
  paged_prefill_kernel<D, 16, F><<<grid, 64 * nw, 0, stream>>>(
      (const bf16*)q, q_stride, (const T*)k_cache, (const T*)v_cache, block_tables, bt_stride, cu_q, kv_lens,
      (const int2*)items, (bf16*)out, out_stride, Hq, Hkv, scl, window, v_scale, sinks, row_hi);
}

template <int D>
static void prefill_dispatch(int kv_fmt, int variant, int rows, int G, dim3 grid, hipStream_t stream, const void* q,
                             int64_t q_stride, const void* k_cache, const void* v_cache, const int* block_tables,
                             int bt_stride, const int* cu_q, const int* kv_lens, const int* items, void* out,
                             int64_t out_stride, int Hq, int Hkv, Scaler scl, int window, float v_scale,
                             const float* sinks, const int* row_hi) {
#define ARGS                                                                                                   \
  variant, rows, G, grid, stream, q, q_stride, k_cache, v_cache, block_tables, bt_stride, cu_q, kv_lens, items, \
      out, out_stride, Hq, Hkv, scl, window, v_scale, sinks, row_hi
  if (kv_fmt == KV_BF16) launch_prefill<D, KV_BF16>(ARGS);
  else if (kv_fmt == KV_E4M3) launch_prefill<D, KV_E4M3>(ARGS);
  else launch_prefill<D, KV_E5M2>(ARGS);
#undef ARGS
}

OME_API int ome_paged_prefill(const void* q, int64_t q_stride, const void* k_cache, const void* v_cache,
                              const int* block_tables, int bt_stride, const int* cu_q, const int* kv_lens,
                              const int* items, int n_items, void* out, int64_t out_stride, int Hq, int Hkv, int D,
                              int P, float scale, int window, int kv_fmt, float k_scale, float v_scale,
                              float softcap, const float* sinks, const float* alibi, const int* row_hi,
                              int rows, int64_t bsparse, hipStream_t stream) {
  if (n_items <= 0) return 0;
  if (rows != 32 && rows != 64) return -2;
  if ((D != 64 && D != 128 && D != 256) || P != 16) return -2;
  if (Hq % Hkv != 0) return -3;
  if (kv_fmt < 0 || kv_fmt > 2) return -5;
  const int G = Hq / Hkv;
  const Scaler scl = make_scaler(scale * k_scale, softcap, alibi, bsparse);
  dim3 grid(n_items, Hkv);
  const char* ve = getenv("OME_PREFILL_ATTN");
  const int variant = ve ? atoi(ve) : 2;
  // 64-row items exist only for the 8-wave GQA-4 / D = 128 kernel; every other kernel would
  // treat them as 32-row items and silently skip rows 32..63
  if (rows == 64 && !(D == 128 && variant == 2 && G == 4)) return -2;
#define ARGS                                                                                                     \
  kv_fmt, variant, rows, G, grid, stream, q, q_stride, k_cache, v_cache, block_tables, bt_stride, cu_q, kv_lens,  \
      items, out, out_stride, Hq, Hkv, scl, window, v_scale, sinks, row_hi
  if (D == 64) prefill_dispatch<64>(ARGS);
  else if (D == 256) prefill_dispatch<256>(ARGS);
  else prefill_dispatch<128>(ARGS);
#undef ARGS
  OME_CHECK_LAUNCH();
  return 0;
}

// Split-KV prefill (D = 128, P = 16, G = Hq / Hkv = 4, no row_hi): items4 [n_items][4], comb
// [n_comb][4]; part_o [parts][Hkv][4][32][128] and part_ml [parts][Hkv][4][32][2] fp32 workspaces.
OME_API int ome_paged_prefill_split(const void* q, int64_t q_stride, const void* k_cache, const void* v_cache,
                                    const int* block_tables, int bt_stride, const int* cu_q, const int* kv_lens,
                                    const int* items4, int n_items, const int* comb, int n_comb, int chunk,
                                    void* part_o, void* part_ml, void* out, int64_t out_stride, int Hq, int Hkv,
                                    float scale, int window, int kv_fmt, float k_scale, float v_scale, float softcap,
                                    const float* sinks, const float* alibi, int64_t bsparse, hipStream_t stream) {
  if (n_items <= 0) return 0;
  if (Hq != 4 * Hkv || chunk % 64 || kv_fmt < 0 || kv_fmt > 2) return -2;
  const Scaler scl = make_scaler(scale * k_scale, softcap, alibi, bsparse);
  dim3 grid(n_items, Hkv);
#define OME_PFS(F, FAST)                                                                                       \
  if (FAST && scl.bs_shift >= 6)                                                                               \
    paged_prefill_v2_kernel<2, F, true, FAST, 4, 0, FAST><<<grid, 256, 0, stream>>>(                           \
        (const bf16*)q, q_stride, (const typename KVStore<F>::T*)k_cache,                                      \
        (const typename KVStore<F>::T*)v_cache, block_tables, bt_stride, cu_q, kv_lens, (const int2*)items4,   \
        (bf16*)out, out_stride, Hq, Hkv, scl, window, v_scale, sinks, nullptr, chunk, (float*)part_o,          \
        (float*)part_ml);                                                                                      \
  else                                                                                                         \
  paged_prefill_v2_kernel<2, F, true, FAST><<<grid, 256, 0, stream>>>(                                         \
      (const bf16*)q, q_stride, (const typename KVStore<F>::T*)k_cache, (const typename KVStore<F>::T*)v_cache, \
      block_tables, bt_stride, cu_q, kv_lens, (const int2*)items4, (bf16*)out, out_stride, Hq, Hkv, scl, window,  \
      v_scale, sinks, nullptr, chunk, (float*)part_o, (float*)part_ml)
  // block-sparse with blocks < 64 keys: generic body (mask only)
  const bool fast = prefill_fast(scl, window, nullptr) && (scl.bs_shift == 0 || scl.bs_shift >= 6);
  if (kv_fmt == KV_BF16) {
    if (fast) OME_PFS(KV_BF16, true);
    else OME_PFS(KV_BF16, false);
  } else if (kv_fmt == KV_E4M3) {
    if (fast) OME_PFS(KV_E4M3, true);
    else OME_PFS(KV_E4M3, false);
  } else {
    if (fast) OME_PFS(KV_E5M2, true);
    else OME_PFS(KV_E5M2, false);
  }
#undef OME_PFS
  OME_CHECK_LAUNCH();
  if (n_comb > 0) {
    prefill_combine_kernel<<<dim3(4 * n_comb, Hq), 256, 0, stream>>>((const int4*)comb, cu_q, (const float*)part_o,
                                                                  (const float*)part_ml, (bf16*)out, out_stride, Hkv,
                                                                  v_scale, sinks);
    OME_CHECK_LAUNCH();
  }
  return 0;
}
