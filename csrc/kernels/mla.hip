// Multi-head latent attention (DeepSeek-V2/V3, Kimi-K2) in the absorbed
// form, for gfx950.
//
// Every layer caches one latent row per token: [c_kv (kv_lora_rank, kv_a_layernorm'd) | k_pe
// (roped)], paged as cache[pages, 16, DK] bf16 -- DK = 576 = 512 + 64 for DeepSeek-V2/V3 / Kimi-K2,
// 288 = 256 + 32 for MiniCPM3 (template instances below).  With W_UK folded into the query
// (q_lat = [q_nope . W_UK | q_pe], 576 wide) and W_UV applied after the attention, MLA is
// multi-QUERY attention over that latent: scores use all 576 dims, values are the first 512.
// The same kernel serves decode, prefill and chunked prefill: a work item is one query token
// x 16 heads (every head of a token shares the causal limit) x one split-K partition.
//
// Workgroup = 4 waves: all four compute S^T for the same 16 heads x 32 keys (the K tile is
// staged once in LDS and read by all), and each wave owns 128 of the 512 value dims.
//   S^T = K . Q^T     v_mfma_f32_16x16x32_bf16, A = K rows from LDS (ds_read_b128),
//                     B = Q held in registers (18 k-steps of 32 dims)
//   O^T += V^T . P^T  A = V^T from the SAME LDS image via ds_read_b64_tr_b16 (hardware
//                     transpose, cdna_hip_programming.md T10), B = P^T straight from the S^T
//                     accumulators in the permuted k-slot order of attention.hip
// LDS rows are 1152 B (72 x 16-B chunks); chunk x of key row r lives at x ^ (r & 7), which
// spreads both the row reads and the transposed reads over the banks.
#include "common.h"

#include <cstdlib>

#ifndef OME_NEG_INF
#define OME_NEG_INF (-__builtin_inff())
#endif

namespace {

constexpr int KT = 32;   // keys per iteration (two 16-token pages)
typedef short s16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma16x32(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// LDS row stride in 16-byte chunks, padded to a multiple of 8 so the xor swizzle stays in the row
template <int DK>
constexpr int lds_chunks() { return ((DK / 8) + 7) / 8 * 8; }
template <int DK>
__device__ __forceinline__ int swz(int row, int chunk) { return row * lds_chunks<DK>() + (chunk ^ (row & 7)); }

__device__ __forceinline__ bf16x4 tr_read(const bf16* lds_base, int byte_off) {
  const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (s16x4 __attribute__((address_space(3)))*)((__attribute__((address_space(3))) char*)(
          (__attribute__((address_space(3))) bf16*)lds_base) + byte_off));
  return __builtin_bit_cast(bf16x4, v);
}

}  // namespace

template <int DK, int DV>
__global__ __launch_bounds__(256) void mla_attn_kernel(
    const bf16* __restrict__ q, int64_t q_stride_t, const bf16* __restrict__ cache,
    const int* __restrict__ block_tables, int bt_stride, const int* __restrict__ tok_row,
    const int* __restrict__ kv_lens, int H, float scale_log2, int parts, bf16* __restrict__ out,
    int64_t out_stride_t, float* __restrict__ ws_o, float* __restrict__ ws_ml) {
  constexpr int CH = DK / 8, NB = DV / 64, NST = (KT * CH + 255) / 256;   // NB 16-dim blocks per wave
  __shared__ __attribute__((aligned(16))) bf16 sK[KT * lds_chunks<DK>() * 8];
  const int t = blockIdx.x, h0 = blockIdx.y * 16, part = blockIdx.z;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int col = lane & 15, g = lane >> 4;
  const int L = kv_lens[t];
  const int n_pages = (L + 15) >> 4;
  const int pairs = (n_pages + 1) >> 1;
  const int per_part = (pairs + parts - 1) / parts;
  const int pair_begin = part * per_part, pair_end = min(pairs, pair_begin + per_part);
  const int* bt = block_tables + (int64_t)tok_row[t] * bt_stride;
  const int64_t ws_row = ((int64_t)t * H + h0 + col) * parts + part;

  const bool hv = h0 + col < H;   // head groups are 16 wide; the last may be partial (MiniCPM3: 40)

  // ---- Q^T operand: lane (col, g) holds Q[h0+col][32 s + 8 g + j] ----
  bf16x8 qf[DK / 32];
  const bf16* qp = q + (int64_t)t * q_stride_t + (int64_t)(hv ? h0 + col : 0) * DK + 8 * g;
#pragma unroll
  for (int s = 0; s < DK / 32; ++s) qf[s] = hv ? ld8(qp + 32 * s) : bf16x8{};

  f32x4 o[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = OME_NEG_INF, lsum = 0.f;

  // staging: 32 keys x CH chunks, NST per thread; chunk c -> (key c / CH, x c % CH)
  bf16x8 stage[NST];
  auto load_pair = [&](int pr) {
#pragma unroll
    for (int i = 0; i < NST; ++i) {
      const int c = tid + 256 * i;
      if ((KT * CH) % 256 != 0 && c >= KT * CH) break;
      const int key = c / CH, x = c - key * CH;
      const int pg = 2 * pr + (key >> 4);
      const int page = bt[pg < n_pages ? pg : 0];
      stage[i] = ld8(cache + ((int64_t)page * 16 + (key & 15)) * DK + 8 * x);
    }
  };
  if (pair_begin < pair_end) load_pair(pair_begin);

  for (int pr = pair_begin; pr < pair_end; ++pr) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NST; ++i) {
      const int c = tid + 256 * i;
      if ((KT * CH) % 256 != 0 && c >= KT * CH) break;
      const int key = c / CH, x = c - key * CH;
      *reinterpret_cast<bf16x8*>(&sK[swz<DK>(key, x) * 8]) = stage[i];
    }
    __syncthreads();
    if (pr + 1 < pair_end) load_pair(pr + 1);

    // ---- S^T [32 keys x 16 heads] ----
    f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < DK / 32; ++s) {
      const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(&sK[swz<DK>(col, 4 * s + g) * 8]);
      const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(&sK[swz<DK>(16 + col, 4 * s + g) * 8]);
      s0 = mfma16x32(a0, qf[s], s0);
      s1 = mfma16x32(a1, qf[s], s1);
    }
    // ---- mask + online softmax (column = head, lane-local up to the 4 lane groups) ----
    const int kbase = pr * KT;
    float mx = OME_NEG_INF;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      s0[i] = (kbase + 4 * g + i < L) ? s0[i] * scale_log2 : OME_NEG_INF;
      s1[i] = (kbase + 16 + 4 * g + i < L) ? s1[i] * scale_log2 : OME_NEG_INF;
      mx = fmaxf(mx, fmaxf(s0[i], s1[i]));
    }
    mx = group4_max(mx);
    const float m_new = fmaxf(m, mx);
    const float alpha = (m_new == OME_NEG_INF) ? 1.f : __builtin_amdgcn_exp2f(m - m_new);
    bf16x8 pb;
    float ps = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float p0 = (m_new == OME_NEG_INF) ? 0.f : __builtin_amdgcn_exp2f(s0[i] - m_new);
      const float p1 = (m_new == OME_NEG_INF) ? 0.f : __builtin_amdgcn_exp2f(s1[i] - m_new);
      ps += p0 + p1;
      pb[i] = (bf16)p0;
      pb[4 + i] = (bf16)p1;
    }
    ps = group4_sum(ps);
    lsum = lsum * alpha + ps;
    m = m_new;
    // ---- O^T [this wave's DV / 4 dims x 16 heads] += V^T . P^T ----
    // tr-read block: rows = keys 4g + q (+16 for page B), cols = 16 dims; lane 4q+p of the
    // group addresses row q, columns 4p..4p+3.
    const int qrow = (lane & 15) >> 2, pcol = lane & 3;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const int d0 = wave * (DV / 4) + 16 * nb + 4 * pcol;  // first of this lane's 4 dims
      const int ra = 4 * g + qrow, rb = 16 + 4 * g + qrow;
      const int oa = swz<DK>(ra, d0 >> 3) * 16 + (d0 & 7) * 2;
      const int ob = swz<DK>(rb, d0 >> 3) * 16 + (d0 & 7) * 2;
      const bf16x4 va = tr_read(sK, oa), vb = tr_read(sK, ob);
      bf16x8 a;
      a[0] = va[0]; a[1] = va[1]; a[2] = va[2]; a[3] = va[3];
      a[4] = vb[0]; a[5] = vb[1]; a[6] = vb[2]; a[7] = vb[3];
#pragma unroll
      for (int i = 0; i < 4; ++i) o[nb][i] *= alpha;
      o[nb] = mfma16x32(a, pb, o[nb]);
    }
  }

  // ---- epilogue: O^T lane map dim = 16 nb + 4 g + i, head = col ----
  const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
  if (!hv) return;
  if (parts == 1) {
    bf16* op = out + (int64_t)t * out_stride_t + (int64_t)(h0 + col) * DV + wave * (DV / 4) + 4 * g;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      bf16x4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = (bf16)(o[nb][i] * inv);
      *reinterpret_cast<bf16x4*>(op + 16 * nb) = v;
    }
  } else {
    float* wp = ws_o + ws_row * DV + wave * (DV / 4) + 4 * g;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
      *reinterpret_cast<f32x4*>(wp + 16 * nb) = f32x4{o[nb][0] * inv, o[nb][1] * inv, o[nb][2] * inv,
                                                       o[nb][3] * inv};
    if (wave == 0 && g == 0) {
      ws_ml[2 * ws_row] = m;
      ws_ml[2 * ws_row + 1] = lsum;
    }
  }
}

// ------------------------------------------------------------------------------------------
// All-heads variant: one workgroup of NW waves owns 16 * NW heads of a token and one split-K
// partition, so each latent key tile is streamed from HBM and staged in LDS ONCE for all of them
// (the 16-head kernel above re-reads every token's latent KV H / 16 times -- 8x for DeepSeek-V3's
// 128 heads -- and its four waves each recompute the same S^T).  Wave w owns heads 16 w .. 16 w + 15
// and ALL DV value dims:
//   S^T [32 keys x 16 heads] = K . Q^T   (2 x DK/32 MFMAs, Q^T resident in 72 VGPRs)
//   O^T [DV x 16] += V^T . P^T           (DV/16 MFMAs, V^T by hardware-transposed LDS reads)
// Key tiles arrive by LDS DMA (buffer_load ... lds) into a double-buffered image: the DMA of tile
// n+1 is issued before tile n is computed and retired (vmcnt(0) + barrier) after it.
// ------------------------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void mla_lds_t;

template <int DK, int DV, int NW>
__global__ __launch_bounds__(64 * NW, 1) void mla_attn_all_kernel(
    const bf16* __restrict__ q, int64_t q_stride_t, const bf16* __restrict__ cache,
    const int* __restrict__ block_tables, int bt_stride, const int* __restrict__ tok_row,
    const int* __restrict__ kv_lens, int H, float scale_log2, int parts, bf16* __restrict__ out,
    int64_t out_stride_t, float* __restrict__ ws_o, float* __restrict__ ws_ml) {
  static_assert(DK == 576 && lds_chunks<DK>() == DK / 8, "LDS DMA image assumes unpadded 72-chunk rows");
  constexpr int CH = DK / 8, NI = KT * CH / 64, NB = DV / 16;
  constexpr int IMG = KT * CH * 8;   // bf16 elements per K-tile image
  __shared__ __attribute__((aligned(16))) bf16 sK[2 * IMG];
  const int t = blockIdx.x, part = blockIdx.z;
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int col = lane & 15, g = lane >> 4;
  const int head = blockIdx.y * 16 * NW + wave * 16 + col;   // this lane's head (S^T / O^T column)
  const int L = kv_lens[t];
  const int n_pages = (L + 15) >> 4;
  const int pairs = (n_pages + 1) >> 1;
  const int per_part = (pairs + parts - 1) / parts;
  const int pair_begin = part * per_part, pair_end = min(pairs, pair_begin + per_part);
  const int* bt = block_tables + (int64_t)tok_row[t] * bt_stride;

  // K tile pair -> LDS image: instruction i writes chunks [64 i, 64 i + 64) lane-linearly, each
  // lane fetching the source chunk the row's XOR swizzle puts there.  A page is 16 rows x 72 chunks
  // = 18 instructions, so each instruction reads one page: its descriptor is based at that page.
  auto dma_pair = [&](int pr, bf16* img) {
#pragma unroll
    for (int j = 0; j < (NI + NW - 1) / NW; ++j) {
      const int i = wave + NW * j;
      if (i >= NI) break;
      const int c = 64 * i + lane, row = c / CH, xl = c - row * CH;
      const int pg = 2 * pr + (i >= NI / 2);
      const int page = bt[pg < n_pages ? pg : 0];
      const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(cache + (int64_t)page * 16 * DK), (short)0,
                                                        16 * DK * 2, 0x00020000);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (mla_lds_t*)(img + 64 * 8 * i), 16,
                                               (uint32_t)(((row & 15) * CH + (xl ^ (row & 7))) * 16), 0, 0, 0);
    }
  };
  if (pair_begin < pair_end) dma_pair(pair_begin, sK);

  bf16x8 qf[DK / 32];
  const bf16* qp = q + (int64_t)t * q_stride_t + (int64_t)head * DK + 8 * g;
#pragma unroll
  for (int s = 0; s < DK / 32; ++s) qf[s] = ld8(qp + 32 * s);

  f32x4 o[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = OME_NEG_INF, lsum = 0.f;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // The XOR swizzle makes every LDS offset lane-dependent; split it so the compiler sees a lane
  // base plus an immediate: (8k + c) ^ z = 8k + (c ^ z) for c, z < 8.  S^T reads chunk 4 s + g of
  // row col (2 bases by s parity); V^T reads chunk 2 nb + pcol/2 of row 4 g + qrow (4 bases by
  // nb mod 4).  Rows 16..31 sit 16 * CH chunks further on with the same (row & 7).
  const int qrow = (lane & 15) >> 2, pcol = lane & 3;
  int sofs[2], vofs[4];
#pragma unroll
  for (int e = 0; e < 2; ++e) sofs[e] = (col * CH + ((4 * e + g) ^ (col & 7))) * 16;
  const int rv = 4 * g + qrow;
#pragma unroll
  for (int e = 0; e < 4; ++e) vofs[e] = (rv * CH + ((2 * e + (pcol >> 1)) ^ (rv & 7))) * 16 + (pcol & 1) * 8;
  int buf = 0;
  for (int pr = pair_begin; pr < pair_end; ++pr) {
    const bf16* img = sK + buf * IMG;
    // the other image's last readers passed the barrier that ended the previous tile
    if (pr + 1 < pair_end) dma_pair(pr + 1, sK + (buf ^ 1) * IMG);
    // ---- S^T [32 keys x 16 heads] ----
    const char* ib = reinterpret_cast<const char*>(img);
    f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < DK / 32; ++s) {
      const int off = sofs[s & 1] + (s >> 1) * 128;   // swz(col, 4 s + g): lane base + immediate
      const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(ib + off);
      const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(ib + off + 16 * CH * 16);
      s0 = mfma16x32(a0, qf[s], s0);
      s1 = mfma16x32(a1, qf[s], s1);
    }
    const int kbase = pr * KT;
    float mx = OME_NEG_INF;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      s0[i] = (kbase + 4 * g + i < L) ? s0[i] * scale_log2 : OME_NEG_INF;
      s1[i] = (kbase + 16 + 4 * g + i < L) ? s1[i] * scale_log2 : OME_NEG_INF;
      mx = fmaxf(mx, fmaxf(s0[i], s1[i]));
    }
    mx = group4_max(mx);
    const float m_new = fmaxf(m, mx);
    const float alpha = (m_new == OME_NEG_INF) ? 1.f : __builtin_amdgcn_exp2f(m - m_new);
    bf16x8 pb;
    float ps = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float p0 = (m_new == OME_NEG_INF) ? 0.f : __builtin_amdgcn_exp2f(s0[i] - m_new);
      const float p1 = (m_new == OME_NEG_INF) ? 0.f : __builtin_amdgcn_exp2f(s1[i] - m_new);
      ps += p0 + p1;
      pb[i] = (bf16)p0;
      pb[4 + i] = (bf16)p1;
    }
    ps = group4_sum(ps);
    lsum = lsum * alpha + ps;
    m = m_new;
    // ---- O^T [DV x 16 heads] += V^T . P^T (keys permuted as in pb: 4g + i, 16 + 4g + i) ----
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const int off = vofs[nb & 3] + (nb >> 2) * 128;   // swz(4g + qrow, 2 nb + pcol/2) + 8 (pcol & 1)
      const bf16x4 va = tr_read(img, off);
      const bf16x4 vb = tr_read(img, off + 16 * CH * 16);
      bf16x8 a;
      a[0] = va[0]; a[1] = va[1]; a[2] = va[2]; a[3] = va[3];
      a[4] = vb[0]; a[5] = vb[1]; a[6] = vb[2]; a[7] = vb[3];
      o[nb] *= alpha;
      o[nb] = mfma16x32(a, pb, o[nb]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the next tile's DMA has landed
    __syncthreads();
    buf ^= 1;
  }

  // ---- epilogue: O^T lane map dim = 16 nb + 4 g + i, head = col ----
  const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
  if (parts == 1) {
    bf16* op = out + (int64_t)t * out_stride_t + (int64_t)head * DV + 4 * g;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      bf16x4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = (bf16)(o[nb][i] * inv);
      *reinterpret_cast<bf16x4*>(op + 16 * nb) = v;
    }
  } else {
    const int64_t ws_row = ((int64_t)t * H + head) * parts + part;
    float* wp = ws_o + ws_row * DV + 4 * g;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
      *reinterpret_cast<f32x4*>(wp + 16 * nb) = f32x4{o[nb][0] * inv, o[nb][1] * inv, o[nb][2] * inv,
                                                       o[nb][3] * inv};
    if (g == 0) {
      ws_ml[2 * ws_row] = m;
      ws_ml[2 * ws_row + 1] = lsum;
    }
  }
}

// merge split-K partitions: one workgroup per (token, head), DV / 4 threads x 4 dims.  Partitions
// are consumed 8 at a time with all their loads issued up front (online max rescaling), so up to
// 64 partitions cost ~8 memory latencies rather than one each.
template <int DV>
__global__ __launch_bounds__(128) void mla_reduce_kernel(const float* __restrict__ ws_o,
                                                         const float* __restrict__ ws_ml, int H, int parts,
                                                         bf16* __restrict__ out, int64_t out_stride_t) {
  const int t = blockIdx.x, h = blockIdx.y;
  const int64_t row0 = ((int64_t)t * H + h) * parts;
  float M = OME_NEG_INF, den = 0.f;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int p0 = 0; p0 < parts; p0 += 8) {
    float mm[8], ll[8];
    f32x4 vv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int64_t r = row0 + min(p0 + j, parts - 1);
      mm[j] = ws_ml[2 * r];
      ll[j] = p0 + j < parts ? ws_ml[2 * r + 1] : 0.f;
      vv[j] = *reinterpret_cast<const f32x4*>(ws_o + r * DV + 4 * threadIdx.x);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (!(ll[j] > 0.f)) continue;
      const float mn = fmaxf(M, mm[j]);
      const float a = __builtin_amdgcn_exp2f(M - mn), w = ll[j] * __builtin_amdgcn_exp2f(mm[j] - mn);
      acc = acc * a + w * vv[j];
      den = den * a + w;
      M = mn;
    }
  }
  const float inv = den > 0.f ? 1.f / den : 0.f;
  bf16x4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = (bf16)(acc[i] * inv);
  *reinterpret_cast<bf16x4*>(out + (int64_t)t * out_stride_t + (int64_t)h * DV + 4 * threadIdx.x) = r;
}

// q [T, H, DK] (token stride q_stride_t), cache [pages, 16, DK], out [T, H, DV] with
// (DK, DV) = (576, 512) or (288, 256).  tok_row[t] = block-table row of token t; kv_lens[t] =
// keys visible to token t (causal).  parts > 1 needs ws_o [T*H*parts*DV] f32 and ws_ml
// [T*H*parts*2] f32.
template <int DK, int DV>
static void mla_launch(const void* q, int64_t q_stride_t, const void* cache, const int* block_tables, int bt_stride,
                       const int* tok_row, const int* kv_lens, int T, int H, float scale_log2, int parts, void* out,
                       int64_t out_stride_t, float* ws_o, float* ws_ml, hipStream_t stream) {
  // all-heads kernel when the heads tile into groups of 128 (DeepSeek-V3 / Kimi-K2 at TP 1) or 64
  // (TP 2): one latent stream per token and partition; else the 16-head kernel.  OME_MLA_ALL=0
  // forces the 16-head kernel (A/B timing).  Batches of at most OME_MLA_ALL_MIN_T tokens (default
  // 2) also take the 16-head kernel: the all-heads kernel's fixed cost (Q load, first DMA, fp32
  // partials + reduce) loses at T = 1 / 2 (41.0 / 40.1 vs 35.2 / 36.0 us) and wins from T = 4
  // (43.1 vs 61.4 us) -- profiles/r06_mla_cutover.txt.
  static const bool all_env = !getenv("OME_MLA_ALL") || atoi(getenv("OME_MLA_ALL")) != 0;
  static const int min_t = getenv("OME_MLA_ALL_MIN_T") ? atoi(getenv("OME_MLA_ALL_MIN_T")) : 2;
  const bool all_ok = all_env && T > min_t;
  bool done = false;
  if constexpr (DK == 576) {
    if (all_ok && H % 128 == 0) {
      mla_attn_all_kernel<DK, DV, 8><<<dim3(T, H / 128, parts), 512, 0, stream>>>(
          (const bf16*)q, q_stride_t, (const bf16*)cache, block_tables, bt_stride, tok_row, kv_lens, H, scale_log2,
          parts, (bf16*)out, out_stride_t, ws_o, ws_ml);
      done = true;
    } else if (all_ok && H % 64 == 0) {
      mla_attn_all_kernel<DK, DV, 4><<<dim3(T, H / 64, parts), 256, 0, stream>>>(
          (const bf16*)q, q_stride_t, (const bf16*)cache, block_tables, bt_stride, tok_row, kv_lens, H, scale_log2,
          parts, (bf16*)out, out_stride_t, ws_o, ws_ml);
      done = true;
    }
  }
  if (!done)
    mla_attn_kernel<DK, DV><<<dim3(T, (H + 15) / 16, parts), 256, 0, stream>>>(
        (const bf16*)q, q_stride_t, (const bf16*)cache, block_tables, bt_stride, tok_row, kv_lens, H, scale_log2,
        parts, (bf16*)out, out_stride_t, ws_o, ws_ml);
  if (parts > 1)
    mla_reduce_kernel<DV><<<dim3(T, H), DV / 4, 0, stream>>>(ws_o, ws_ml, H, parts, (bf16*)out, out_stride_t);
}

OME_API int ome_mla_attn(const void* q, int64_t q_stride_t, const void* cache, const int* block_tables,
                         int bt_stride, const int* tok_row, const int* kv_lens, int T, int H, int dk, int dv,
                         float scale, int parts, void* out, int64_t out_stride_t, float* ws_o, float* ws_ml,
                         hipStream_t stream) {
  if (T <= 0) return 0;
  if (H <= 0 || parts < 1 || (parts > 1 && (!ws_o || !ws_ml))) return -2;
  const float scale_log2 = scale * 1.4426950408889634f;
  if (dk == 576 && dv == 512)
    mla_launch<576, 512>(q, q_stride_t, cache, block_tables, bt_stride, tok_row, kv_lens, T, H, scale_log2, parts, out,
                         out_stride_t, ws_o, ws_ml, stream);
  else if (dk == 288 && dv == 256)
    mla_launch<288, 256>(q, q_stride_t, cache, block_tables, bt_stride, tok_row, kv_lens, T, H, scale_log2, parts, out,
                         out_stride_t, ws_o, ws_ml, stream);
  else
    return -3;
  OME_CHECK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------------------------------------
// MLA pre-attention glue as ONE launch per layer (it was ~25 PyTorch elementwise / cat /
// index_select / index_copy kernels per layer: profiles/r03_deepseek_v3_fp8_reduced.md "other").
// One workgroup per token t:
//   cache[slot_t][0 : lat]          = RMSNorm(a[t, qlr : qlr + lat]) * w       (kv_a_layernorm)
//   cache[slot_t][lat : lat + rope] = RoPE_pos(a[t, qlr + lat : qlr + lat + rope])
//   qf[t, h, lat : lat + rope]      = RoPE_pos(q[t, h, nope : nope + rope])   for every head h
// RoPE in NeoX halves (the checkpoint's interleaved rows are permuted at load), table cs[pos] =
// [cos | sin] fp32; fp32 math, bf16 stores (the reference op's order: x * rs * w, rounded once).
// Padding rows (slot < 0) write row 0 of the scratch page, as the eager path did.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void mla_prep_kernel(const bf16* __restrict__ a, int64_t lda, int qlr, int lat,
                                                       int rope, const bf16* __restrict__ w, float eps,
                                                       const int* __restrict__ pos, const float* __restrict__ cs,
                                                       const int* __restrict__ slots, bf16* __restrict__ cache,
                                                       int64_t cache_row, const bf16* __restrict__ q, int64_t q_tok,
                                                       int64_t q_head, int nope, int H, bf16* __restrict__ qf,
                                                       int64_t qf_tok, int64_t qf_head) {
  __shared__ float red[4];
  const int t = blockIdx.x, tid = threadIdx.x;
  const bf16* ar = a + (int64_t)t * lda + qlr;
  int slot = slots[t];
  slot = slot < 0 ? 0 : slot;
  bf16* crow = cache + (int64_t)slot * cache_row;
  float ss = 0.f;
  for (int i = tid; i < lat; i += 256) {
    const float v = (float)ar[i];
    ss += v * v;
  }
  for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o);
  if ((tid & 63) == 0) red[tid >> 6] = ss;
  __syncthreads();
  const float rs = rsqrtf((red[0] + red[1] + red[2] + red[3]) / (float)lat + eps);
  for (int i = tid; i < lat; i += 256) crow[i] = (bf16)((float)ar[i] * rs * (float)w[i]);
  const int half = rope >> 1;
  const float* c = cs + (int64_t)pos[t] * rope;
  // k_pe: pairs (j, j + half)
  for (int j = tid; j < half; j += 256) {
    const float x1 = (float)ar[lat + j], x2 = (float)ar[lat + half + j];
    const float co = c[j], si = c[half + j];
    crow[lat + j] = (bf16)(x1 * co - x2 * si);
    crow[lat + half + j] = (bf16)(x2 * co + x1 * si);
  }
  // q_pe of every head
  for (int k = tid; k < H * half; k += 256) {
    const int h = k / half, j = k - h * half;
    const bf16* qr = q + (int64_t)t * q_tok + (int64_t)h * q_head + nope;
    const float x1 = (float)qr[j], x2 = (float)qr[half + j];
    const float co = c[j], si = c[half + j];
    bf16* o = qf + (int64_t)t * qf_tok + (int64_t)h * qf_head + lat;
    o[j] = (bf16)(x1 * co - x2 * si);
    o[half + j] = (bf16)(x2 * co + x1 * si);
  }
}

OME_API int ome_mla_prep(const void* a, int64_t lda, int qlr, int lat, int rope, const void* w, float eps,
                         const int* pos, const float* cs, const int* slots, void* cache, int64_t cache_row,
                         const void* q, int64_t q_tok, int64_t q_head, int nope, int H, void* qf, int64_t qf_tok,
                         int64_t qf_head, int T, hipStream_t stream) {
  if (T <= 0) return 0;
  if (rope % 2 || lat <= 0 || H <= 0) return -2;
  mla_prep_kernel<<<T, 256, 0, stream>>>((const bf16*)a, lda, qlr, lat, rope, (const bf16*)w, eps, pos, cs, slots,
                                         (bf16*)cache, cache_row, (const bf16*)q, q_tok, q_head, nope, H, (bf16*)qf,
                                         qf_tok, qf_head);
  return (int)hipGetLastError();
}
