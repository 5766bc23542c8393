// ome_amd — varlen attention over contiguous (non-paged) Q/K/V for encoder models and vision
// towers: BERT / XLM-RoBERTa embedders and rerankers, the Qwen2-VL / Mllama ViTs.  SURVEY.md
// §2.9 K14 (embedding serving) and the multimodal towers behind the reference's VLM runtimes
// (e.g. config/runtimes/srt/BAAI/bge-m3-rt.yaml, .../Qwen/Qwen2.5-VL-7B-Instruct-rt.yaml).
//
// Sequences are packed back to back ([T, H, D] rows, any per-token stride so a fused QKV GEMM
// output is read in place) and delimited by cu_seqlens.  Bidirectional by default (encoders,
// ViT windows), causal on request.
//
// One workgroup = (128-query-row item of one sequence, one query head); its 4 waves own 32 rows
// each and share every K/V stage (2 x 32 keys) through double-buffered LDS:
//   K  [32 keys][DP + 8]  (272 B rows for DP = 128: 16 rows start on distinct bank quads)
//   V^T[DP dims][32 + 8]  keys in the k-slot order of the S^T accumulators, so a lane's A
//                         fragment of O^T = V^T P^T is one 16-B ds_read.
// S^T = K Q^T and O^T = V^T P^T run on v_mfma_f32_16x16x32_bf16 with the online softmax in
// registers (exp2 domain).  Head dims that are not a multiple of 32 (ViT-H 80, Llama-4 ViT 88) are zero-padded
// to DP inside the kernel: padded dims contribute 0 to QK^T and are never stored.
#include "common.h"

#define VA_NEG_INF (-__builtin_inff())

namespace {

__device__ __forceinline__ f32x4 va_mfma(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float va_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// k-slot of key kk (0..31) in an S^T accumulator pair: lane group g holds keys 4g..4g+3 (X = 0)
// and 16+4g..16+4g+3 (X = 1) as slots 8g..8g+7
__device__ __forceinline__ int va_slot(int kk) { return 8 * ((kk & 15) >> 2) + (kk & 3) + ((kk >> 4) << 2); }

// FAST (bidirectional, DP == 128: the long joint sequences of the Qwen-Image MMDiT, ViT-bigG):
// the paged prefill's fast softmax (attention.hip) -- only the last tile masks (a wave-uniform
// branch), the scale folds into the exp2 FMA, per-lane partial row sums (reduced once at the
// end), and O / l are rescaled lazily, only when some row's running max grew by more than 2^8.
template <int DP, bool FAST = false, int SUB = 1, int PROBE = 0>
__global__ __launch_bounds__(256, 2) void varlen_attn_kernel(
    const bf16* __restrict__ q, int64_t q_stride, const bf16* __restrict__ k, int64_t k_stride,
    const bf16* __restrict__ v, int64_t v_stride, const int* __restrict__ cu, const int* __restrict__ cuk,
    const int2* __restrict__ items, bf16* __restrict__ out, int64_t o_stride, int Hq, int Hkv, int D,
    float scale_log2, int causal) {
  constexpr int KS = DP / 32, NB = DP / 16, KLD = DP + 8, VLD = 32 + 8, CPR = DP / 8;
  constexpr int KCH = 32 * CPR;                       // 16-B K chunks per 32-key subtile
  constexpr int NCH = (KCH + 255) / 256;              // K chunks per thread per subtile
  constexpr int VG = 8 * CPR;                         // V groups (4 keys x 8 dims) per subtile
  constexpr int NVG = (VG + 255) / 256;
  // SUB: 32-key subtiles per pipeline stage (one barrier per stage); 2 measured -20 % on the
  // generic body at D 128, the FAST body is re-measured in profiles/r05_varlen_attn.md
  constexpr int KT = 32 * KLD, VT = DP * VLD;         // elements per subtile image
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * SUB * (KT + VT)];
  bf16* sK = smem;                      // [2][SUB][32 * KLD]
  bf16* sV = smem + 2 * SUB * KT;       // [2][SUB][DP * VLD]

  const int2 it = items[blockIdx.x];
  const int s = it.x, r0_item = it.y;
  const int head = blockIdx.y, kvh = head / (Hq / Hkv);
  const int t0 = cu[s], L = cu[s + 1] - t0;
  // cross attention (cuk != null): sequence s's keys are rows cuk[s] .. cuk[s+1] of k / v
  const int tk0 = cuk != nullptr ? cuk[s] : t0, Lk = cuk != nullptr ? cuk[s + 1] - tk0 : L;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int n = lane & 15, g = lane >> 4;
  const int r0 = r0_item + 32 * wave;
  const int kv_end = causal ? min(Lk, r0_item + 128) : Lk;

  // ---- this wave's query fragments (rows r0..r0+31), zero past L and past D ----
  bf16x8 qf[2][KS];
#pragma unroll
  for (int rb = 0; rb < 2; ++rb) {
    const int r = r0 + 16 * rb + n;
    const bf16* qr = q + (int64_t)(t0 + r) * q_stride + (int64_t)head * D;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int d0 = 32 * ks + 8 * g;
      qf[rb][ks] = (r < L && d0 < D) ? ld8(qr + d0) : bf16x8{};
    }
  }
  float m_i[2] = {VA_NEG_INF, VA_NEG_INF}, l_i[2] = {0.f, 0.f};
  f32x4 o[2][NB];
#pragma unroll
  for (int rb = 0; rb < 2; ++rb)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) o[rb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};

  // K: one 16-B chunk (8 dims of one key) per slot; V: groups of 4 consecutive keys x 8 dims, so
  // the transposed V image is written 4 keys (8 B) at a time.  V staging note: lane c takes key
  // group c & 7 and dims 8 (c >> 3): a 16-lane ds_write_b64 group then spans all 8 key-group
  // columns of two image rows (2-way on the (a/4) mod 32 store banks); with the dims across the
  // lanes (r04) all 16 lanes hit one bank pair -- 16-way, ~30 % of the kernel
  // (profiles/r05_varlen_attn.md, OME_VARLEN_PROBE=1).  Global reads stay 128 B per key row.
  // VSPLIT (D 128, 64-key stages): the two subtiles' 128 V groups each go to one half of the
  // workgroup (threads 0-127 subtile 0, 128-255 subtile 1) instead of both to threads 0-127, so
  // every wave issues the same loads and stores (and holds half the V registers)
  constexpr bool VSPLIT = SUB == 2 && VG <= 128;
  constexpr int RVS = VSPLIT ? 1 : SUB;
  // RING (fast body, D 128): two register sets, a stage's global loads issued two compute
  // phases before its LDS store (the paged prefill's A / B ring); otherwise one set, one phase
  constexpr bool RING = FAST && VSPLIT;
  bf16x8 rk[SUB][NCH] = {}, rv[RVS][NVG][4] = {};
  bf16x8 rk2[RING ? SUB : 1][NCH] = {}, rv2[RING ? RVS : 1][NVG][4] = {};
  const int vu = VSPLIT ? (tid >> 7) : 0, vc = VSPLIT ? (tid & 127) : tid;
  auto load_regs = [&](auto& rk, auto& rv, int kb0) {
    if constexpr (PROBE == 2) {   // timing probe only: no global loads (stale registers staged)
#pragma unroll
      for (int u = 0; u < SUB; ++u) {
#pragma unroll
        for (int i = 0; i < NCH; ++i) asm volatile("" : "+v"(rk[u][i]));
      }
#pragma unroll
      for (int u = 0; u < RVS; ++u)
#pragma unroll
        for (int i = 0; i < NVG; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) asm volatile("" : "+v"(rv[u][i][j]));
      return;
    }
#pragma unroll
    for (int u = 0; u < SUB; ++u) {
      const int kb = kb0 + 32 * u;
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        const int c = tid + 256 * i;
        const int key = c / CPR, d0 = (c % CPR) * 8;
        const bool ok = c < KCH && kb + key < Lk && d0 < D;
        rk[u][i] = ok ? ld8(k + (int64_t)(tk0 + kb + key) * k_stride + (int64_t)kvh * D + d0) : bf16x8{};
      }
    }
#pragma unroll
    for (int u = 0; u < RVS; ++u) {
      const int kb = kb0 + 32 * (VSPLIT ? vu : u);
#pragma unroll
      for (int i = 0; i < NVG; ++i) {
        const int c = vc + 256 * i;
        const int kq = c & 7, d0 = (c >> 3) * 8;   // 8 key groups across lanes: see V staging note
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int key = 4 * kq + j;
          const bool ok = c < VG && kb + key < Lk && d0 < D;
          rv[u][i][j] = ok ? ld8(v + (int64_t)(tk0 + kb + key) * v_stride + (int64_t)kvh * D + d0) : bf16x8{};
        }
      }
    }
  };
  auto store_regs = [&](const auto& rk, const auto& rv, int buf) {
#pragma unroll
    for (int u = 0; u < SUB; ++u) {
      bf16* Ks = sK + (buf * SUB + u) * KT;
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        const int c = tid + 256 * i;
        if (c < KCH) *reinterpret_cast<bf16x8*>(&Ks[(c / CPR) * KLD + (c % CPR) * 8]) = rk[u][i];
      }
    }
#pragma unroll
    for (int u = 0; u < RVS; ++u) {
      bf16* Vs = sV + (buf * SUB + (VSPLIT ? vu : u)) * VT;
#pragma unroll
      for (int i = 0; i < NVG; ++i) {
        const int c = vc + 256 * i;
        if (PROBE == 1) {   // timing probe only (wrong results): V image writes skipped
          asm volatile("" ::"v"(rv[u][i][0]), "v"(rv[u][i][1]), "v"(rv[u][i][2]), "v"(rv[u][i][3]));
          continue;
        }
        if (c < VG) {
          const int kq = c & 7, d0 = (c >> 3) * 8;   // 8 key groups across lanes: see V staging note
          bf16* vt = &Vs[d0 * VLD + va_slot(4 * kq)];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            bf16x4 w = {rv[u][i][0][j], rv[u][i][1][j], rv[u][i][2][j], rv[u][i][3][j]};
            *reinterpret_cast<bf16x4*>(vt + j * VLD) = w;
          }
        }
      }
    }
  };

  const bool active = r0 < L;
  auto compute_stage = [&](int kb0, int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < SUB; ++u) {
      const int kb = kb0 + 32 * u;
      if (!(active && kb < kv_end && (!causal || kb <= r0 + 31))) continue;
      const bf16* Kt = sK + (buf * SUB + u) * KT;
      const bf16* Vt = sV + (buf * SUB + u) * VT;
      f32x4 sc[2][2];
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) sc[rb][0] = sc[rb][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(&Kt[n * KLD + 32 * ks + 8 * g]);
        const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(&Kt[(16 + n) * KLD + 32 * ks + 8 * g]);
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
          sc[rb][0] = va_mfma(a0, qf[rb][ks], sc[rb][0]);
          sc[rb][1] = va_mfma(a1, qf[rb][ks], sc[rb][1]);
        }
      }
      if constexpr (FAST) {
        if (kb + 32 > Lk) {   // the sequence's last tile (wave-uniform)
          asm volatile("" ::: "memory");
#pragma unroll
          for (int rb = 0; rb < 2; ++rb)
#pragma unroll
            for (int X = 0; X < 2; ++X)
#pragma unroll
              for (int i = 0; i < 4; ++i)
                if (kb + 16 * X + 4 * g + i >= Lk) sc[rb][X][i] = VA_NEG_INF;
        }
        float mt[2];
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
          float v = VA_NEG_INF;
#pragma unroll
          for (int X = 0; X < 2; ++X)
#pragma unroll
            for (int i = 0; i < 4; ++i) v = fmaxf(v, sc[rb][X][i]);
          mt[rb] = group4_max(v) * scale_log2;
        }
        if (__ballot(mt[0] > m_i[0] + 8.f || mt[1] > m_i[1] + 8.f) != 0) {
          asm volatile("" ::: "memory");
#pragma unroll
          for (int rb = 0; rb < 2; ++rb) {
            const float m_new = fmaxf(m_i[rb], mt[rb]);
            const float alpha = va_exp2(m_i[rb] - m_new);   // m_new is finite: key 0 of the first tile is real
            l_i[rb] *= alpha;
#pragma unroll
            for (int nb = 0; nb < NB; ++nb) o[rb][nb] = o[rb][nb] * alpha;
            m_i[rb] = m_new;
          }
        }
        bf16x8 pb[2];
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
          float rs = 0.f;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float p0 = va_exp2(__builtin_fmaf(sc[rb][0][i], scale_log2, -m_i[rb]));
            const float p1 = va_exp2(__builtin_fmaf(sc[rb][1][i], scale_log2, -m_i[rb]));
            pb[rb][i] = (bf16)p0;
            pb[rb][4 + i] = (bf16)p1;
            rs += p0 + p1;
          }
          l_i[rb] += rs;   // this lane's partial row sum
        }
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
          const bf16x8 a = *reinterpret_cast<const bf16x8*>(&Vt[(16 * nb + n) * VLD + 8 * g]);
#pragma unroll
          for (int rb = 0; rb < 2; ++rb) o[rb][nb] = va_mfma(a, pb[rb], o[rb][nb]);
        }
        continue;
      }
      const bool need_mask = kb + 32 > Lk || (causal && kb + 32 > r0 + 1);
      bf16x8 pb[2];
      float alpha[2];
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
        const int qpos = r0 + 16 * rb + n;
        float mt = VA_NEG_INF;
#pragma unroll
        for (int X = 0; X < 2; ++X)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float val = sc[rb][X][i] * scale_log2;
            if (need_mask) {
              const int key = kb + 16 * X + 4 * g + i;
              const bool ok = key < Lk && (!causal || key <= qpos);
              val = ok ? val : VA_NEG_INF;
            }
            sc[rb][X][i] = val;
            mt = fmaxf(mt, val);
          }
        mt = group4_max(mt);
        const float m_new = fmaxf(m_i[rb], mt);
        const float m_use = (m_new == VA_NEG_INF) ? 0.f : m_new;
        alpha[rb] = va_exp2(m_i[rb] - m_use);
        float rs = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float p0 = va_exp2(sc[rb][0][i] - m_use), p1 = va_exp2(sc[rb][1][i] - m_use);
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
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(&Vt[(16 * nb + n) * VLD + 8 * g]);
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
          o[rb][nb] = o[rb][nb] * alpha[rb];
          o[rb][nb] = va_mfma(a, pb[rb], o[rb][nb]);
        }
      }
    }
  };
  constexpr int STEP = 32 * SUB;
  if constexpr (RING) {
    // invariant at the top: LDS buf 0 = stage kb, registers B (rk2 / rv2) = kb + STEP, A = kb + 2 STEP
    int kb = 0;
    if (kv_end > 0) {
      load_regs(rk, rv, 0);
      if (STEP < kv_end) load_regs(rk2, rv2, STEP);
      store_regs(rk, rv, 0);
    }
    __syncthreads();
    if (2 * STEP < kv_end) load_regs(rk, rv, 2 * STEP);
    for (; kb < kv_end; kb += 2 * STEP) {
      compute_stage(kb, 0);
      if (kb + STEP >= kv_end) break;
      store_regs(rk2, rv2, 1);   // buf 1 was last read before the previous barrier
      __syncthreads();
      if (kb + 3 * STEP < kv_end) load_regs(rk2, rv2, kb + 3 * STEP);
      compute_stage(kb + STEP, 1);
      if (kb + 2 * STEP >= kv_end) break;
      store_regs(rk, rv, 0);
      __syncthreads();
      if (kb + 4 * STEP < kv_end) load_regs(rk, rv, kb + 4 * STEP);
    }
  } else {
    int buf = 0;
    if (kv_end > 0) {
      load_regs(rk, rv, 0);
      store_regs(rk, rv, 0);
    }
    __syncthreads();
    for (int kb0 = 0; kb0 < kv_end; kb0 += STEP) {
      const bool more = kb0 + STEP < kv_end;
      if (more) load_regs(rk, rv, kb0 + STEP);  // in flight while this stage is consumed from LDS
      compute_stage(kb0, buf);
      if (more) store_regs(rk, rv, buf ^ 1);  // the other buffer was last read before the previous barrier
      __syncthreads();
      buf ^= 1;
    }
  }
  if (!active) return;
  if constexpr (FAST) {   // the row's 4 lanes' partial sums
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      l_i[rb] = group4_sum(l_i[rb]);
    }
  }
  // ---- epilogue: O^T accumulators hold O[row n][dims 16nb + 4g .. +3] ----
#pragma unroll
  for (int rb = 0; rb < 2; ++rb) {
    const int r = r0 + 16 * rb + n;
    if (r < L) {
      const float inv = l_i[rb] > 0.f ? 1.f / l_i[rb] : 0.f;
      bf16* orow = out + (int64_t)(t0 + r) * o_stride + (int64_t)head * D;
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        if (16 * nb + 4 * g < D) {  // D % 8 == 0: a lane's 4 dims are all in or all out
          bf16x4 w;
#pragma unroll
          for (int i = 0; i < 4; ++i) w[i] = (bf16)(o[rb][nb][i] * inv);
          *reinterpret_cast<bf16x4*>(orow + 16 * nb + 4 * g) = w;
        }
      }
    }
  }
}

int getenv_int(const char* name, int dflt) {
  static const char* v = getenv(name);   // read once: one variable per call site here
  return v ? atoi(v) : dflt;
}

}  // namespace

// items: int2 (sequence, first row) per 128-row work item, n_items of them (host-built).
// cuk: null (self attention: keys are the query rows) or the key row ranges of each sequence
// (cross attention: queries cu[s] .. cu[s+1] attend to keys cuk[s] .. cuk[s+1]; not causal).
// Strides are in elements per token; head h of a token starts at h * D.  D % 8 == 0, D <= 128;
// every pointer and stride 16-B aligned.
OME_API int ome_varlen_attention(const void* q, int64_t q_stride, const void* k, int64_t k_stride, const void* v,
                                 int64_t v_stride, const int* cu, const int* cuk, const int* items, int n_items,
                                 void* out, int64_t o_stride, int Hq, int Hkv, int D, float scale, int causal,
                                 hipStream_t stream) {
  if (n_items <= 0) return 0;
  // bit 1 of `causal`: force the generic body for a bidirectional call (ops.varlen_generic(), the
  // fast-vs-generic equivalence tests); bit 0: causal
  const bool force_generic = (causal & 2) != 0;
  causal &= 1;
  if (cuk != nullptr && causal) return -6;   // cross attention is bidirectional
  if (D <= 0 || D > 128 || D % 8 != 0) return -2;
  if (Hkv <= 0 || Hq % Hkv != 0) return -3;
  if ((q_stride | k_stride | v_stride | o_stride) % 8 != 0) return -4;
  if (Hq > 65535) return -5;
  const float sl2 = scale * 1.4426950408889634f;
  dim3 grid(n_items, Hq);
#define ARGS                                                                                                  \
  (const bf16*)q, q_stride, (const bf16*)k, k_stride, (const bf16*)v, v_stride, cu, cuk, (const int2*)items,  \
      (bf16*)out, o_stride, Hq, Hkv, D, sl2, causal
  // bidirectional calls take the FAST body (OME_VARLEN_FAST=0: generic); D 128 with 64-key
  // stages (OME_VARLEN_SUB=1: 32) -- profiles/r05_varlen_attn.md
  const bool fast = !causal && !force_generic && getenv_int("OME_VARLEN_FAST", 1);
  static const int sub = getenv("OME_VARLEN_SUB") ? atoi(getenv("OME_VARLEN_SUB")) : 2;
  static const int sub_small = getenv("OME_VARLEN_SUB_SMALL") ? atoi(getenv("OME_VARLEN_SUB_SMALL")) : 2;
  if (D <= 64) {
    if (fast && sub_small == 2) varlen_attn_kernel<64, true, 2><<<grid, 256, 0, stream>>>(ARGS);
    else if (fast) varlen_attn_kernel<64, true><<<grid, 256, 0, stream>>>(ARGS);
    else varlen_attn_kernel<64><<<grid, 256, 0, stream>>>(ARGS);
  } else if (D <= 96) {
    if (fast && sub_small == 2) varlen_attn_kernel<96, true, 2><<<grid, 256, 0, stream>>>(ARGS);
    else if (fast) varlen_attn_kernel<96, true><<<grid, 256, 0, stream>>>(ARGS);
    else varlen_attn_kernel<96><<<grid, 256, 0, stream>>>(ARGS);
  } else if (fast) {
    static const int probe = getenv("OME_VARLEN_PROBE") ? atoi(getenv("OME_VARLEN_PROBE")) : 0;
    if (probe == 1) varlen_attn_kernel<128, true, 2, 1><<<grid, 256, 0, stream>>>(ARGS);
    else if (probe == 2) varlen_attn_kernel<128, true, 2, 2><<<grid, 256, 0, stream>>>(ARGS);
    else if (sub == 2) varlen_attn_kernel<128, true, 2><<<grid, 256, 0, stream>>>(ARGS);
    else varlen_attn_kernel<128, true, 1><<<grid, 256, 0, stream>>>(ARGS);
  } else {
    varlen_attn_kernel<128><<<grid, 256, 0, stream>>>(ARGS);
  }
#undef ARGS
  OME_CHECK_LAUNCH();
  return 0;
}
