// Token sampling over [B, V] logits (kernel K12): greedy, temperature, top-k, top-p, min-p.
//
// One 1024-thread workgroup per row.  The kept set {top-k} ∩ {top-p} ∩ {min-p} is found by
// bisection on the logit threshold (exact counts / masses over the row each step, the row
// stays L2-resident: 256 KB for a 128k vocab), and the token is then drawn with the
// Gumbel-max trick over the kept set (argmax of l/T - log(-log u)), which samples exactly
// from the renormalised softmax without a sort.  RNG: counter-based splitmix64 on
// (seed, row, step, index) — reproducible per request seed, graph-capture safe.
#include "common.h"

#define NT 1024

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

template <typename T>
__device__ __forceinline__ float ldf(const T* p, int64_t i) { return (float)p[i]; }

struct ValIdx {
  float v;
  int i;
};

__device__ __forceinline__ ValIdx vi_max(ValIdx a, ValIdx b) {
  if (b.v > a.v || (b.v == a.v && b.i < a.i)) return b;
  return a;
}

__device__ ValIdx block_argmax(ValIdx x, float* sv, int* si) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    ValIdx y{__shfl_xor(x.v, o), __shfl_xor(x.i, o)};
    x = vi_max(x, y);
  }
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) { sv[w] = x.v; si[w] = x.i; }
  __syncthreads();
  ValIdx r{sv[0], si[0]};
  for (int k = 1; k < NT / 64; ++k) r = vi_max(r, ValIdx{sv[k], si[k]});
  __syncthreads();
  return r;
}

__device__ float block_sumf(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
  for (int k = 0; k < NT / 64; ++k) t += red[k];
  __syncthreads();
  return t;
}

// ---- threshold select by a two-level histogram (top-k by count, top-p by mass) ----
// The kept set of a constraint is {z >= t} for the LARGEST t that still keeps >= target of
// count / mass.  Level 1 bins z in [-64, 0] into HB bins of 1/32 (z below -64, p < e^-64, all in
// the last bin), the crossing bin is found by a block prefix scan, and level 2 splits that bin
// into HB sub-bins (z resolution 1.5e-5, finer than a bf16 logit step): three row passes instead
// of the 26 bisection passes per constraint.  Values in the crossing sub-bin are all kept (the
// same tie rule as a threshold compare).  Counts are exact (integer-valued float adds); the
// top-p mass bins sum in atomic order, so a target within float rounding of a bin edge may pick
// the neighbouring sub-bin from run to run (a 1.5e-5-wide logit band): seeded draws are
// reproducible everywhere else.
constexpr int HB = 2048;
constexpr float HZ = 64.f;

// inclusive block scan of one value per thread (NT threads), returns the prefix
__device__ float block_scan(float v, float* wtot) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) wtot[w] = x;
  __syncthreads();
  float before = 0.f;
  for (int k = 0; k < w; ++k) before += wtot[k];
  __syncthreads();
  return x + before;
}

template <typename Row>
__device__ float hist_threshold(const Row& row, float mx, float invT, bool mass, float target, float* hist,
                                float* wtot, int* sel) {
  float upper = 0.f, width = HZ / HB;
  float carried = 0.f;
  for (int level = 0; level < 2; ++level) {
    for (int b = threadIdx.x; b < HB; b += NT) hist[b] = 0.f;
    __syncthreads();
    const float lo_edge = upper - HB * width;
    row([&](float l) {
      const float z = (l - mx) * invT;
      if (level == 1 && (z > upper || z <= lo_edge)) return;   // outside the refined bin
      int b = (int)((upper - z) * (1.f / width));
      b = b < 0 ? 0 : (b > HB - 1 ? HB - 1 : b);
      atomicAdd(&hist[b], mass ? __expf(z) : 1.f);
    });
    __syncthreads();
    // each thread owns bins 2t, 2t+1 (HB == 2 * NT)
    const float v0 = hist[2 * threadIdx.x], v1 = hist[2 * threadIdx.x + 1];
    const float incl = block_scan(v0 + v1, wtot) + carried;
    const float excl = incl - v0 - v1;
    if (threadIdx.x == 0) *sel = -1;
    __syncthreads();
    if (excl < target && incl >= target) *sel = (excl + v0 >= target) ? 2 * threadIdx.x : 2 * threadIdx.x + 1;
    __syncthreads();
    const int b = *sel;
    if (b < 0) return -__builtin_inff();   // the whole row does not reach the target: keep all
    if (b == HB - 1 && level == 0) return -__builtin_inff();   // crossing in the underflow bin
    // mass / count above the crossing bin carries into the next level
    float above = 0.f;
    {
      float part = 0.f;
      for (int i = threadIdx.x; i < b; i += NT) part += hist[i];
      above = block_sumf(part, wtot);
    }
    __syncthreads();
    if (level == 1) return upper - (b + 1) * width;   // lower edge of the crossing sub-bin
    carried += above;
    upper = upper - b * width;
    width = width / HB;
  }
  return -__builtin_inff();
}

template <typename T>
__global__ __launch_bounds__(NT) void sample_kernel(const T* __restrict__ logits, int64_t stride, int V,
                                                    const float* __restrict__ temperature,
                                                    const int* __restrict__ top_k, const float* __restrict__ top_p,
                                                    const float* __restrict__ min_p,
                                                    const uint64_t* __restrict__ seeds, uint64_t step,
                                                    int* __restrict__ out_ids, float* __restrict__ out_logprob) {
  __shared__ float sv[NT / 64];
  __shared__ int si[NT / 64];
  const int row = blockIdx.x;
  const T* lr = logits + (int64_t)row * stride;
  const float temp = temperature ? temperature[row] : 0.f;

  // pass 1, ONE read of the row: argmax + the softmax denominator at temperature (online: the
  // running sum is rescaled when the lane's max grows), 16-byte loads for bf16 rows -- the old
  // two scalar passes (max, then sum) were ~100 us per 256-row decode step over a 128k vocab
  const float invT = temp > 0.f ? 1.f / temp : 1.f;
  ValIdx best{-__builtin_inff(), 0};
  float lsum = 0.f;
  auto add = [&](float f, int i) {
    if (f > best.v) {
      lsum = (best.v == -__builtin_inff() ? 0.f : lsum * __expf((best.v - f) * invT)) + 1.f;
      best = ValIdx{f, i};
    } else {
      lsum += __expf((f - best.v) * invT);
    }
  };
  bool vec = false;
  if constexpr (sizeof(T) == 2) vec = (V % 8 == 0) && (stride % 8 == 0) && ((uintptr_t)lr % 16 == 0);
  if (vec) {
    if constexpr (sizeof(T) == 2) {
      for (int v = threadIdx.x; v < V / 8; v += NT) {
        const bf16x8 x = ld8(reinterpret_cast<const bf16*>(lr) + 8 * v);
        float lm = (float)x[0];
        int li = 0;
#pragma unroll
        for (int j = 1; j < 8; ++j)
          if ((float)x[j] > lm) lm = (float)x[j], li = j;
        if (lm > best.v) {   // rescale once per vector, then add all 8 at the new max
          lsum = best.v == -__builtin_inff() ? 0.f : lsum * __expf((best.v - lm) * invT);
          best = ValIdx{lm, 8 * v + li};
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) lsum += __expf(((float)x[j] - best.v) * invT);
      }
    }
  } else {
    for (int i = threadIdx.x; i < V; i += NT) add(ldf(lr, i), i);
  }
  // block reduction of (max, argmax, sum at that max)
  float den;
  {
    __shared__ float ss[NT / 64];
    const float m_lane = best.v;
    best = block_argmax(best, sv, si);
    const float mx0 = best.v;
    float part = m_lane == -__builtin_inff() ? 0.f : lsum * __expf((m_lane - mx0) * invT);
    den = block_sumf(part, ss);
  }
  const float mx = best.v;

  if (temp <= 0.f) {
    if (threadIdx.x == 0) {
      out_ids[row] = best.i;
      if (out_logprob) out_logprob[row] = -__logf(den);
    }
    return;
  }
  const int k = top_k ? top_k[row] : -1;
  const float pp = top_p ? top_p[row] : 1.f;
  const float mp = min_p ? min_p[row] : 0.f;

  // Threshold on scaled logit z = (l - mx) / T  (z <= 0).  Keep z >= thr.
  float thr = -__builtin_inff();
  if (mp > 0.f) thr = fmaxf(thr, __logf(mp));  // p_i / p_max >= min_p  <=>  z >= log(min_p)
  const bool need_k = k > 0 && k < V;
  const bool need_p = pp < 1.f;
  // count(z >= t) and mass(z >= t) are monotone non-increasing in t, so each constraint's
  // threshold is the LARGEST t that still keeps >= k tokens (top-k) / >= p of the mass
  // (top-p).  The kept set is the intersection: the max of the two thresholds.
  if (need_k || need_p) {
    __shared__ float hist[HB];
    __shared__ float wtot[NT / 64];
    __shared__ int sel;
    auto row = [&](auto&& f) {
      if (vec) {
        if constexpr (sizeof(T) == 2) {
          for (int v = threadIdx.x; v < V / 8; v += NT) {
            const bf16x8 x = ld8(reinterpret_cast<const bf16*>(lr) + 8 * v);
#pragma unroll
            for (int j = 0; j < 8; ++j) f((float)x[j]);
          }
        }
      } else {
        for (int i = threadIdx.x; i < V; i += NT) f(ldf(lr, i));
      }
    };
    if (need_k) thr = fmaxf(thr, hist_threshold(row, mx, invT, false, (float)k, hist, wtot, &sel));
    if (need_p) thr = fmaxf(thr, hist_threshold(row, mx, invT, true, pp * den, hist, wtot, &sel));
  }
  // Gumbel-max over the kept set
  const uint64_t seed = seeds ? seeds[row] : 0x1234ull;
  ValIdx pick{-__builtin_inff(), best.i};
  auto gumbel = [&](float l, int i) {
    const float z = (l - mx) * invT;
    if (z >= thr) {
      const uint64_t h = splitmix64(seed ^ splitmix64(step * 0x100000001B3ull + (uint64_t)i));
      const float u = ((float)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);
      pick = vi_max(pick, ValIdx{z - __logf(-__logf(u)), i});
    }
  };
  if (vec) {
    if constexpr (sizeof(T) == 2) {
      for (int v = threadIdx.x; v < V / 8; v += NT) {
        const bf16x8 x = ld8(reinterpret_cast<const bf16*>(lr) + 8 * v);
#pragma unroll
        for (int j = 0; j < 8; ++j) gumbel((float)x[j], 8 * v + j);
      }
    }
  } else {
    for (int i = threadIdx.x; i < V; i += NT) gumbel(ldf(lr, i), i);
  }
  pick = block_argmax(pick, sv, si);
  if (threadIdx.x == 0) {
    out_ids[row] = pick.i;
    if (out_logprob) out_logprob[row] = (ldf(lr, pick.i) - mx) * invT - __logf(den);
  }
}

OME_API int ome_sample(const void* logits, int is_bf16, int64_t stride, int B, int V, const float* temperature,
                       const int* top_k, const float* top_p, const float* min_p, const uint64_t* seeds,
                       uint64_t step, int* out_ids, float* out_logprob, hipStream_t stream) {
  if (B <= 0) return 0;
  if (is_bf16)
    sample_kernel<bf16><<<B, NT, 0, stream>>>((const bf16*)logits, stride, V, temperature, top_k, top_p, min_p,
                                              seeds, step, out_ids, out_logprob);
  else
    sample_kernel<float><<<B, NT, 0, stream>>>((const float*)logits, stride, V, temperature, top_k, top_p, min_p,
                                               seeds, step, out_ids, out_logprob);
  OME_CHECK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------------------------------------
// Repetition / frequency / presence penalties (K12, vLLM / OpenAI semantics):
//   counts[slot, v] low 24 bits = occurrences of v in the OUTPUT so far, bit 24 = v occurs in
//   the prompt or output ("seen", for the repetition penalty).
//   logit' = seen ? (logit > 0 ? logit / rep : logit * rep) : logit
//   logit' -= freq * out_count + pres * (out_count > 0)
// Rows whose three penalties are neutral return immediately, so the kernels stay in the decode
// graph at ~zero cost when no request uses penalties.
// ------------------------------------------------------------------------------------------
constexpr int kSeenBit = 1 << 24;

template <typename T>
__global__ __launch_bounds__(256) void apply_penalties_kernel(T* __restrict__ logits, int64_t stride, int V,
                                                              const int* __restrict__ counts, int64_t cstride,
                                                              const int* __restrict__ slot,
                                                              const float* __restrict__ rep,
                                                              const float* __restrict__ freq,
                                                              const float* __restrict__ pres) {
  const int row = blockIdx.y;
  const float rp = rep[row], fp = freq[row], pp = pres[row];
  if (rp == 1.f && fp == 0.f && pp == 0.f) return;
  const int* cr = counts + (int64_t)slot[row] * cstride;
  T* lr = logits + (int64_t)row * stride;
  for (int v = blockIdx.x * blockDim.x + threadIdx.x; v < V; v += gridDim.x * blockDim.x) {
    const int c = cr[v];
    if (c == 0) continue;
    float x = (float)lr[v];
    if ((c & kSeenBit) && rp != 1.f) x = x > 0.f ? x / rp : x * rp;
    const int oc = c & (kSeenBit - 1);
    x -= fp * (float)oc + (oc > 0 ? pp : 0.f);
    lr[v] = (T)x;
  }
}

OME_API int ome_apply_penalties(void* logits, int is_bf16, int64_t stride, int B, int V, const int* counts,
                                int64_t cstride, const int* slot, const float* rep, const float* freq,
                                const float* pres, hipStream_t stream) {
  if (B <= 0) return 0;
  dim3 grid(16, B);
  if (is_bf16)
    apply_penalties_kernel<bf16><<<grid, 256, 0, stream>>>((bf16*)logits, stride, V, counts, cstride, slot, rep,
                                                           freq, pres);
  else
    apply_penalties_kernel<float><<<grid, 256, 0, stream>>>((float*)logits, stride, V, counts, cstride, slot, rep,
                                                            freq, pres);
  OME_CHECK_LAUNCH();
  return 0;
}

// After sampling: count the new token for rows that use penalties.
__global__ void update_counts_kernel(int* __restrict__ counts, int64_t cstride, const int* __restrict__ slot,
                                     const int* __restrict__ ids, const float* __restrict__ rep,
                                     const float* __restrict__ freq, const float* __restrict__ pres, int B) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  if (rep[i] == 1.f && freq[i] == 0.f && pres[i] == 0.f) return;
  int* c = counts + (int64_t)slot[i] * cstride + ids[i];
  *c = ((*c) + 1) | kSeenBit;  // one writer per (slot, token): a request occupies one row per step
}

OME_API int ome_update_counts(int* counts, int64_t cstride, const int* slot, const int* ids, const float* rep,
                              const float* freq, const float* pres, int B, hipStream_t stream) {
  if (B <= 0) return 0;
  update_counts_kernel<<<(B + 255) / 256, 256, 0, stream>>>(counts, cstride, slot, ids, rep, freq, pres, B);
  OME_CHECK_LAUNCH();
  return 0;
}
