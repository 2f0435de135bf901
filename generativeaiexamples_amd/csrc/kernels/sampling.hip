// Token sampling: greedy / temperature / top-k / top-p, and OpenAI-style
// frequency / presence penalties.
//
// One 1024-thread workgroup per row. No sort: the top-k and top-p thresholds
// are found by radix selection on an order-preserving uint32 key of the logit
// (4 passes x 8 bits, count- or probability-mass-weighted LDS histograms), then
// the token is drawn with the Gumbel-max trick restricted to the surviving set,
// argmax(z_i + G_i) with G_i = -log(-log(u_i)) from a counter-based hash of
// (seed, step, i) -- exact sampling from the renormalised nucleus in a single
// extra pass, reproducible for a fixed seed. Top-p without top-k first tries the
// LDS fast path (nucleus_fast: one fused mass + compaction pass, exact cut resolved
// on <= 4096 candidates in LDS) and falls back to the radix passes.
#include "gai_common.h"
#include "gai_kernels.h"

using namespace gai;

namespace {

constexpr int kThreads = 1024;

__device__ __forceinline__ uint32_t fkey(float x) {
  const uint32_t b = __float_as_uint(x);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ float gumbel(uint64_t seed, uint64_t step, uint32_t i) {
  const uint64_t h = splitmix64(seed ^ splitmix64(step * 0x632BE59BD9B4E019ull + i));
  const float u = ((uint32_t)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);  // (0,1)
  return -__logf(-__logf(u));
}

struct ArgMax {
  float v;
  int i;
};

__device__ __forceinline__ ArgMax argmax_merge(ArgMax a, ArgMax b) {
  if (b.v > a.v || (b.v == a.v && b.i < a.i)) return b;
  return a;
}

__device__ ArgMax block_argmax(ArgMax a, float* sv, int* si) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    ArgMax b{__shfl_xor(a.v, o, 64), __shfl_xor(a.i, o, 64)};
    a = argmax_merge(a, b);
  }
  __syncthreads();
  if (lane == 0) {
    sv[wid] = a.v;
    si[wid] = a.i;
  }
  __syncthreads();
  ArgMax r{sv[0], si[0]};
  for (int w = 1; w < kThreads / 64; ++w) r = argmax_merge(r, ArgMax{sv[w], si[w]});
  return r;
}

// Calls f(value, index) for every element of a row; 16-byte loads, four in flight per thread, when the
// row is 16-byte aligned (the per-row passes are latency-bound with one workgroup per row).
template <class F>
__device__ __forceinline__ void row_for_each(const float* x, int V, F&& f) {
  if ((V & 3) == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0) {
    const float4* x4 = reinterpret_cast<const float4*>(x);
    const int V4 = V >> 2;
    int i = threadIdx.x;
    for (; i + 3 * kThreads < V4; i += 4 * kThreads) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = x4[i + u * kThreads];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int b = 4 * (i + u * kThreads);
        f(v[u].x, b);
        f(v[u].y, b + 1);
        f(v[u].z, b + 2);
        f(v[u].w, b + 3);
      }
    }
    for (; i < V4; i += kThreads) {
      const float4 v = x4[i];
      f(v.x, 4 * i);
      f(v.y, 4 * i + 1);
      f(v.z, 4 * i + 2);
      f(v.w, 4 * i + 3);
    }
  } else {
    for (int i = threadIdx.x; i < V; i += kThreads) f(x[i], i);
  }
}

// Histogram add for the radix passes. Near the top of the distribution the keys share their high bytes, so in
// the first passes most lanes of a wave hit one or two bins and plain LDS atomics serialise lane by lane (the
// split resolve spent ~100 us per decode step in them at the headline's ~3K candidates per row). Up to 4 bins per
// wave instruction are summed across the wave first (one atomic each); the rest add lane by lane. Every lane of
// the wave must call it (uniform trip counts), valid or not.
__device__ __forceinline__ void hist_add(float* hist, int bin, float w, bool valid) {
  const int lane = threadIdx.x & 63;
  unsigned long long act = __ballot(valid);
#pragma unroll 1
  for (int it = 0; it < 4 && act; ++it) {
    const int lead = __ffsll((long long)act) - 1;
    const int lb = __shfl(bin, lead, 64);
    const bool mine = valid && bin == lb;
    if (__popcll(__ballot(mine)) < 8) break;  // spread bins (later passes): lane-by-lane atomics are cheaper
    float v = mine ? w : 0.f;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == lead) atomicAdd(&hist[lb], v);
    act &= ~__ballot(mine);
    valid = valid && !mine;
  }
  if (valid) atomicAdd(&hist[bin], w);
}

// Finds the largest key threshold K* with weight(key >= K*) >= target, where the weight of
// element i is 1 (counting) or exp((x_i - mx) * invT) (mass), over elements with key >= floor_key.
template <bool MASS>
__device__ uint32_t radix_select(const float* x, int V, float mx, float invT, uint32_t floor_key, float target,
                                 float* hist, float* red) {
  uint32_t prefix = 0;
  float remaining = target;
#pragma unroll 1
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    for (int b = threadIdx.x; b < 256; b += kThreads) hist[b] = 0.f;
    __syncthreads();
    const uint32_t hi_mask = pass == 0 ? 0u : (0xFFFFFFFFu << (shift + 8));
    // whole rows spread over many exponent bins already: plain lane atomics (hist_add measured slower here)
    for (int i = threadIdx.x; i < V; i += kThreads) {
      const float xv = x[i];
      const uint32_t k = fkey(xv);
      if (k < floor_key || (k & hi_mask) != prefix) continue;
      const float w = MASS ? __expf((xv - mx) * invT) : 1.f;
      atomicAdd(&hist[(k >> shift) & 255], w);
    }
    __syncthreads();
    // scan buckets from the top (done by wave 0, 4 buckets per lane)
    if (threadIdx.x < 64) {
      const int l = threadIdx.x;
      float loc[4];
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        loc[j] = hist[255 - (4 * l + j)];
        s += loc[j];
      }
      // exclusive prefix over lanes (descending bucket order)
      float incl = s;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const float t = __shfl_up(incl, o, 64);
        if (l >= o) incl += t;
      }
      float run = incl - s;
      int found = -1;
      float above = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (found < 0 && run + loc[j] >= remaining) {
          found = 255 - (4 * l + j);
          above = run;
        }
        run += loc[j];
      }
      // first lane (lowest l) with a hit holds the highest bucket
      const unsigned long long hit = __ballot(found >= 0);
      int src = hit ? __ffsll((long long)hit) - 1 : 63;
      const int fb = __shfl(found, src, 64);
      const float ab = __shfl(above, src, 64);
      if (l == 0) {
        red[0] = hit ? (float)fb : 0.f;
        red[1] = hit ? ab : 0.f;
      }
    }
    __syncthreads();
    const int b = (int)red[0];
    remaining -= red[1];
    prefix |= ((uint32_t)b) << shift;
    __syncthreads();
  }
  return prefix;
}

__device__ __forceinline__ float key_to_float(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

// Top-p fast path. With the temperatures LLM serving uses, the nucleus lies within a few temperatures
// of the max logit, so ONE fused pass sums the softmax mass S in registers and compacts every element
// with d = (mx - x) / T < kCut into LDS (wave-aggregated slots, no histogram atomics). The exact cut is
// resolved there: bitonic sort of (key, index), prefix sum of the weights, cut at the first prefix >=
// p * S -- the same set as the radix path (largest key K* with mass(key >= K*) >= p * S), since every
// element outside the list has a smaller key. Gumbel-max then runs over the candidates only. Returns
// false (the caller takes the full radix path) when more than kCap elements qualify or the candidates
// hold less than p of the mass (flat distributions).
// LDS candidate capacity: the headline's random-init Llama-3 logits (~N(0, 1), T = 0.2) put 3-7K of 128K tokens within
// kCut temperatures of the row max, which overflowed 4096 on most rows and sent them to the whole-row radix passes
// (the split resolve at 131 us per decode step instead of ~25)
constexpr int kCap = 16384;
constexpr float kCut = 12.f;  // candidates: logits within 12 temperatures of the max (weight >= e^-12)

__device__ bool nucleus_fast(const float* x, int V, float mx, float invT, float p, uint64_t seed, int64_t step,
                             float* sv, int* si, uint64_t* cand, int* cnt, int* out) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (tid == 0) cnt[0] = 0, cnt[1] = 0x7fffffff;
  __syncthreads();
  // one fused pass: S = sum of exp(-d) in registers, elements with d < kCut compacted into LDS
  // (wave-aggregated slots; every lane runs the same trip count so each ballot sees the whole wave)
  float S = 0.f;
  auto visit = [&](float xv, int i, bool valid) {
    const float d = (mx - xv) * invT;
    S += valid ? __expf(-d) : 0.f;
    const bool c = valid && d < kCut;
    const unsigned long long m = __ballot(c);
    if (m == 0) return;
    int base = 0;
    if (lane == 0) base = atomicAdd(&cnt[0], __popcll(m));
    base = __shfl(base, 0, 64);
    const int pos = base + __popcll(m & ((1ull << lane) - 1ull));
    if (c && pos < kCap) cand[pos] = ((uint64_t)fkey(xv) << 32) | (uint32_t)i;
  };
  if ((V & 3) == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0) {
    const float4* x4 = reinterpret_cast<const float4*>(x);
    const int V4 = V >> 2;
    for (int j0 = 0; j0 < V4; j0 += 2 * kThreads) {
      float4 v[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int j = j0 + u * kThreads + tid;
        v[u] = j < V4 ? x4[j] : make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int j = j0 + u * kThreads + tid;
        const bool ok = j < V4;
        visit(v[u].x, 4 * j, ok);
        visit(v[u].y, 4 * j + 1, ok);
        visit(v[u].z, 4 * j + 2, ok);
        visit(v[u].w, 4 * j + 3, ok);
      }
    }
  } else {
    for (int i0 = 0; i0 < V; i0 += kThreads) {
      const int i = i0 + tid;
      visit(i < V ? x[i] : -INFINITY, i, i < V);
    }
  }
  S = block_sum(S, sv);  // (its barriers also publish the candidate list)
  const float target = p * S;
  const int n = cnt[0];
  if (n > kCap) return false;
  int P = 2;
  while (P < n) P <<= 1;
  for (int j = n + tid; j < P; j += kThreads) cand[j] = 0ull;
  __syncthreads();
  // bitonic sort, descending
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int t = tid; t < P / 2; t += kThreads) {
        const int a = (t / j) * 2 * j + (t % j), b = a + j;
        const uint64_t va = cand[a], vb = cand[b];
        if (((a & k) == 0) ? (va < vb) : (va > vb)) {
          cand[a] = vb;
          cand[b] = va;
        }
      }
      __syncthreads();
    }
  }
  // inclusive prefix of weights in sorted order; 4 consecutive candidates per thread
  float w[4], s = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int j = 4 * tid + q;
    w[q] = j < n ? __expf((key_to_float((uint32_t)(cand[j] >> 32)) - mx) * invT) : 0.f;
    s += w[q];
  }
  float incl = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  if (lane == 63) sv[wid] = incl;
  __syncthreads();
  float run = incl - s;
  for (int q = 0; q < wid; ++q) run += sv[q];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    run += w[q];
    if (4 * tid + q < n && run >= target) {
      atomicMin(&cnt[1], 4 * tid + q);
      break;
    }
  }
  __syncthreads();
  if (cnt[1] >= n) return false;  // the candidates hold less than p of the mass: the nucleus reaches past kCut
  const int jcut = cnt[1];
  const uint32_t kcut = (uint32_t)(cand[jcut] >> 32);
  ArgMax best{-INFINITY, 0x7fffffff};
  for (int j = tid; j < n; j += kThreads) {
    const uint64_t e = cand[j];
    const uint32_t kk = (uint32_t)(e >> 32);
    if (kk < kcut) continue;
    const uint32_t idx = (uint32_t)e;
    best = argmax_merge(best, ArgMax{(key_to_float(kk) - mx) * invT + gumbel(seed, (uint64_t)step, idx), (int)idx});
  }
  best = block_argmax(best, sv, si);
  if (tid == 0) *out = best.i;
  return true;
}

struct SampleSmem {
  float hist[256];
  float sv[16];
  int si[16];
  float red[4];
  uint64_t cand[kCap];
  int cnt[2];
};

// Whole-row sampler, one 1024-thread workgroup: argmax, then the nucleus fast path or the radix passes.
__device__ void sample_row_full(const float* x, int V, float T, int k, float p, uint64_t seed, int64_t step,
                                SampleSmem& sm, int* out) {
  ArgMax am{-INFINITY, 0x7fffffff};
  row_for_each(x, V, [&](float xv, int i) { am = argmax_merge(am, ArgMax{xv, i}); });
  am = block_argmax(am, sm.sv, sm.si);
  if (T <= 0.f) {
    if (threadIdx.x == 0) *out = am.i;
    return;
  }
  const float mx = am.v, invT = 1.f / T;
  if ((k <= 0 || k >= V) && p < 1.f && nucleus_fast(x, V, mx, invT, p, seed, step, sm.sv, sm.si, sm.cand, sm.cnt, out))
    return;
  uint32_t floor_key = 0;
  if (k > 0 && k < V) floor_key = radix_select<false>(x, V, mx, invT, 0u, (float)k, sm.hist, sm.red);
  if (p < 1.f) {
    float s = 0.f;
    for (int i = threadIdx.x; i < V; i += kThreads) {
      const float xv = x[i];
      if (fkey(xv) >= floor_key) s += __expf((xv - mx) * invT);
    }
    s = block_sum(s, sm.sv);
    floor_key = radix_select<true>(x, V, mx, invT, floor_key, p * s, sm.hist, sm.red);
  }
  ArgMax best{-INFINITY, 0x7fffffff};
  for (int i = threadIdx.x; i < V; i += kThreads) {
    const float xv = x[i];
    if (fkey(xv) < floor_key) continue;
    best = argmax_merge(best, ArgMax{(xv - mx) * invT + gumbel(seed, (uint64_t)step, (uint32_t)i), i});
  }
  best = block_argmax(best, sm.sv, sm.si);
  if (threadIdx.x == 0) *out = best.i < V ? best.i : am.i;
}

__global__ __launch_bounds__(kThreads) void sample_kernel(const float* __restrict__ logits, int V, long ld,
                                                          const float* __restrict__ temperature,
                                                          const float* __restrict__ top_p,
                                                          const int* __restrict__ top_k,
                                                          const int64_t* __restrict__ seeds, int64_t step,
                                                          int* __restrict__ out_tokens) {
  __shared__ SampleSmem sm;
  const int row = blockIdx.x;
  sample_row_full(logits + (size_t)row * ld, V, temperature[row], top_k[row], top_p[row], (uint64_t)seeds[row], step,
                  sm, out_tokens + row);
}

// ---------------------------------------------------------------------------------------------
// Split-row sampler (V >= kSplitMinV). One workgroup per row leaves 3/4 of the chip idle at batch 64 and
// streams each 513 KB row through one CU (~125 us per decode step at B = 64, V = 128256). Here:
//  1. split_stats   grid (S, B), 256 threads, kChunk logits per workgroup held in registers: chunk max,
//                   argmax, sum exp((x - max) / T); for pure-temperature rows the chunk's Gumbel-max, otherwise
//                   every element within kCut temperatures of the CHUNK max compacted to global slots (one pass
//                   over the logits: the row max is not known yet);
//  2. resolve       grid B, 1024 threads: the row's softmax mass from the partials, the candidates within kCut
//                   of the ROW max (nucleus_fast's set) gathered from the chunks that can hold any, in LDS,
//                   count-radix top-k / mass-radix top-p cut on the candidates, Gumbel-max over the
//                   survivors. Rows whose cut is not decidable on the candidates (top-k beyond them, a
//                   nucleus reaching past kCut, > kSlot candidates in a chunk) take sample_row_full.
// Same token as sample_kernel for a fixed (seed, step) up to float summation order at exact-cut ties.
constexpr int kChunk = 8192;   // logits per split workgroup (32 per thread, 8 float4 registers)
constexpr int kSplitT = 256;
// candidate slots per chunk (compacted relative to the CHUNK max: the headline's random-init logits, ~N(0, 1) at
// T = 0.2, put up to ~2.2K of a chunk's 8192 within kCut of it; 1024 slots overflowed and sent the row to the
// whole-row fallback)
constexpr int kSlot = 4096;
constexpr int kSplitMinV = 16384;
constexpr int kMaxSplits = 128;  // chunks per row the resolve kernel takes (V <= 1M); wider rows: whole-row kernel
constexpr int kPartW = 8;      // words per (row, split) partial: max, sum, argmax, gval, gidx, count

__device__ __forceinline__ int nsplit(int V) { return (V + kChunk - 1) / kChunk; }

__device__ __forceinline__ bool split_needs_cands(float T, float p, int k, int V) {
  return T > 0.f && (p < 1.f || (k > 0 && k < V));
}

__global__ __launch_bounds__(kSplitT) void sample_split_stats(const float* __restrict__ logits, int V, long ld,
                                                              const float* __restrict__ temperature,
                                                              const float* __restrict__ top_p,
                                                              const int* __restrict__ top_k,
                                                              const int64_t* __restrict__ seeds, int64_t step,
                                                              float* __restrict__ part,
                                                              uint64_t* __restrict__ cands) {
  __shared__ float sv[8];
  __shared__ int si[8];
  __shared__ int cnt;
  const int row = blockIdx.y, sp = blockIdx.x, S = gridDim.x, tid = threadIdx.x;
  const int c0 = sp * kChunk;
  const float* x = logits + (size_t)row * ld;
  constexpr int U = kChunk / (4 * kSplitT);
  float4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int i = c0 + 4 * (u * kSplitT + tid);
    if (i + 3 < V) {
      v[u] = *reinterpret_cast<const float4*>(x + i);
    } else {
      v[u].x = i < V ? x[i] : -INFINITY;
      v[u].y = i + 1 < V ? x[i + 1] : -INFINITY;
      v[u].z = i + 2 < V ? x[i + 2] : -INFINITY;
      v[u].w = i + 3 < V ? x[i + 3] : -INFINITY;
    }
  }
  ArgMax am{-INFINITY, 0x7fffffff};
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int i = c0 + 4 * (u * kSplitT + tid);
    am = argmax_merge(am, ArgMax{v[u].x, i});
    am = argmax_merge(am, ArgMax{v[u].y, i + 1});
    am = argmax_merge(am, ArgMax{v[u].z, i + 2});
    am = argmax_merge(am, ArgMax{v[u].w, i + 3});
  }
  // workgroup argmax (4 waves)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) am = argmax_merge(am, ArgMax{__shfl_xor(am.v, o, 64), __shfl_xor(am.i, o, 64)});
  if ((tid & 63) == 0) sv[tid >> 6] = am.v, si[tid >> 6] = am.i;
  __syncthreads();
  am = ArgMax{sv[0], si[0]};
  for (int w = 1; w < kSplitT / 64; ++w) am = argmax_merge(am, ArgMax{sv[w], si[w]});
  __syncthreads();
  const float T = temperature[row];
  float* pw = part + ((size_t)row * S + sp) * kPartW;
  if (T <= 0.f) {
    if (tid == 0) pw[0] = am.v, pw[2] = __int_as_float(am.i);
    return;
  }
  const float m = am.v, invT = 1.f / T;
  float s = 0.f;
  if (m > -INFINITY) {
#pragma unroll
    for (int u = 0; u < U; ++u)
      s += __expf((v[u].x - m) * invT) + __expf((v[u].y - m) * invT) + __expf((v[u].z - m) * invT) +
           __expf((v[u].w - m) * invT);
  }
  s = wave_sum(s);
  if ((tid & 63) == 0) sv[tid >> 6] = s;
  __syncthreads();
  if (tid == 0) {
    float t = 0.f;
    for (int w = 0; w < kSplitT / 64; ++w) t += sv[w];
    pw[0] = m, pw[1] = t, pw[2] = __int_as_float(am.i);
    cnt = 0;
  }
  const int k = top_k[row];
  if (split_needs_cands(T, top_p[row], k, V)) {
    // candidates relative to THIS chunk's max (the values are still in registers: one pass over the logits);
    // the resolve kernel keeps those within kCut temperatures of the row max, i.e. nucleus_fast's set
    __syncthreads();
    uint64_t* out = cands + ((size_t)row * S + sp) * kSlot;
    const int lane = tid & 63;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = c0 + 4 * (u * kSplitT + tid);
      const float e[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bool c = e[q] > -INFINITY && (m - e[q]) * invT < kCut;
        const unsigned long long msk = __ballot(c);
        if (msk == 0) continue;
        int base = 0;
        if (lane == 0) base = atomicAdd(&cnt, __popcll(msk));
        base = __shfl(base, 0, 64);
        const int pos = base + __popcll(msk & ((1ull << lane) - 1ull));
        if (c && pos < kSlot) out[pos] = ((uint64_t)fkey(e[q]) << 32) | (uint32_t)(i + q);
      }
    }
    __syncthreads();
    if (tid == 0) pw[5] = __int_as_float(cnt);
    return;
  }
  // pure temperature sampling: Gumbel-max over the whole row = max over chunks of x / T + G_i
  __syncthreads();
  const uint64_t seed = (uint64_t)seeds[row];
  ArgMax g{-INFINITY, 0x7fffffff};
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int i = c0 + 4 * (u * kSplitT + tid);
    const float e[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (i + q < V && e[q] > -INFINITY)
        g = argmax_merge(g, ArgMax{(e[q] - m) * invT + gumbel(seed, (uint64_t)step, (uint32_t)(i + q)), i + q});
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) g = argmax_merge(g, ArgMax{__shfl_xor(g.v, o, 64), __shfl_xor(g.i, o, 64)});
  if ((tid & 63) == 0) sv[tid >> 6] = g.v, si[tid >> 6] = g.i;
  __syncthreads();
  if (tid == 0) {
    g = ArgMax{sv[0], si[0]};
    for (int w = 1; w < kSplitT / 64; ++w) g = argmax_merge(g, ArgMax{sv[w], si[w]});
    pw[3] = g.v + m * invT;  // comparable across chunks: x / T + G
    pw[4] = __int_as_float(g.i);
  }
}

// radix_select over the LDS candidate list (keys in the high words)
template <bool MASS>
__device__ uint32_t radix_select_cands(const uint64_t* cand, int n, float mx, float invT, uint32_t floor_key,
                                       float target, float* hist, float* red) {
  uint32_t prefix = 0;
  float remaining = target;
#pragma unroll 1
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    for (int b = threadIdx.x; b < 256; b += kThreads) hist[b] = 0.f;
    __syncthreads();
    const uint32_t hi_mask = pass == 0 ? 0u : (0xFFFFFFFFu << (shift + 8));
    for (int j0 = 0; j0 < n; j0 += kThreads) {
      const int j = j0 + threadIdx.x;
      const uint32_t kk = j < n ? (uint32_t)(cand[j] >> 32) : 0u;
      const bool ok = j < n && kk >= floor_key && (kk & hi_mask) == prefix;
      const float w = MASS && ok ? __expf((key_to_float(kk) - mx) * invT) : 1.f;
      hist_add(hist, (kk >> shift) & 255, w, ok);
    }
    __syncthreads();
    if (threadIdx.x < 64) {
      const int l = threadIdx.x;
      float loc[4];
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        loc[j] = hist[255 - (4 * l + j)];
        s += loc[j];
      }
      float incl = s;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const float t = __shfl_up(incl, o, 64);
        if (l >= o) incl += t;
      }
      float run = incl - s;
      int found = -1;
      float above = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (found < 0 && run + loc[j] >= remaining) {
          found = 255 - (4 * l + j);
          above = run;
        }
        run += loc[j];
      }
      const unsigned long long hit = __ballot(found >= 0);
      int src = hit ? __ffsll((long long)hit) - 1 : 63;
      const int fb = __shfl(found, src, 64);
      const float ab = __shfl(above, src, 64);
      if (l == 0) {
        red[0] = hit ? (float)fb : 0.f;
        red[1] = hit ? ab : 0.f;
      }
    }
    __syncthreads();
    const int b = (int)red[0];
    remaining -= red[1];
    prefix |= ((uint32_t)b) << shift;
    __syncthreads();
  }
  return prefix;
}

__global__ __launch_bounds__(kThreads) void sample_split_resolve(const float* __restrict__ logits, int V, long ld,
                                                                 const float* __restrict__ temperature,
                                                                 const float* __restrict__ top_p,
                                                                 const int* __restrict__ top_k,
                                                                 const int64_t* __restrict__ seeds, int64_t step,
                                                                 const float* __restrict__ part,
                                                                 const uint64_t* __restrict__ cands, int S,
                                                                 int* __restrict__ out_tokens) {
  __shared__ SampleSmem sm;
  __shared__ int cnt_sh;
  __shared__ int flag;
  __shared__ float pr[kMaxSplits * kPartW];
  const int row = blockIdx.x, tid = threadIdx.x;
  const float T = temperature[row];
  const int k = top_k[row];
  const float p = top_p[row];
  const uint64_t seed = (uint64_t)seeds[row];
  // the row's partials land in LDS in one round of loads (runtime-trip loops over global memory below would each
  // wait out a full load latency per chunk)
  for (int e = tid; e < S * kPartW; e += kThreads) pr[e] = part[(size_t)row * S * kPartW + e];
  __syncthreads();
  // row max / argmax from the partials (first index among equal maxima, as the whole-row kernel)
  ArgMax am{-INFINITY, 0x7fffffff};
  for (int j = 0; j < S; ++j) am = argmax_merge(am, ArgMax{pr[j * kPartW], __float_as_int(pr[j * kPartW + 2])});
  if (T <= 0.f) {
    if (tid == 0) out_tokens[row] = am.i;
    return;
  }
  const float M = am.v, invT = 1.f / T;
  if (!split_needs_cands(T, p, k, V)) {
    ArgMax g{-INFINITY, 0x7fffffff};
    for (int j = 0; j < S; ++j) g = argmax_merge(g, ArgMax{pr[j * kPartW + 3], __float_as_int(pr[j * kPartW + 4])});
    if (tid == 0) out_tokens[row] = g.i < V ? g.i : am.i;
    return;
  }
  // candidate list: the chunks whose max lies within kCut of the row max contribute their candidates that do
  // too (nucleus_fast's set); such a chunk that overflowed its slots may have dropped one -> whole-row path
  if (tid == 0) cnt_sh = 0, flag = 0;
  __syncthreads();
  if (tid < S) {  // a contributing chunk that overflowed its slots may have dropped a candidate
    const float mj = pr[tid * kPartW];
    if (mj > -INFINITY && (M - mj) * invT < kCut && __float_as_int(pr[tid * kPartW + 5]) > kSlot) flag = 1;
  }
  __syncthreads();
  // every slot of every contributing chunk at once: kGather independent loads per thread in flight
  constexpr int kGather = 4;
  const uint64_t* src = cands + (size_t)row * S * kSlot;
  for (int e0 = 0; e0 < S * kSlot && !flag; e0 += kGather * kThreads) {
    uint64_t ev[kGather];
    bool live[kGather];
#pragma unroll
    for (int u = 0; u < kGather; ++u) {
      const int e = e0 + u * kThreads + tid;
      const int j = e / kSlot, q = e % kSlot;
      live[u] = false;
      if (e < S * kSlot) {
        const float mj = pr[j * kPartW];
        live[u] = mj > -INFINITY && (M - mj) * invT < kCut && q < __float_as_int(pr[j * kPartW + 5]);
      }
      ev[u] = live[u] ? src[e] : 0ull;
    }
#pragma unroll
    for (int u = 0; u < kGather; ++u) {
      const bool keep = live[u] && (M - key_to_float((uint32_t)(ev[u] >> 32))) * invT < kCut;
      const unsigned long long msk = __ballot(keep);
      int base = 0;
      if ((tid & 63) == 0 && msk) base = atomicAdd(&cnt_sh, __popcll(msk));
      base = __shfl(base, 0, 64);
      const int pos = base + __popcll(msk & ((1ull << (tid & 63)) - 1ull));
      if (keep && pos < kCap) sm.cand[pos] = ev[u];
    }
  }
  __syncthreads();
  if (flag || cnt_sh > kCap) {
    sample_row_full(logits + (size_t)row * ld, V, T, k, p, seed, step, sm, out_tokens + row);
    return;
  }
  const int n = cnt_sh;
  uint32_t floor_key = 0;
  int fallback = 0;
  if (k > 0 && k < V) {
    if (n < k) fallback = 1;  // the k-th largest lies outside the candidates
    else floor_key = radix_select_cands<false>(sm.cand, n, M, invT, 0u, (float)k, sm.hist, sm.red);
  }
  if (!fallback && p < 1.f) {
    float total = 0.f;
    if (k > 0 && k < V) {  // mass of the top-k set (all candidates)
      float s = 0.f;
      for (int j = tid; j < n; j += kThreads) {
        const uint32_t kk = (uint32_t)(sm.cand[j] >> 32);
        if (kk >= floor_key) s += __expf((key_to_float(kk) - M) * invT);
      }
      total = block_sum(s, sm.sv);
    } else {
      for (int j = 0; j < S; ++j) {
        const float mj = pr[j * kPartW];
        if (mj > -INFINITY) total += pr[j * kPartW + 1] * __expf((mj - M) * invT);
      }
    }
    // the candidates must hold >= p of the mass, else the nucleus reaches past kCut
    float s = 0.f;
    for (int j = tid; j < n; j += kThreads) {
      const uint32_t kk = (uint32_t)(sm.cand[j] >> 32);
      if (kk >= floor_key) s += __expf((key_to_float(kk) - M) * invT);
    }
    s = block_sum(s, sm.sv);
    if (s < p * total) fallback = 1;
    else floor_key = radix_select_cands<true>(sm.cand, n, M, invT, floor_key, p * total, sm.hist, sm.red);
  }
  if (fallback) {
    __syncthreads();
    sample_row_full(logits + (size_t)row * ld, V, T, k, p, seed, step, sm, out_tokens + row);
    return;
  }
  ArgMax best{-INFINITY, 0x7fffffff};
  for (int j = tid; j < n; j += kThreads) {
    const uint64_t e = sm.cand[j];
    const uint32_t kk = (uint32_t)(e >> 32);
    if (kk < floor_key) continue;
    const uint32_t idx = (uint32_t)e;
    best = argmax_merge(best, ArgMax{(key_to_float(kk) - M) * invT + gumbel(seed, (uint64_t)step, idx), (int)idx});
  }
  best = block_argmax(best, sm.sv, sm.si);
  if (tid == 0) out_tokens[row] = best.i < V ? best.i : am.i;
}

// ---------------------------------------------------------------------------------------------
// Vocab-parallel (TP) sampling without gathering the logits. Every TP rank reduces its logit shard to a
// packet per row [max, sum exp((x - max) / T), Gumbel-max value, its id, C candidate values, C candidate
// global ids (ids as exact floats)] (sample_tp_stats + its top-C, ops.sample_tp). The packets of all R ranks are gathered (one small peer-memory all-reduce of a
// zero-padded [R, B, W] buffer) and every rank runs this kernel on the same bytes, so all ranks draw the
// same token with no further collective. The candidate list holds every token above a cut K* when K* is
// above every rank's C-th value; then the result is exactly the whole-row sampler's (same nucleus, same
// Gumbel noise gumbel(seed, step, id)). Otherwise the draw is restricted to the R x C candidates and the
// row is counted in flags[0] (diagnostics).
constexpr int kTpThreads = 256;
constexpr int kTpMaxCand = 1024;

__global__ __launch_bounds__(kTpThreads) void sample_tp_resolve(const float* __restrict__ pk, int R, int B, int W, int C,
                                                                int V, const float* __restrict__ temperature,
                                                                const float* __restrict__ top_p,
                                                                const int* __restrict__ top_k,
                                                                const int64_t* __restrict__ seeds, int64_t step,
                                                                int* __restrict__ out_tokens, int* __restrict__ flags) {
  __shared__ float val[kTpMaxCand];
  __shared__ int idx[kTpMaxCand];
  __shared__ float wsum[kTpThreads / 64];
  __shared__ float cutv;
  __shared__ int cutj;
  __shared__ float sv[4];
  __shared__ int si[4];
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int n = R * C;
  int P = 1;
  while (P < n) P <<= 1;
  // candidates -> LDS (padding: -inf, id INT_MAX)
  for (int j = tid; j < P; j += kTpThreads) {
    if (j < n) {
      const int r = j / C, c = j % C;
      const float* q = pk + ((size_t)r * B + row) * W;
      val[j] = q[4 + c];
      idx[j] = (int)q[4 + C + c];
    } else {
      val[j] = -INFINITY;
      idx[j] = 0x7fffffff;
    }
  }
  const float T = temperature[row];
  float M = -INFINITY, kth_max = -INFINITY;
  for (int r = 0; r < R; ++r) {
    const float* q = pk + ((size_t)r * B + row) * W;
    M = fmaxf(M, q[0]);
    kth_max = fmaxf(kth_max, q[4 + C - 1]);
  }
  __syncthreads();
  // sort descending by value, ties: smaller id first
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int t = tid; t < P / 2; t += kTpThreads) {
        const int a = (t / j) * 2 * j + (t % j), b = a + j;
        const float va = val[a], vb = val[b];
        const int ia = idx[a], ib = idx[b];
        const bool b_first = vb > va || (vb == va && ib < ia);
        if (((a & k) == 0) ? b_first : !b_first) {
          val[a] = vb, val[b] = va;
          idx[a] = ib, idx[b] = ia;
        }
      }
      __syncthreads();
    }
  }
  if (T <= 0.f) {  // greedy: the global max is every rank's first candidate
    if (tid == 0) out_tokens[row] = idx[0];
    return;
  }
  const float invT = 1.f / T;
  float S = 0.f;
  for (int r = 0; r < R; ++r) {
    const float* q = pk + ((size_t)r * B + row) * W;
    if (q[0] > -INFINITY) S += q[1] * __expf((q[0] - M) * invT);
  }
  const int k = top_k[row];
  const float p = top_p[row];
  if (p >= 1.f && (k <= 0 || k >= V)) {  // pure temperature: the max over the ranks' shard Gumbel-maxima (exact)
    if (tid == 0) {
      ArgMax g{-INFINITY, 0x7fffffff};
      for (int r = 0; r < R; ++r) {
        const float* q = pk + ((size_t)r * B + row) * W;
        g = argmax_merge(g, ArgMax{q[2], (int)q[3]});
      }
      out_tokens[row] = g.i < V ? g.i : idx[0];
    }
    return;
  }
  int nk = n;            // candidates inside the top-k set
  bool exact = true;
  if (k > 0 && k < V) {
    if (k > n) exact = false;
    else nk = k;
  }
  // mass of the top-k set (or the whole row), then the first prefix reaching p of it
  if (tid == 0) cutj = nk - 1;
  float total = S;
  if (k > 0 && k < V) {
    float s = 0.f;
    for (int j = tid; j < nk; j += kTpThreads) s += __expf((val[j] - M) * invT);
    s = wave_sum(s);
    if (lane == 0) wsum[wid] = s;
    __syncthreads();
    total = 0.f;
    for (int w = 0; w < kTpThreads / 64; ++w) total += wsum[w];
    __syncthreads();
  }
  if (p < 1.f) {
    const float target = p * total;
    // inclusive prefix over the sorted list in chunks of kTpThreads
    float carry = 0.f;
    for (int base = 0; base < nk; base += kTpThreads) {
      const int j = base + tid;
      const float w = j < nk ? __expf((val[j] - M) * invT) : 0.f;
      float incl = w;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const float t = __shfl_up(incl, o, 64);
        if (lane >= o) incl += t;
      }
      if (lane == 63) wsum[wid] = incl;
      __syncthreads();
      float before = carry;
      for (int w2 = 0; w2 < wid; ++w2) before += wsum[w2];
      const bool hit = j < nk && before + incl >= target;
      const unsigned long long m = __ballot(hit);
      if (m && lane == __ffsll((long long)m) - 1) atomicMin(&cutj, j);
      float tot = 0.f;
      for (int w2 = 0; w2 < kTpThreads / 64; ++w2) tot += wsum[w2];
      __syncthreads();
      carry += tot;
      if (cutj < nk - 1 || carry >= target) break;
    }
    if (carry < target && cutj == nk - 1 && (k <= 0 || k >= V)) exact = false;  // nucleus beyond the list
  }
  __syncthreads();
  if (tid == 0) cutv = val[cutj];
  __syncthreads();
  const float K = cutv;
  if ((k <= 0 || k >= V) && !(K > kth_max)) exact = false;  // a token outside every list could tie / pass K
  const uint64_t seed = (uint64_t)seeds[row];
  ArgMax best{-INFINITY, 0x7fffffff};
  for (int j = tid; j < n; j += kTpThreads) {
    if (val[j] < K || idx[j] >= V) continue;
    best = argmax_merge(best, ArgMax{(val[j] - M) * invT + gumbel(seed, (uint64_t)step, (uint32_t)idx[j]), idx[j]});
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) best = argmax_merge(best, ArgMax{__shfl_xor(best.v, o, 64), __shfl_xor(best.i, o, 64)});
  if (lane == 0) sv[wid] = best.v, si[wid] = best.i;
  __syncthreads();
  if (tid == 0) {
    ArgMax b{sv[0], si[0]};
    for (int w = 1; w < kTpThreads / 64; ++w) b = argmax_merge(b, ArgMax{sv[w], si[w]});
    out_tokens[row] = b.i < V ? b.i : idx[0];
    if (!exact && flags) atomicAdd(flags, 1);
  }
}

// logits[b, t] -= freq * count + presence * (count > 0) for the tokens generated so far.
// counts is a sparse list per row: tok_ids[b, j], tok_cnt[b, j] for j < n[b] (unique ids).
__global__ void penalty_kernel(float* logits, long ld, const int* __restrict__ tok_ids,
                               const int* __restrict__ tok_cnt, const int* __restrict__ n, int max_n,
                               const float* __restrict__ freq, const float* __restrict__ pres,
                               const float* __restrict__ rep) {
  const int row = blockIdx.x;
  const float f = freq[row], pr = pres[row], rp = rep[row];
  for (int j = threadIdx.x; j < n[row]; j += blockDim.x) {
    const int t = tok_ids[(size_t)row * max_n + j];
    const int c = tok_cnt[(size_t)row * max_n + j];
    float v = logits[(size_t)row * ld + t];
    if (rp != 1.f) v = v > 0.f ? v / rp : v * rp;
    v -= f * c + (c > 0 ? pr : 0.f);
    logits[(size_t)row * ld + t] = v;
  }
}

// Constrained decoding: logits[rows[r], t] = -inf wherever bit t of mask[r] is clear. One thread per
// 32-token mask word; a 64-lane wave covers 2048 vocabulary entries with coalesced 128-B row loads.
__global__ void token_mask_kernel(float* logits, long ld, int V, const int* __restrict__ rows,
                                  const uint32_t* __restrict__ mask, int W) {
  const int r = blockIdx.y;
  const int w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= W) return;
  const uint32_t bits = mask[(size_t)r * W + w];
  if (bits == 0xFFFFFFFFu) return;
  float* row = logits + (size_t)rows[r] * ld;
  const int t0 = w * 32;
#pragma unroll 4
  for (int b = 0; b < 32; ++b)
    if (!(bits >> b & 1u) && t0 + b < V) row[t0 + b] = -INFINITY;
}

}  // namespace

void gai_token_mask(float* logits, long ld, int V, const int* rows, int R, const uint32_t* mask, int W,
                    hipStream_t st) {
  if (R == 0) return;
  token_mask_kernel<<<dim3((W + 255) / 256, R), 256, 0, st>>>(logits, ld, V, rows, mask, W);
  GAI_LAUNCH_CHECK();
}

size_t gai_sample_ws_bytes(int B, int V) {
  if (V < kSplitMinV) return 0;
  const size_t S = (size_t)((V + kChunk - 1) / kChunk);
  return (size_t)B * S * (kPartW * sizeof(float) + kSlot * sizeof(uint64_t));
}

void gai_sample(const float* logits, int B, int V, long ld, const float* temperature, const float* top_p,
                const int* top_k, const int64_t* seeds, int64_t step, int* out_tokens, void* ws, size_t ws_bytes,
                hipStream_t st) {
  if (B == 0) return;
  const size_t need = gai_sample_ws_bytes(B, V);
  const int S = (V + kChunk - 1) / kChunk;
  if (need == 0 || ws == nullptr || ws_bytes < need || S > 128 || (ld & 3) ||
      (reinterpret_cast<uintptr_t>(logits) & 15)) {
    sample_kernel<<<B, kThreads, 0, st>>>(logits, V, ld, temperature, top_p, top_k, seeds, step, out_tokens);
    GAI_LAUNCH_CHECK();
    return;
  }
  uint64_t* cands = reinterpret_cast<uint64_t*>(ws);
  float* part = reinterpret_cast<float*>(cands + (size_t)B * S * kSlot);
  sample_split_stats<<<dim3(S, B), kSplitT, 0, st>>>(logits, V, ld, temperature, top_p, top_k, seeds, step, part,
                                                      cands);
  GAI_LAUNCH_CHECK();
  sample_split_resolve<<<B, kThreads, 0, st>>>(logits, V, ld, temperature, top_p, top_k, seeds, step, part, cands,
                                               S, out_tokens);
  GAI_LAUNCH_CHECK();
}

// Per-row stats of a vocab shard for sample_tp_resolve: out[b] = {max, sum exp((x - max) / T), Gumbel-max of
// x / T + G(seed, step, vstart + i) over the shard, its global id}. Shard columns >= V - vstart (vocab padding)
// are ignored.
__global__ __launch_bounds__(kTpThreads) void sample_tp_stats(const float* __restrict__ x, long ld, int Vl, int vstart,
                                                              int V, const float* __restrict__ temperature,
                                                              const int64_t* __restrict__ seeds, int64_t step,
                                                              float* __restrict__ out, long ostride) {
  __shared__ float sv[4];
  __shared__ int si[4];
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const float* xr = x + (size_t)row * ld;
  const int n = min(Vl, V - vstart);
  float m = -INFINITY;
  for (int i = tid; i < n; i += kTpThreads) m = fmaxf(m, xr[i]);
  m = wave_max(m);
  if (lane == 0) sv[wid] = m;
  __syncthreads();
  m = fmaxf(fmaxf(sv[0], sv[1]), fmaxf(sv[2], sv[3]));
  __syncthreads();
  const float T = temperature[row];
  const float invT = T > 0.f ? 1.f / T : 1.f;
  const uint64_t seed = (uint64_t)seeds[row];
  float s = 0.f;
  ArgMax g{-INFINITY, 0x7fffffff};
  for (int i = tid; i < n; i += kTpThreads) {
    const float v = xr[i];
    if (m > -INFINITY) s += __expf((v - m) * invT);
    if (T > 0.f && v > -INFINITY)
      g = argmax_merge(g, ArgMax{v * invT + gumbel(seed, (uint64_t)step, (uint32_t)(vstart + i)), vstart + i});
  }
  s = wave_sum(s);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) g = argmax_merge(g, ArgMax{__shfl_xor(g.v, o, 64), __shfl_xor(g.i, o, 64)});
  __syncthreads();
  if (lane == 0) sv[wid] = s, si[wid] = 0;
  __syncthreads();
  float st = sv[0] + sv[1] + sv[2] + sv[3];
  __syncthreads();
  if (lane == 0) sv[wid] = g.v, si[wid] = g.i;
  __syncthreads();
  if (tid == 0) {
    ArgMax b{sv[0], si[0]};
    for (int w = 1; w < kTpThreads / 64; ++w) b = argmax_merge(b, ArgMax{sv[w], si[w]});
    float* o = out + (size_t)row * ostride;
    o[0] = m;
    o[1] = st;
    o[2] = b.v;
    o[3] = (float)(b.i == 0x7fffffff ? vstart : b.i);
  }
}

void gai_sample_tp_stats(const float* x, long ld, int B, int Vl, int vstart, int V, const float* temperature,
                         const int64_t* seeds, int64_t step, float* out, long ostride, hipStream_t st) {
  if (B == 0) return;
  sample_tp_stats<<<B, kTpThreads, 0, st>>>(x, ld, Vl, vstart, V, temperature, seeds, step, out, ostride);
  GAI_LAUNCH_CHECK();
}

int gai_sample_tp_resolve(const float* packets, int R, int B, int W, int C, int V, const float* temperature,
                          const float* top_p, const int* top_k, const int64_t* seeds, int64_t step, int* out_tokens,
                          int* flags, hipStream_t st) {
  if (B == 0) return 1;
  if (R * C > kTpMaxCand || W < 4 + 2 * C) return 0;
  sample_tp_resolve<<<B, kTpThreads, 0, st>>>(packets, R, B, W, C, V, temperature, top_p, top_k, seeds, step, out_tokens,
                                              flags);
  GAI_LAUNCH_CHECK();
  return 1;
}

void gai_apply_penalties(float* logits, int B, long ld, const int* tok_ids, const int* tok_cnt, const int* n,
                         int max_n, const float* freq, const float* pres, const float* rep, hipStream_t st) {
  if (B == 0) return;
  penalty_kernel<<<B, 256, 0, st>>>(logits, ld, tok_ids, tok_cnt, n, max_n, freq, pres, rep);
  GAI_LAUNCH_CHECK();
}
