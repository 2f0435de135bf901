// Token sampling: greedy / temperature / top-k / top-p, and OpenAI-style
// frequency / presence penalties.
//
// One 1024-thread workgroup per row. No sort: the top-k and top-p thresholds
// are found by radix selection on an order-preserving uint32 key of the logit
// (4 passes x 8 bits, count- or probability-mass-weighted LDS histograms), then
// the token is drawn with the Gumbel-max trick restricted to the surviving set,
// argmax(z_i + G_i) with G_i = -log(-log(u_i)) from a counter-based hash of
// (seed, step, i) -- exact sampling from the renormalised nucleus in a single
// extra pass, reproducible for a fixed seed.
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

__global__ __launch_bounds__(kThreads) void sample_kernel(const float* __restrict__ logits, int V, long ld,
                                                          const float* __restrict__ temperature,
                                                          const float* __restrict__ top_p,
                                                          const int* __restrict__ top_k,
                                                          const int64_t* __restrict__ seeds, int64_t step,
                                                          int* __restrict__ out_tokens) {
  __shared__ float hist[256];
  __shared__ float sv[16];
  __shared__ int si[16];
  __shared__ float red[4];
  const int row = blockIdx.x;
  const float* x = logits + (size_t)row * ld;
  const float T = temperature[row];

  ArgMax am{-INFINITY, 0x7fffffff};
  for (int i = threadIdx.x; i < V; i += kThreads) am = argmax_merge(am, ArgMax{x[i], i});
  am = block_argmax(am, sv, si);
  if (T <= 0.f) {
    if (threadIdx.x == 0) out_tokens[row] = am.i;
    return;
  }
  const float mx = am.v, invT = 1.f / T;
  uint32_t floor_key = 0;
  const int k = top_k[row];
  if (k > 0 && k < V) floor_key = radix_select<false>(x, V, mx, invT, 0u, (float)k, hist, red);
  const float p = top_p[row];
  if (p < 1.f) {
    float s = 0.f;
    for (int i = threadIdx.x; i < V; i += kThreads) {
      const float xv = x[i];
      if (fkey(xv) >= floor_key) s += __expf((xv - mx) * invT);
    }
    s = block_sum(s, sv);
    floor_key = radix_select<true>(x, V, mx, invT, floor_key, p * s, hist, red);
  }
  const uint64_t seed = (uint64_t)seeds[row];
  ArgMax best{-INFINITY, 0x7fffffff};
  for (int i = threadIdx.x; i < V; i += kThreads) {
    const float xv = x[i];
    if (fkey(xv) < floor_key) continue;
    best = argmax_merge(best, ArgMax{(xv - mx) * invT + gumbel(seed, (uint64_t)step, (uint32_t)i), i});
  }
  best = block_argmax(best, sv, si);
  if (threadIdx.x == 0) out_tokens[row] = best.i < V ? best.i : am.i;
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

void gai_sample(const float* logits, int B, int V, long ld, const float* temperature, const float* top_p,
                const int* top_k, const int64_t* seeds, int64_t step, int* out_tokens, hipStream_t st) {
  if (B == 0) return;
  sample_kernel<<<B, kThreads, 0, st>>>(logits, V, ld, temperature, top_p, top_k, seeds, step, out_tokens);
  GAI_LAUNCH_CHECK();
}

void gai_apply_penalties(float* logits, int B, long ld, const int* tok_ids, const int* tok_cnt, const int* n,
                         int max_n, const float* freq, const float* pres, const float* rep, hipStream_t st) {
  if (B == 0) return;
  penalty_kernel<<<B, 256, 0, st>>>(logits, ld, tok_ids, tok_cnt, n, max_n, freq, pres, rep);
  GAI_LAUNCH_CHECK();
}
