// Small memory-bound kernels: embedding gather (vocab-parallel aware), sequence
// pooling + L2 normalisation, standalone activations.
// All loads/stores are 16-byte bf16x8 vectors (cdna_hip_programming Guideline 13).
#include "gai_common.h"
#include "gai_kernels.h"

using namespace gai;

namespace {

// out[t] = table[ids[t] - vstart] if vstart <= ids[t] < vend else 0 (vocab-parallel shard)
__global__ __launch_bounds__(256) void embedding_kernel(const int* __restrict__ ids, const bf16* __restrict__ table,
                                                        bf16* __restrict__ out, int T, int D, int vstart, int vend) {
  const int units = D / 8;
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long)T * units) return;
  const int t = (int)(e / units), u = (int)(e % units);
  const int id = ids[t];
  bf16x8 v = bf16x8{};
  if (id >= vstart && id < vend) v = load8(table + (size_t)(id - vstart) * D + u * 8);
  store8(out + (size_t)t * D + u * 8, v);
}

// Pool each sequence of hidden [T, D] (varlen via cu_seqlens) into out [B, D] fp32.
// mode 0 = masked mean, 1 = first token (CLS), 2 = last token. normalize -> v / ||v||.
__global__ __launch_bounds__(256) void pool_kernel(const bf16* __restrict__ h, const int* __restrict__ cu,
                                                   float* __restrict__ out, int D, int mode, int normalize) {
  extern __shared__ float sh[];  // D floats + 16 scratch
  float* acc = sh;
  float* scratch = sh + D;
  const int b = blockIdx.x;
  const int s0 = cu[b], s1 = cu[b + 1], n = s1 - s0;
  for (int d = threadIdx.x; d < D; d += 256) acc[d] = 0.f;
  __syncthreads();
  int r0 = s0, r1 = s1;
  if (mode == 1) r1 = min(s0 + 1, s1);
  if (mode == 2) r0 = max(s1 - 1, s0);
  const int units = D / 8;
  // each thread accumulates a fixed unit across rows
  for (int u = threadIdx.x; u < units; u += 256) {
    float a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int r = r0; r < r1; ++r) {
      const bf16x8 v = load8(h + (size_t)r * D + u * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] += (float)v[j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[u * 8 + j] = a[j];
  }
  __syncthreads();
  const float div = (mode == 0 && n > 0) ? 1.f / n : 1.f;
  float ss = 0.f;
  for (int d = threadIdx.x; d < D; d += 256) {
    const float v = acc[d] * div;
    acc[d] = v;
    ss += v * v;
  }
  float scale = 1.f;
  if (normalize) {
    ss = block_sum(ss, scratch);
    scale = 1.f / fmaxf(sqrtf(ss), 1e-12f);
  }
  for (int d = threadIdx.x; d < D; d += 256) out[(size_t)b * D + d] = acc[d] * scale;
}

// MODE 0: y[t, i] = silu(x[t, i]) * x[t, I + i] (non-interleaved gate|up); 1: gelu_erf(x);
// 2: SwiGLU on the interleaved-per-16 [gate16|up16] layout; 3: gelu_tanh(x); 4: GeGLU (gelu_tanh(gate) * up,
// interleaved layout: Gemma).
template <int MODE>
__global__ __launch_bounds__(256) void act_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, int T, int I) {
  const int units = I / 8;
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long)T * units) return;
  const int t = (int)(e / units), u = (int)(e % units);
  bf16x8 o;
  if (MODE == 2 || MODE == 4) {  // gate/up interleaved per 16 columns (the fused-GLU weight layout)
    const int c = u * 8, p = c >> 4, c0 = c & 15;
    const bf16x8 g = load8(x + (size_t)t * 2 * I + 32 * p + c0);
    const bf16x8 up = load8(x + (size_t)t * 2 * I + 32 * p + 16 + c0);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      o[j] = (bf16)((MODE == 2 ? silu((float)g[j]) : gelu_tanh((float)g[j])) * (float)up[j]);
  } else if (MODE == 3) {
    const bf16x8 a = load8(x + (size_t)t * I + u * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16)gelu_tanh((float)a[j]);
  } else if (MODE == 0) {
    const bf16x8 g = load8(x + (size_t)t * 2 * I + u * 8);
    const bf16x8 up = load8(x + (size_t)t * 2 * I + I + u * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16)(silu((float)g[j]) * (float)up[j]);
  } else {
    const bf16x8 a = load8(x + (size_t)t * I + u * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16)gelu_erf((float)a[j]);
  }
  store8(y + (size_t)t * I + u * 8, o);
}

// Multi-step decode: feed the token sampled at step j back as step j+1's input, inside one HIP
// graph. Row r < *n_valid: ids <- toks, pos += 1, ctx = pos + 1, slot from the block table
// (pages for the whole run are reserved by Scheduler.reserve_decode). Padded rows stay frozen
// on the scratch page.
__global__ __launch_bounds__(256) void decode_advance_kernel(const int* __restrict__ toks, int* __restrict__ ids,
                                                             int* __restrict__ pos, int* __restrict__ ctx,
                                                             int* __restrict__ slots, const int* __restrict__ bt,
                                                             int max_blocks, const int* __restrict__ n_valid, int B,
                                                             int block) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= B || r >= *n_valid) return;
  const int p = pos[r] + 1;
  ids[r] = toks[r];
  pos[r] = p;
  ctx[r] = p + 1;
  slots[r] = bt[(size_t)r * max_blocks + p / block] * block + p % block;
}

}  // namespace

void gai_decode_advance(const int* toks, int* ids, int* pos, int* ctx, int* slots, const int* bt, int max_blocks,
                        const int* n_valid, int B, int block, hipStream_t st) {
  if (B == 0) return;
  decode_advance_kernel<<<(B + 255) / 256, 256, 0, st>>>(toks, ids, pos, ctx, slots, bt, max_blocks, n_valid, B,
                                                         block);
  GAI_LAUNCH_CHECK();
}

void gai_embedding(const int* ids, const void* table, void* out, int T, int D, int vstart, int vend, hipStream_t st) {
  if (T == 0) return;
  const long n = (long)T * (D / 8);
  embedding_kernel<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(ids, (const bf16*)table, (bf16*)out, T, D, vstart,
                                                                 vend);
  GAI_LAUNCH_CHECK();
}

void gai_pool(const void* h, const int* cu, float* out, int B, int D, int mode, int normalize, hipStream_t st) {
  if (B == 0) return;
  pool_kernel<<<B, 256, (D + 16) * sizeof(float), st>>>((const bf16*)h, cu, out, D, mode, normalize);
  GAI_LAUNCH_CHECK();
}

void gai_silu_mul(const void* x, void* y, int T, int I, hipStream_t st) {
  if (T == 0) return;
  const long n = (long)T * (I / 8);
  act_kernel<0><<<(unsigned)((n + 255) / 256), 256, 0, st>>>((const bf16*)x, (bf16*)y, T, I);
  GAI_LAUNCH_CHECK();
}

void gai_silu_mul_interleaved(const void* x, void* y, int T, int I, hipStream_t st) {
  if (T == 0) return;
  const long n = (long)T * (I / 8);
  act_kernel<2><<<(unsigned)((n + 255) / 256), 256, 0, st>>>((const bf16*)x, (bf16*)y, T, I);
  GAI_LAUNCH_CHECK();
}

void gai_gelu_tanh(const void* x, void* y, int T, int I, hipStream_t st) {
  if (T == 0) return;
  const long n = (long)T * (I / 8);
  act_kernel<3><<<(unsigned)((n + 255) / 256), 256, 0, st>>>((const bf16*)x, (bf16*)y, T, I);
  GAI_LAUNCH_CHECK();
}

void gai_geglu_interleaved(const void* x, void* y, int T, int I, hipStream_t st) {
  if (T == 0) return;
  const long n = (long)T * (I / 8);
  act_kernel<4><<<(unsigned)((n + 255) / 256), 256, 0, st>>>((const bf16*)x, (bf16*)y, T, I);
  GAI_LAUNCH_CHECK();
}

void gai_gelu(const void* x, void* y, int T, int I, hipStream_t st) {
  if (T == 0) return;
  const long n = (long)T * (I / 8);
  act_kernel<1><<<(unsigned)((n + 255) / 256), 256, 0, st>>>((const bf16*)x, (bf16*)y, T, I);
  GAI_LAUNCH_CHECK();
}
