// Gated DeltaNet recurrent decode step (Qwen3-Next linear-attention layers).
//
// Per (sequence b, value head h) the layer keeps a fp32 state S [DK][DV] in a slot pool; one decode
// token applies
//     S <- exp(g) S;  m = S^T k;  d = beta (v - m);  S <- S + k d^T;  o = S^T q
// (q, k l2-normalised, q pre-scaled by DK^-1/2). The step is a pure state stream: read + write
// DK*DV*4 bytes per head, ~4 flops per byte, so it is HBM-bound. One workgroup per (h, b); thread (r, j)
// owns rows [32r, 32r+32) of state column j: it walks the DK rows with coalesced 4-B loads (a row of DV floats is
// contiguous across the workgroup), keeps its slice of the column in VGPRs between the read and the
// write-back, and q / k live in LDS. The update is in place through `slots` (no gather / scatter copies), so the
// launch is graph-capturable with the slot vector as a static input.
#include "gai_common.h"
#include "gai_kernels.h"

using namespace gai;

namespace {

// DK / 32 row groups x 128 columns: thread (r, j) keeps rows [32r, 32r + 32) of column j in VGPRs;
// the two column reductions (m = S^T k, o = S^T q) combine the row groups through LDS.
template <int DK>
__global__ __launch_bounds__(DK * 4) void gdn_decode_kernel(const float* __restrict__ q, const float* __restrict__ k,
                                                            const float* __restrict__ v, const float* __restrict__ g,
                                                            const float* __restrict__ beta, float* __restrict__ state,
                                                            const int* __restrict__ slots, float* __restrict__ out,
                                                            int Hv, int DV) {
  constexpr int RG = DK / 32;
  __shared__ float qs[DK], ks[DK], red[RG][128];
  const int h = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int j0 = tid & 127, r = tid >> 7;  // r is wave-uniform (128 = 2 waves)
  const size_t bh = (size_t)b * Hv + h;
  if (tid < DK) {
    qs[tid] = q[bh * DK + tid];
    ks[tid] = k[bh * DK + tid];
  }
  __syncthreads();
  const float eg = __expf(g[bh]), bt = beta[bh];
  float* S = state + ((size_t)slots[b] * Hv + h) * DK * DV + (size_t)(32 * r) * DV;
  for (int jb = 0; jb < DV; jb += 128) {
    const int j = jb + j0;
    const bool on = j < DV;
    float col[32];
    float m = 0.f;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      col[i] = on ? S[(size_t)i * DV + j] * eg : 0.f;
      m += col[i] * ks[32 * r + i];
    }
    red[r][j0] = m;
    __syncthreads();
    m = 0.f;
#pragma unroll
    for (int t = 0; t < RG; ++t) m += red[t][j0];
    const float d = on ? (v[bh * DV + j] - m) * bt : 0.f;
    float o = 0.f;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      col[i] += ks[32 * r + i] * d;
      o += col[i] * qs[32 * r + i];
      if (on) S[(size_t)i * DV + j] = col[i];
    }
    __syncthreads();  // every thread has read red[][] for m
    red[r][j0] = o;
    __syncthreads();
    if (r == 0 && on) {
      float acc = 0.f;
#pragma unroll
      for (int t = 0; t < RG; ++t) acc += red[t][j0];
      out[bh * DV + j] = acc;
    }
    __syncthreads();
  }
}

}  // namespace

void gai_gdn_decode(const float* q, const float* k, const float* v, const float* g, const float* beta, float* state,
                    const int* slots, float* out, int B, int Hv, int DK, int DV, hipStream_t st) {
  if (B == 0) return;
  const dim3 grid(Hv, B);
#define GAI_GDN(D)                                                                                    \
  if (DK == D) {                                                                                      \
    gdn_decode_kernel<D><<<grid, D * 4, 0, st>>>(q, k, v, g, beta, state, slots, out, Hv, DV);        \
    GAI_LAUNCH_CHECK();                                                                               \
    return;                                                                                           \
  }
  GAI_GDN(64)
  GAI_GDN(128)
  GAI_GDN(256)
#undef GAI_GDN
  gai_launch_error(__FILE__, __LINE__, "gdn_decode: key head dim must be 64, 128 or 256");
}
