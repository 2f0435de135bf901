// RMSNorm / LayerNorm with optional fused residual add.
//
// One wave64 per row, 16-byte (bf16x8) vectorised loads, the whole row held in
// registers (NCH chunks of 512 elements per lane-sweep), fp32 statistics.
// Fused residual: r = x + residual (rounded to bf16, matching torch bf16
// semantics); residual <- r when `residual_out` is set; y = norm(r) * w (+ b).
#include "gai_common.h"
#include "gai_kernels.h"

using namespace gai;

namespace {

template <int NCH, bool LAYERNORM>
__global__ __launch_bounds__(256) void norm_kernel(const bf16* __restrict__ x, const bf16* residual_in,
                                                   bf16* residual_out, const bf16* __restrict__ w,
                                                   const bf16* __restrict__ b, bf16* __restrict__ out, int T,
                                                   int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= T) return;
  const size_t base = (size_t)row * D;
  // Issue every load of the row (x, residual, gamma) before the first store: residual_out usually
  // aliases residual_in, so a store inside the load loop would pin each later load behind it and
  // serialise NCH memory round trips (10+ us for a 64-row decode norm instead of one trip).
  bf16x8 xa[NCH], ra[NCH], ga[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int idx = (c * 64 + lane) * 8;
    if (idx < D) {
      xa[c] = load8(x + base + idx);
      ra[c] = residual_in ? load8(residual_in + base + idx) : bf16x8{};
      ga[c] = load8(w + idx);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int idx = (c * 64 + lane) * 8;
    if (idx < D) {
      bf16x8 a = xa[c];
      if (residual_in) {
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = (bf16)((float)a[j] + (float)ra[c][j]);
        xa[c] = a;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s += LAYERNORM ? (float)a[j] : (float)a[j] * (float)a[j];
    }
  }
  if (residual_in && residual_out) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int idx = (c * 64 + lane) * 8;
      if (idx < D) store8(residual_out + base + idx, xa[c]);
    }
  }
  s = wave_sum(s);
  float mean = 0.f, inv;
  if (LAYERNORM) {
    mean = s / D;
    float q = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int idx = (c * 64 + lane) * 8;
      if (idx < D) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = (float)xa[c][j] - mean;
          q += d * d;
        }
      }
    }
    q = wave_sum(q);
    inv = rsqrtf(q / D + eps);
  } else {
    inv = rsqrtf(s / D + eps);
  }
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int idx = (c * 64 + lane) * 8;
    if (idx < D) {
      const bf16x8 g = ga[c];
      bf16x8 o;
      if (LAYERNORM) {
        const bf16x8 bb = b ? load8(b + idx) : bf16x8{};
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (bf16)(((float)xa[c][j] - mean) * inv * (float)g[j] + (b ? (float)bb[j] : 0.f));
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (bf16)((float)xa[c][j] * inv * (float)g[j]);
      }
      store8(out + base + idx, o);
    }
  }
}

template <bool LN>
void dispatch_norm(const void* x, const void* rin, void* rout, const void* w, const void* b, void* out, int T,
                   int D, float eps, hipStream_t st) {
  const dim3 grid((T + 3) / 4), block(256);
  const int nch = (D + 511) / 512;
#define GAI_NORM_CASE(N)                                                                                   \
  if (nch <= N) {                                                                                          \
    norm_kernel<N, LN><<<grid, block, 0, st>>>((const bf16*)x, (const bf16*)rin, (bf16*)rout,             \
                                                (const bf16*)w, (const bf16*)b, (bf16*)out, T, D, eps);   \
    GAI_LAUNCH_CHECK();                                                                                    \
    return;                                                                                                \
  }
  GAI_NORM_CASE(1)
  GAI_NORM_CASE(2)
  GAI_NORM_CASE(3)
  GAI_NORM_CASE(4)
  GAI_NORM_CASE(8)
  GAI_NORM_CASE(16)
#undef GAI_NORM_CASE
  gai_launch_error(__FILE__, __LINE__, "norm: hidden size > 8192 unsupported");
}

}  // namespace

void gai_rmsnorm(const void* x, const void* residual_in, void* residual_out, const void* w, void* out, int T, int D,
                 float eps, hipStream_t st) {
  if (T == 0) return;
  dispatch_norm<false>(x, residual_in, residual_out, w, nullptr, out, T, D, eps, st);
}

void gai_layernorm(const void* x, const void* residual_in, void* residual_out, const void* w, const void* b,
                   void* out, int T, int D, float eps, hipStream_t st) {
  if (T == 0) return;
  dispatch_norm<true>(x, residual_in, residual_out, w, b, out, T, D, eps, st);
}
