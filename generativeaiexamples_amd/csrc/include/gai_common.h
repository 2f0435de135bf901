// Common device-side definitions for the gfx950 (CDNA4, MI355X) kernels.
//
// Everything here is written for wave64 + MFMA: vector types that match the
// MFMA operand registers, wave reductions over 64 lanes, and small helpers
// for 16-byte vectorised bf16 access (hipcc does not auto-vectorise bf16).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gai {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kWave = 64;

#define GAI_LDS(p) ((__attribute__((address_space(3))) void*)(p))

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Reduce within aligned groups of `W` lanes (W power of two <= 64).
template <int W>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = W / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int W>
__device__ __forceinline__ float group_max(float v) {
#pragma unroll
  for (int o = W / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ bf16x8 load8(const bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }
__device__ __forceinline__ void store8(bf16* p, bf16x8 v) { *reinterpret_cast<bf16x8*>(p) = v; }

// ---- fp8 KV cache (OCP e4m3fn, gfx950 native conversions) ----
typedef uint8_t fp8;
// 8 fp8 values (one 8-byte load) -> 8 bf16, each multiplied by `s` (v_cvt_scalef32_pk_bf16_fp8)
__device__ __forceinline__ bf16x8 fp8x8_to_bf16(uint2 v, float s) {
  const bf16x2 a = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(v.x, s, false);
  const bf16x2 b = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(v.x, s, true);
  const bf16x2 c = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(v.y, s, false);
  const bf16x2 d = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(v.y, s, true);
  return bf16x8{a[0], a[1], b[0], b[1], c[0], c[1], d[0], d[1]};
}
// 4 floats * inv_s -> 4 packed e4m3fn bytes, saturated to +-448
__device__ __forceinline__ uint32_t f32x4_to_fp8(float a, float b, float c, float d, float inv_s) {
  auto sat = [&](float x) { return fminf(fmaxf(x * inv_s, -448.f), 448.f); };
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(sat(a), sat(b), 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(sat(c), sat(d), w, true);
  return (uint32_t)w;
}
// 8 cache elements -> bf16x8: a plain 16-byte load for bf16, an 8-byte load + conversion for fp8
__device__ __forceinline__ bf16x8 load_kv8(const bf16* p, float) { return load8(p); }
__device__ __forceinline__ bf16x8 load_kv8(const fp8* p, float s) {
  return fp8x8_to_bf16(*reinterpret_cast<const uint2*>(p), s);
}

__device__ __forceinline__ float silu(float x) { return x / (1.0f + __expf(-x)); }
// erf by Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7), branch-free: one v_rcp_f32, one v_exp_f32 and ~10 FMAs per
// element. The device libm erff is piecewise with data-dependent branches: in the 256x256 GEMM epilogue of an encoder
// FFN-up projection (K = 1024, so the epilogue is not hidden behind a long main loop) it made the bias + GELU GEMM
// 2x slower than the bias-only one (e5-large ingest at M = 65536: 990 vs ~450 us per layer, profiles/r6).
__device__ __forceinline__ float erf_fast(float x) {
  const float z = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float y = 1.0f - p * t * __builtin_amdgcn_exp2f(-z * z * 1.4426950408889634f);
  return copysignf(y, x);
}
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erf_fast(x * 0.70710678118654752f)); }
// tanh-GELU as x * sigmoid(2u): 0.5 x (1 + tanh(u)) == x / (1 + e^{-2u}), no libm tanhf
__device__ __forceinline__ float gelu_tanh(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float u = k0 * fmaf(k1 * x, x * x, x);
  return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-2.0f * 1.4426950408889634f * u));
}

// Block-level reduction for up to 1024 threads (16 waves). `scratch` holds >= 16 floats.
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = 0.f;
  for (int i = 0; i < nw; ++i) r += scratch[i];
  return r;
}

__device__ __forceinline__ float block_max(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = -INFINITY;
  for (int i = 0; i < nw; ++i) r = fmaxf(r, scratch[i]);
  return r;
}

// XCD-aware, bijective remap of a linear workgroup id (cdna_hip_programming §5 T1):
// consecutive logical ids land on the same XCD (blocks b and b+8 share one).
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

}  // namespace gai

#define GAI_LAUNCH_CHECK()                                                        \
  do {                                                                            \
    hipError_t e_ = hipGetLastError();                                            \
    if (e_ != hipSuccess) gai_launch_error(__FILE__, __LINE__, hipGetErrorString(e_)); \
  } while (0)

void gai_launch_error(const char* file, int line, const char* msg);
