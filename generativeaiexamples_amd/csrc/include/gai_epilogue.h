// GEMM epilogue shared by the bf16 and fp8 GEMM kernels: bias / activation / residual, bf16 or fp32 out.
#pragma once
#include "gai_common.h"

namespace gai {

enum { EPI_NONE = 0, EPI_BIAS = 1, EPI_BIAS_GELU = 2, EPI_RESIDUAL = 3, EPI_SWIGLU = 4, EPI_BIAS_RESIDUAL = 5,
       EPI_BIAS_RELU = 6, EPI_BIAS_QUICKGELU = 7 };

__device__ __forceinline__ float quick_gelu(float x) { return x / (1.0f + __expf(-1.702f * x)); }

template <int EPI, bool OUTF32>
__device__ __forceinline__ void store_out(void* C, const bf16* bias, const bf16* R, int ldc, int m, int n, float v) {
  if (EPI == EPI_BIAS || EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_RESIDUAL || EPI == EPI_BIAS_RELU ||
      EPI == EPI_BIAS_QUICKGELU)
    v += (float)bias[n];
  if (EPI == EPI_BIAS_GELU) v = gelu_erf(v);
  if (EPI == EPI_BIAS_RELU) v = fmaxf(v, 0.f);
  if (EPI == EPI_BIAS_QUICKGELU) v = quick_gelu(v);
  // residual with bf16 output = the unfused pair: bf16 projection output, then the add rounded again (the rounding of
  // the decode add+RMSNorm tails and of norm_kernel's residual add, so a fused prefill residual is bitwise theirs)
  if (EPI == EPI_RESIDUAL || EPI == EPI_BIAS_RESIDUAL) v = (OUTF32 ? v : (float)(bf16)v) + (float)R[(size_t)m * ldc + n];
  if (OUTF32)
    reinterpret_cast<float*>(C)[(size_t)m * ldc + n] = v;
  else
    reinterpret_cast<bf16*>(C)[(size_t)m * ldc + n] = (bf16)v;
}

}  // namespace gai
