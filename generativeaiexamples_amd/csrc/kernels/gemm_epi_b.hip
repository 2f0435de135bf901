// bf16 GEMM instantiations for the bias + GELU, bias + ReLU epilogues (gemm_impl.h; dispatched by gai_gemm in gemm.hip).
#include "gemm_impl.h"

GAI_GEMM_RUN(2)
GAI_GEMM_RUN(6)
