// bf16 GEMM instantiations for the residual, bias + residual epilogues (gemm_impl.h; dispatched by gai_gemm in gemm.hip).
#include "gemm_impl.h"

GAI_GEMM_RUN(3)
GAI_GEMM_RUN(5)
