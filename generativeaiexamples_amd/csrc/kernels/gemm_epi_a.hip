// bf16 GEMM instantiations for the none, bias epilogues (gemm_impl.h; dispatched by gai_gemm in gemm.hip).
#include "gemm_impl.h"

GAI_GEMM_RUN(0)
GAI_GEMM_RUN(1)
