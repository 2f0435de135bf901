// bf16 GEMM instantiations for the SwiGLU, bias + quick-GELU epilogues (gemm_impl.h; dispatched by gai_gemm in gemm.hip).
#include "gemm_impl.h"

GAI_GEMM_RUN(4)
GAI_GEMM_RUN(7)
