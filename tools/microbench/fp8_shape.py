"""Time one fp8 GEMM shape on the 128x128 (force 2) and 256x256 (force 3) fp8 kernels.
python tools/microbench/fp8_shape.py M N K [epi]"""
import sys
import time

import torch

from generativeaiexamples_amd import ops

M, N, K = (int(v) for v in sys.argv[1:4])
epi = int(sys.argv[4]) if len(sys.argv) > 4 else 0
x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
w = ops.Fp8Weight.quantize((torch.randn(N, K, device="cuda") / K ** 0.5).to(torch.bfloat16))
xq, sx = ops.quant_fp8(x)
bias = torch.randn(N, device="cuda", dtype=torch.bfloat16) if epi in (1, 2, 5, 6, 7) else None
res = torch.randn(M, N, device="cuda", dtype=torch.bfloat16) if epi in (3, 5) else None
out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
nat = ops.native()
for force in (2, 3):
    f = lambda: nat.gemm_fp8(xq, w.q, sx, w.scale, out, bias, res, epi, force)  # noqa: E731
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(10):
        f()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / 10
    print(f"M={M} N={N} K={K} epi={epi} force={force}: {dt * 1e6:.0f} us, {2 * M * N * K / dt / 1e15:.2f} PF/s")
