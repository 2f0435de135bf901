"""Run one GEMM arm repeatedly (for rocprofv3 PMC passes): python tools/gemm_one.py ARM N K [M] [iters]
ARM: w4p | w4d | w4r | blas (hipBLASLt); the ring / large stepping stones left the build in round 4."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from generativeaiexamples_amd import ops  # noqa: E402

arm, N, K = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
M = int(sys.argv[4]) if len(sys.argv) > 4 else 16384
iters = int(sys.argv[5]) if len(sys.argv) > 5 else 30
x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
w = (torch.randn(N, K, device="cuda") / math.sqrt(K)).to(torch.bfloat16)
out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
force = {"w4p": 8, "w4d": 9, "w4r": 10}.get(arm)
nat = ops.native()
for _ in range(iters):
    if force is None:
        torch.mm(x, w.t(), out=out)
    else:
        nat.gemm(x, w, out, None, None, 0, force)
torch.cuda.synchronize()
print("done", arm, M, N, K)
