"""hipBLASLt (torch.mm) on the Llama-3-8B projection shapes, for reading the winning library kernels' names
(macro tile, MFMA, workgroup shape) out of a rocprofv3 kernel trace: a reference design point, not a code path.

rocprofv3 --kernel-trace --stats -d out -o run -- python3 tools/microbench/blas_shapes.py --m 16384
"""
import argparse
import math

import torch

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}

ap = argparse.ArgumentParser()
ap.add_argument("--m", default="16384,2406")
ap.add_argument("--iters", type=int, default=10)
a = ap.parse_args()
for M in [int(x) for x in a.m.split(",")]:
    for name, (N, K) in SHAPES.items():
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = (torch.randn(N, K, device="cuda") / math.sqrt(K)).to(torch.bfloat16)
        for _ in range(a.iters):
            torch.mm(x, w.t())
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            torch.mm(x, w.t())
        e.record()
        e.synchronize()
        ms = s.elapsed_time(e) / a.iters
        print(f"{name} M={M}: {ms * 1e3:.1f} us, {2 * M * N * K / ms / 1e9:.0f} TF/s", flush=True)
