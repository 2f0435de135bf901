"""Time ops.moe_dispatch (native single-workgroup kernel vs the stable-argsort plan) by row count.
python tools/microbench/moe_dispatch.py"""
import time

import torch

from generativeaiexamples_amd import ops

E, k = 8, 2
for T in (32, 64, 512, 2048, 8192, 16384):
    ids = torch.randint(0, E, (T, k), device="cuda", dtype=torch.int32)
    res = {}
    for name, cap in (("native", 1 << 30), ("argsort", 0)):
        ops._MOE_DISPATCH_MAX = cap
        for _ in range(3):
            ops.moe_dispatch(ids, E)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(20):
                ops.moe_dispatch(ids, E)
        g.replay()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(5):
            g.replay()
        torch.cuda.synchronize()
        res[name] = (time.perf_counter() - t) / 100 * 1e6
    print(f"rows {T * k}: native {res['native']:.1f} us, argsort {res['argsort']:.1f} us", flush=True)
