"""Exact index scan (sim_topk) vs torch mm + topk: N x 1024 bf16 rows, nq queries, k = 4, random data.
Prints one JSON line per (N, nq): ms, effective HBM GB/s of the X scan. usage: python tools/topk_bench.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from generativeaiexamples_amd import ops  # noqa: E402


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else None
    rows = []
    D = 1024
    for N in (1_000_000, 10_000_000):
        X = torch.randn(N, D, device="cuda", dtype=torch.bfloat16)
        bias = torch.zeros(N, device="cuda")
        for nq in (1, 16, 64):
            Q = torch.randn(nq, D, device="cuda", dtype=torch.bfloat16)
            t = timeit(lambda: ops.sim_topk(Q, X, bias, N, 4))
            t_ref = timeit(lambda: torch.topk(Q @ X.t(), 4, dim=-1)) if N <= 1_000_000 or nq <= 16 else None
            v, i = ops.sim_topk(Q, X, bias, N, 4)
            vr, ir = torch.topk((Q.float() @ X.float().t()) if N <= 1_000_000 else (Q @ X.t()).float(), 4, dim=-1)
            ok = bool(((v - vr).abs() <= 2e-2 * vr.abs() + 2e-2).all())
            r = dict(op="sim_topk", N=N, D=D, nq=nq, k=4, ours_ms=round(t, 4),
                     torch_ms=None if t_ref is None else round(t_ref, 4),
                     ours_tbs=round(N * D * 2 / t / 1e9, 3), speedup=None if t_ref is None else round(t_ref / t, 3),
                     matches_torch=ok)
            print(json.dumps(r), flush=True)
            rows.append(r)
        del X
        torch.cuda.empty_cache()
    if out:
        with open(out, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
