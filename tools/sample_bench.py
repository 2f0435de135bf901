"""Sampler timing on the headline shape: 64 rows x 128256 vocab, fp32 logits (random-init Llama-3 scale).

    python tools/sample_bench.py  ->  one JSON line per case (us per call, CUDA-event timed)
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from generativeaiexamples_amd import ops  # noqa: E402


def main():
    dev = "cuda"
    B, V = 64, 128256
    torch.manual_seed(0)
    # scale 1.0 / T 0.2 / p 0.7 = the headline bench (random-init lm_head std 1/sqrt(d): unit-variance logits)
    cases = [("greedy", 1.28, 0.0, 1.0), ("T0.2_p0.7", 1.28, 0.2, 0.7), ("bench_T0.2_p0.7", 1.0, 0.2, 0.7),
             ("T1_p0.9", 3.0, 1.0, 0.9),
             ("flat_T1_p0.9", 0.01, 1.0, 0.9), ("T0.7_p1", 1.28, 0.7, 1.0)]
    for name, scale, T, p in cases:
        logits = torch.randn(B, V, device=dev) * scale
        temp = torch.full((B,), T, device=dev)
        top_p = torch.full((B,), p, device=dev)
        top_k = torch.zeros(B, dtype=torch.int32, device=dev)
        seeds = torch.arange(B, dtype=torch.int64, device=dev)
        for _ in range(3):
            ops.sample(logits, temp, top_p, top_k, seeds, 0)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 50
        s.record()
        for i in range(n):
            ops.sample(logits, temp, top_p, top_k, seeds, i)
        e.record()
        torch.cuda.synchronize()
        print(json.dumps({"case": name, "rows": B, "vocab": V, "us": round(s.elapsed_time(e) * 1000 / n, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
