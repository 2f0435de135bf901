"""Prefill GEMM A/B: the hand-written persistent kernels (w4p / w4d / w4r) vs hipBLASLt (default + tuned table) on the
Llama-3-8B projection shapes at M = 16384 (one 16K-token prefill chunk; --m 2406 = one RAG query), plus the
stream-K walk (w4s) and the 128x128 tiled kernel, random operands, interleaved
rounds in one process (cdna_hip_programming §5.4 rules 24/25). One JSON line per shape.

usage: python tools/gemm_bench.py [--m 16384[,2406,...]] [--rounds 5] [--out FILE]
"""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from generativeaiexamples_amd import ops
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from blas_ab import enable_tuned_blas  # noqa: E402  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "e5_ffn_up": (4096, 1024), "e5_qkv": (3072, 1024), "e5_o": (1024, 1024), "e5_down": (1024, 4096),
          # one rank of Llama-3-70B at TP = 8 (tools/tp_rank_profile.py)
          "tp8_qkv": (1280, 8192), "tp8_o": (8192, 1024), "tp8_gate_up": (7168, 8192), "tp8_down": (8192, 3584)}


def timeit(fn, iters=10):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", default="16384", help="comma-separated M values")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--out", default=None)
    ap.add_argument("--cold", action="store_true",
                    help="cycle operand copies (> 512 MB in all) so weights / activations stream from HBM as in the "
                         "model, not from the 256 MB Infinity Cache")
    a = ap.parse_args()
    nat = ops.native()
    rows = []
    for M, name in [(int(m), n) for m in str(a.m).split(",") for n in a.shapes.split(",")]:
        N, K = SHAPES[name]
        ncopy = max(1, -(-(512 << 20) // ((M + N) * K * 2))) if a.cold else 1
        xs = [torch.randn(M, K, device="cuda", dtype=torch.bfloat16) for _ in range(ncopy)]
        ws = [(torch.randn(N, K, device="cuda") / math.sqrt(K)).to(torch.bfloat16) for _ in range(ncopy)]
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        it = [0]

        def op():  # the next operand pair (one pair unless --cold)
            it[0] = (it[0] + 1) % ncopy
            return xs[it[0]], ws[it[0]]

        def g(force):
            x, w = op()
            nat.gemm(x, w, out, None, None, 0, force)

        def blas():
            x, w = op()
            torch.mm(x, w.t())
        arms = {"auto": lambda: g(0), "w4p": lambda: g(8), "w4d": lambda: g(9), "w4r": lambda: g(10),
                "w4s": lambda: g(11), "w4x": lambda: g(12), "w4d192": lambda: g(13), "tiled": lambda: g(2),
                "hipblaslt": blas}
        ts = {k: [] for k in arms}
        for _ in range(a.rounds):
            for k, f in arms.items():
                ts[k].append(timeit(f))
        fl = 2 * M * N * K
        r = {"gemm": name, "M": M, "N": N, "K": K, "cold": bool(a.cold)}
        for k, v in ts.items():
            v.sort()
            r[f"{k}_ms"] = round(v[len(v) // 2], 4)
            r[f"{k}_tflops"] = round(fl / v[len(v) // 2] / 1e9, 1)
        r["w4p_vs_blas"] = round(r["hipblaslt_ms"] / r["w4p_ms"], 3)
        r["w4d_vs_blas"] = round(r["hipblaslt_ms"] / r["w4d_ms"], 3)
        r["w4r_vs_blas"] = round(r["hipblaslt_ms"] / r["w4r_ms"], 3)
        r["w4s_vs_blas"] = round(r["hipblaslt_ms"] / r["w4s_ms"], 3)
        r["w4x_vs_blas"] = round(r["hipblaslt_ms"] / r["w4x_ms"], 3)
        r["w4d192_vs_blas"] = round(r["hipblaslt_ms"] / r["w4d192_ms"], 3)
        r["auto_vs_blas"] = round(r["hipblaslt_ms"] / r["auto_ms"], 3)
        print(json.dumps(r), flush=True)
        rows.append(r)
    if not a.cold and enable_tuned_blas():
        for r in rows:
            M, N, K = r["M"], r["N"], r["K"]
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            w = (torch.randn(N, K, device="cuda") / math.sqrt(K)).to(torch.bfloat16)
            t = sorted(timeit(lambda: torch.mm(x, w.t())) for _ in range(a.rounds))[a.rounds // 2]
            r["hipblaslt_tuned_ms"] = round(t, 4)
            r["hipblaslt_tuned_tflops"] = round(2 * M * N * K / t / 1e9, 1)
            print(json.dumps({"gemm": r["gemm"], "tuned_tflops": r["hipblaslt_tuned_tflops"]}), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
