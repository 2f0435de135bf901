"""Does hipBLASLt solution tuning (PyTorch TunableOp) beat the default heuristic on the prefill GEMMs?
Times y = x @ W^T for the Llama-3-8B prefill shapes (M = 16384 tokens) with the default selection, then
with PYTORCH_TUNABLEOP tuning on (results written to --csv for reuse with tuning off).

python tools/tunableop_probe.py --csv gpurun_out/tunableop_mi355x.csv
"""
import argparse
import json

import torch

SHAPES = [(16384, 6144, 4096, "qkv"), (16384, 4096, 4096, "o"), (16384, 28672, 4096, "gate_up"),
          (16384, 4096, 14336, "down"), (16384, 128256, 4096, "lm_head_all_rows")]


def bench(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--csv", default="gpurun_out/tunableop_mi355x.csv")
    a = ap.parse_args()
    data = []
    for M, N, K, name in SHAPES[:4]:
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
        data.append((name, M, N, K, x, w))
    base = {n: bench(lambda: torch.mm(x, w.t())) for n, M, N, K, x, w in data}
    import torch.cuda.tunable as tunable
    tunable.enable(True)
    tunable.tuning_enable(True)
    tunable.set_filename(a.csv)
    tunable.set_max_tuning_duration(3000)  # ms per shape
    for n, M, N, K, x, w in data:
        torch.mm(x, w.t())  # tunes this shape
    print(json.dumps({"tuned_entries": len(tunable.get_results())}), flush=True)
    tuned = {n: bench(lambda: torch.mm(x, w.t())) for n, M, N, K, x, w in data}
    for n, M, N, K, x, w in data:
        fl = 2 * M * N * K
        print(json.dumps({"gemm": n, "M": M, "N": N, "K": K, "default_ms": round(base[n], 4),
                          "tuned_ms": round(tuned[n], 4), "default_tflops": round(fl / base[n] / 1e9, 1),
                          "tuned_tflops": round(fl / tuned[n] / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
