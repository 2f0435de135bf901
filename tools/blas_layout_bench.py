"""hipBLASLt layout probe for the prefill projections: y = x @ W^T with W stored [N, K] (NT) vs [K, N] (NN),
bf16, M = prefill chunk. Prints TFLOP/s per shape/layout (median of 10 timed calls)."""
import torch


def t(fn, it=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(it):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    return sorted(ts)[len(ts) // 2]


for M in (4096, 16384):
    for N, K, tag in ((6144, 4096, "qkv"), (4096, 4096, "o"), (28672, 4096, "gate_up"), (4096, 14336, "down")):
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
        wt = w.t().contiguous()
        fl = 2 * M * N * K
        a = t(lambda: x @ w.t())
        b = t(lambda: x @ wt)
        c = t(lambda: torch.mm(x, w.t(), out_dtype=torch.bfloat16)) if False else a
        print(f"M={M:6d} {tag:8s} NT {fl / a / 1e9:7.1f} TF/s  NN {fl / b / 1e9:7.1f} TF/s", flush=True)
