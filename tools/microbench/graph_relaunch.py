"""Does relaunching a hipGraph exec that is still executing block the host (ROCm)? A graph of many small kernels
(like an 8-step decode run: ~2000 nodes) is replayed back to back (same exec) and alternately from two execs
captured from the same code; prints host time per replay call and GPU time per replay.

python tools/microbench/graph_relaunch.py
"""
import time

import torch


def build(nodes, x):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            y = x
            for _ in range(nodes):
                y = y * 1.0001 + 0.5
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        y = x
        for _ in range(nodes):
            y = y * 1.0001 + 0.5  # 2 kernels per iteration
        x.copy_(y)
    return g


def main():
    x = torch.randn(64 * 4096, device="cuda")
    big = torch.randn(64 << 20, device="cuda")  # a ~256 MB stream to make each replay take a while
    for nodes in (100, 1000):
        g1 = build(nodes, x)
        g2 = build(nodes, x)
        for name, gs in (("same exec", [g1, g1]), ("two execs alternating", [g1, g2])):
            torch.cuda.synchronize()
            host = []
            t0 = time.perf_counter()
            for i in range(20):
                big.mul_(1.0000001)  # ~0.1 ms of GPU work so replays queue behind each other
                th = time.perf_counter()
                gs[i % 2].replay()
                host.append(time.perf_counter() - th)
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) / 20
            host.sort()
            print(f"{nodes * 2 + 1:5d} nodes, {name:22s}: host per replay call median {1e3 * host[10]:.3f} ms, "
                  f"max {1e3 * host[-1]:.3f} ms; wall per iteration {1e3 * wall:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
