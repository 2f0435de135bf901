"""Single-prompt prefill latency (the c1 TTFT's dominant term) of a model on a synthetic paged KV cache:
one prompt of --tokens tokens, N eager forward passes, logits of its last row only (as the engine samples).

rocprofv3 --kernel-trace --stats -d out -o run -- python3 tools/prefill_latency.py --tokens 2406
"""
import argparse
import time

import torch

from generativeaiexamples_amd import ops
from generativeaiexamples_amd.engine.kv_cache import KVCache
from generativeaiexamples_amd.models.common import ForwardBatch
from generativeaiexamples_amd.models.registry import build_llm


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--tokens", type=int, default=2406)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    m, tok, name = build_llm(a.model, device="cuda")
    c = m.cfg
    T = a.tokens
    nb = (T + ops.BLOCK - 1) // ops.BLOCK
    kv = KVCache(getattr(m, "num_kv_layers", c.num_layers), nb + 1, m.hkv, c.head_dim, m.device, m.dtype)
    bt = torch.arange(1, nb + 1, device="cuda", dtype=torch.int32).view(1, nb)
    pos = torch.arange(T, device="cuda", dtype=torch.int32)
    slots = (bt[0, pos.long() // ops.BLOCK] * ops.BLOCK + pos % ops.BLOCK).int()
    fb = ForwardBatch(token_ids=torch.randint(10, 1000, (T,), device="cuda", dtype=torch.int32), positions=pos,
                      slots=slots, num_prefill_tokens=T,
                      cu_q=torch.tensor([0, T], device="cuda", dtype=torch.int32),
                      prefill_ctx=torch.tensor([T], device="cuda", dtype=torch.int32), prefill_block_tables=bt,
                      prefill_tiles=ops.build_prefill_tiles([T], m.hq, m.hkv, "cuda", head_dim=c.head_dim), prefill_qlen=[T],
                      prefill_ctx_host=[T], sample_rows=torch.tensor([T - 1], device="cuda", dtype=torch.int64))
    with torch.inference_mode():
        for _ in range(3):
            m.forward(fb, kv)
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.iters):
            t0 = time.perf_counter()
            m.forward(fb, kv)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
    ts.sort()
    print(f"{name} prefill of one {T}-token prompt: median {1000 * ts[len(ts) // 2]:.2f} ms, "
          f"min {1000 * ts[0]:.2f} ms (eager, includes launch overhead)")


if __name__ == "__main__":
    main()
