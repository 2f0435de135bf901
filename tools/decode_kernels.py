"""Decode-only forward of a model on a synthetic paged KV cache (no prefill), for kernel traces:
B sequences at context C, N eager forward passes (kernel durations equal the in-graph ones).

rocprofv3 --kernel-trace --stats -d out -o run -- python3 tools/decode_kernels.py --batch 64 --ctx 2600
"""
import os
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
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--ctx", type=int, default=2600)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--no-psw", action="store_true", help="plain-layout decode weights (no fragment copies)")
    a = ap.parse_args()
    m, tok, name = build_llm(a.model, device="cuda")
    if not a.no_psw:
        m.preshuffle_decode_weights(in_place=os.environ.get("GAI_WEIGHT_LAYOUT", "fragment") == "fragment")  # as LLMEngine
    c = m.cfg
    nbps = (a.ctx + 16) // 16 + 1
    kv = KVCache(getattr(m, "num_kv_layers", c.num_layers), a.batch * nbps + 1, m.hkv, c.head_dim, m.device, m.dtype)
    kv.storage.normal_()
    B = a.batch
    bt = torch.arange(B * nbps, device="cuda", dtype=torch.int32).view(B, nbps)
    ctx = torch.full((B,), a.ctx, device="cuda", dtype=torch.int32)
    fb = ForwardBatch(token_ids=torch.randint(10, 1000, (B,), device="cuda", dtype=torch.int32),
                      positions=torch.full((B,), a.ctx - 1, device="cuda", dtype=torch.int32),
                      slots=(bt[:, (a.ctx - 1) // 16] * 16 + (a.ctx - 1) % 16).int(), num_prefill_tokens=0,
                      decode_ctx=ctx, decode_block_tables=bt, max_decode_ctx=a.ctx, sample_rows=None)
    ws = ops.DecodeWorkspace(B, m.hq, c.head_dim, a.ctx + 64, "cuda")
    with torch.inference_mode():
        for _ in range(3):
            m.forward(fb, kv, ws)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            m.forward(fb, kv, ws)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.iters
        print(f"{name} decode B={B} ctx={a.ctx}: {1000 * dt:.3f} ms/forward (eager, includes launch overhead)")
        # the engine's path: the forward captured once, replayed (kernel boundaries only, no host launches)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            m.forward(fb, kv, ws)
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            g.replay()
        torch.cuda.synchronize()
        dg = (time.perf_counter() - t0) / a.iters
        print(f"{name} decode B={B} ctx={a.ctx}: {1000 * dg:.3f} ms/forward (graph replay)")


if __name__ == "__main__":
    main()
