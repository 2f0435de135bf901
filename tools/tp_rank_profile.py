"""Per-rank compute of a tensor-parallel generator on ONE GPU: rank r of a TP = N Llama shard
(default: Llama-3-70B, TP = 8, rank 0 - every rank's shard has the same shapes) with the TP collectives replaced by
identities, so the timings are the rank's kernels alone - exactly what each of the N GPUs computes between its
all-reduces. Not a scaling claim: the all-reduces (2 per layer + the embedding, 1 MiB per call at B = 64, d 8192)
run on xGMI in the real deployment and are reported apart (message sizes, count per step).

Measures, all at the rank's shard widths (70B / TP8: QKV [B, 8192] x [8192, 1280], O [B, 1024] x [1024, 8192],
gate_up [B, 8192] x [8192, 7168], down [B, 3584] x [3584, 8192], LM head V / 8 = 16,032 columns):
  * decode step at batch B (default 64), context C (default 2500): graph replay, ms per forward;
  * one prefill of T tokens (default 2407): ms (eager);
and writes a JSON record (--out). Under `rocprofv3 --kernel-trace --stats` (tools/gpu.sh pyprof) the kernel table
gives each projection's time; `--bytes-table` prints each decode projection's weight bytes for the HBM-rate column.

python tools/tp_rank_profile.py --model llama3-70b --tp 8 --batch 64 --ctx 2500 --tokens 2407 --out rank.json

Reference deployment: /root/reference/RAG/examples/basic_rag/langchain/docker-compose.yaml:29 (llama3-70b-instruct),
/root/reference/docs/support-matrix.md:19 (70B needs 8 GPUs' memory).
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from generativeaiexamples_amd import ops  # noqa: E402
from generativeaiexamples_amd.engine.kv_cache import KVCache  # noqa: E402
from generativeaiexamples_amd.models import LlamaConfig, LlamaModel  # noqa: E402
from generativeaiexamples_amd.models.common import ForwardBatch  # noqa: E402
from generativeaiexamples_amd.parallel.dist import DistContext  # noqa: E402


class ShardRankContext(DistContext):
    """One rank of a TP group, alone: the model shards its weights for (tp_size, rank) but every collective is the
    identity (all-reduce of a rank's partial sum = itself; the vocab all-gather keeps the local V / tp logits). The
    fused all-reduce + add + RMSNorm of the TP block boundary becomes the plain fused add + RMSNorm kernel."""

    def tp_all_reduce(self, t):
        return t

    def tp_linear_all_reduce(self, x, w, bias=None, chunks=None):
        return ops.linear(x, w, bias=bias)

    def tp_all_reduce_rmsnorm(self, h, residual, w, eps):
        return ops.rms_norm(h, w, eps, residual=residual)

    def tp_all_gather_last(self, t):
        return t

    def tp_reduce_scatter_rows(self, t):
        return t

    def tp_all_gather_rows(self, t):
        return t


def build(model: str, tp: int, rank: int, layers: int):
    cfg = {"llama3-70b": LlamaConfig.llama3_70b, "llama3-8b": LlamaConfig.llama3_8b}[model]()
    if layers:
        import dataclasses
        cfg = dataclasses.replace(cfg, num_layers=layers)
    ctx = ShardRankContext(rank=rank, world_size=tp, tp_size=tp, device=torch.device("cuda", 0))
    m = LlamaModel(cfg, device="cuda", dist_ctx=ctx).random_init(5)
    return m


def decode_batch(m, B, C):
    c = m.cfg
    nbps = (C + 16) // 16 + 1
    kv = KVCache(c.num_layers, B * nbps + 1, m.hkv, c.head_dim, m.device, m.dtype)
    kv.storage.normal_()
    bt = torch.arange(B * nbps, device="cuda", dtype=torch.int32).view(B, nbps)
    fb = ForwardBatch(token_ids=torch.randint(10, 1000, (B,), device="cuda", dtype=torch.int32),
                      positions=torch.full((B,), C - 1, device="cuda", dtype=torch.int32),
                      slots=(bt[:, (C - 1) // 16] * 16 + (C - 1) % 16).int(), num_prefill_tokens=0,
                      decode_ctx=torch.full((B,), C, device="cuda", dtype=torch.int32), decode_block_tables=bt,
                      max_decode_ctx=C, sample_rows=None)
    return fb, kv


def prefill_batch(m, T):
    c = m.cfg
    nb = (T + ops.BLOCK - 1) // ops.BLOCK
    kv = KVCache(c.num_layers, nb + 1, m.hkv, c.head_dim, m.device, m.dtype)
    bt = torch.arange(1, nb + 1, device="cuda", dtype=torch.int32).view(1, nb)
    pos = torch.arange(T, device="cuda", dtype=torch.int32)
    fb = ForwardBatch(token_ids=torch.randint(10, 1000, (T,), device="cuda", dtype=torch.int32), positions=pos,
                      slots=(bt[0, pos.long() // ops.BLOCK] * ops.BLOCK + pos % ops.BLOCK).int(), num_prefill_tokens=T,
                      cu_q=torch.tensor([0, T], device="cuda", dtype=torch.int32),
                      prefill_ctx=torch.tensor([T], device="cuda", dtype=torch.int32), prefill_block_tables=bt,
                      prefill_tiles=ops.build_prefill_tiles([T], m.hq, m.hkv, "cuda", head_dim=c.head_dim), prefill_qlen=[T],
                      prefill_ctx_host=[T], sample_rows=torch.tensor([T - 1], device="cuda", dtype=torch.int64))
    return fb, kv


def weight_bytes(m) -> dict:
    w = m.w
    return {k: int(w["l0." + k].numel() * w["l0." + k].element_size()) for k in ("qkv", "o", "gate_up", "down")} | {
        "lm_head": int(w["lm_head"].numel() * w["lm_head"].element_size())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-70b")
    ap.add_argument("--tp", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--layers", type=int, default=0, help="0 = all layers of the model")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--ctx", type=int, default=2500)
    ap.add_argument("--tokens", type=int, default=2407)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    m = build(a.model, a.tp, a.rank, a.layers)
    m.preshuffle_decode_weights(in_place=os.environ.get("GAI_WEIGHT_LAYOUT", "fragment") == "fragment")  # as LLMEngine
    c = m.cfg
    shapes = {k: list(m.w["l0." + k].shape) for k in ("qkv", "o", "gate_up", "down")} | {
        "lm_head": list(m.w["lm_head"].shape)}
    rec = dict(model=c.name, tp=a.tp, rank=a.rank, layers=c.num_layers, batch=a.batch, ctx=a.ctx,
               prefill_tokens=a.tokens, shard_shapes=shapes, weight_bytes_per_layer=weight_bytes(m),
               shard_params_b=round(sum(t.numel() for t in m.w.values()) / 1e9, 3),
               all_reduce_per_step=dict(count=2 * c.num_layers + 1, bytes_decode=a.batch * c.hidden_size * 2,
                                        bytes_prefill=a.tokens * c.hidden_size * 2),
               collectives="identity (one rank's compute only)")
    print(f"[tp_rank] {c.name} TP={a.tp} rank {a.rank}: {rec['shard_params_b']}B params on this rank, shapes {shapes}",
          flush=True)
    with torch.inference_mode():
        fb, kv = decode_batch(m, a.batch, a.ctx)
        ws = ops.DecodeWorkspace(a.batch, m.hq, c.head_dim, a.ctx + 64, "cuda")
        for _ in range(3):
            m.forward(fb, kv, ws)
        torch.cuda.synchronize()
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
        rec["decode_ms_per_step"] = round(1000 * (time.perf_counter() - t0) / a.iters, 3)
        print(f"[tp_rank] decode B={a.batch} ctx={a.ctx}: {rec['decode_ms_per_step']} ms / step (graph replay)",
              flush=True)
        del g, kv, ws
        torch.cuda.empty_cache()
        fb, kv = prefill_batch(m, a.tokens)
        for _ in range(2):
            m.forward(fb, kv)
        torch.cuda.synchronize()
        ts = []
        for _ in range(max(3, a.iters // 4)):
            t0 = time.perf_counter()
            m.forward(fb, kv)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        ts.sort()
        rec["prefill_ms"] = round(1000 * ts[len(ts) // 2], 3)
        print(f"[tp_rank] prefill of {a.tokens} tokens: {rec['prefill_ms']} ms (eager, median)", flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
