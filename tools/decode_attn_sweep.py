"""Decode-attention bandwidth sweep over split length for the kernel variant chosen by
GAI_DECODE_VARIANT (read once per process), plus a numerics check against the fp32 reference.

GAI_DECODE_VARIANT=1 python tools/decode_attn_sweep.py --batch 64 --ctx 2600
"""
import argparse
import json
import math
import os

import torch

from generativeaiexamples_amd import ops
from generativeaiexamples_amd.ops import reference as ref


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--ctx", type=int, default=2600)
    ap.add_argument("--splits", default="384,512,640,768,896,1024,1280")
    a = ap.parse_args()
    B, ctx, Hq, Hkv, D = a.batch, a.ctx, 32, 8, 128
    nbps = (ctx + 15) // 16
    nb = B * nbps
    torch.manual_seed(0)
    kc = torch.randn(nb, Hkv, 16, D, device="cuda", dtype=torch.bfloat16)
    vc = torch.randn(nb, Hkv, D, 16, device="cuda", dtype=torch.bfloat16)
    bt = torch.randperm(nb, device="cuda").int().reshape(B, nbps)
    q = torch.randn(B, Hq, D, device="cuda", dtype=torch.bfloat16)
    cl = torch.randint(ctx - 300, ctx + 1, (B,), device="cuda", dtype=torch.int32)
    scale = 1 / math.sqrt(D)
    want = ref.attention_decode(q[:4].cpu(), kc.cpu(), vc.cpu(), bt[:4].cpu(), cl[:4].cpu(), scale).float()
    by = 2 * int(cl.sum()) * Hkv * D * 2
    for sp in map(int, a.splits.split(",")):
        ws = ops.DecodeWorkspace(B, Hq, D, ctx, "cuda", split_keys=sp)
        out = ops.attention_decode(q, kc, vc, bt, cl, scale, ws=ws, max_ctx=ctx)
        err = (out[:4].float().cpu() - want).abs().max().item()
        for _ in range(3):
            ops.attention_decode(q, kc, vc, bt, cl, scale, ws=ws, max_ctx=ctx)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            ops.attention_decode(q, kc, vc, bt, cl, scale, ws=ws, max_ctx=ctx)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1000 / 20
        print(json.dumps({"variant": os.environ.get("GAI_DECODE_VARIANT", "1"), "B": B, "ctx": ctx, "split": sp,
                          "us": round(us, 1), "TBps": round(by / us / 1e6, 3), "max_err": round(err, 4)}), flush=True)


if __name__ == "__main__":
    main()
