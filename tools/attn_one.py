"""One prefill-attention shape for counter passes (tools/pmc_gemm.sh with PMC_DRIVER=attn_one.py): the headline 16K
chunk (7 prompts x 2406 tokens, causal, 32 q / 8 kv heads, head_dim 128), 10 launches.

usage: python tools/attn_one.py hl1|hl2 [ignored N K]
"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from generativeaiexamples_amd import ops  # noqa: E402


def main():
    arm = sys.argv[1]
    ops.set_prefill_heads_per_wave(2 if arm == "hl2" else 1)
    B, S, Hq, Hkv, D = 7, 2406, 32, 8, 128
    nb = B * ((S + 15) // 16)
    kc = torch.randn(nb, Hkv, 16, D, device="cuda", dtype=torch.bfloat16)
    vc = torch.randn(nb, Hkv, D, 16, device="cuda", dtype=torch.bfloat16)
    bt = torch.arange(nb, device="cuda", dtype=torch.int32).reshape(B, -1)
    q = torch.randn(B * S, Hq, D, device="cuda", dtype=torch.bfloat16)
    cu = torch.arange(0, B * S + 1, S, device="cuda", dtype=torch.int32)
    ctx = torch.full((B,), S, device="cuda", dtype=torch.int32)
    tiles = ops.build_prefill_tiles([S] * B, Hq, Hkv, "cuda", head_dim=D)
    for _ in range(10):
        ops.attention_prefill(q, kc, vc, bt, cu, ctx, 1 / math.sqrt(D), True, tiles=tiles)
    torch.cuda.synchronize()
    print("ok", arm)


if __name__ == "__main__":
    main()
