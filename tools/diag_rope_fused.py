"""Diagnostic: fused QKV split-K + RoPE vs unfused, and run-to-run determinism of each path."""
import math
import torch
from generativeaiexamples_amd import ops

torch.manual_seed(0)
Hq, Hkv, D, K = 32, 8, 128, 4096
N = (Hq + 2 * Hkv) * D
for M in (17, 64):
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") / math.sqrt(K)).bfloat16()
    cs = ops.rope_cos_sin(4096, D, 500000.0, device="cuda")
    pos = torch.randint(0, 4000, (M,), device="cuda", dtype=torch.int32)
    slots = torch.randperm(64 * 16, device="cuda")[:M].to(torch.int32)
    res = {}
    for name in ("fused", "fused2", "unfused", "unfused2"):
        q = torch.zeros(M, Hq, D, device="cuda", dtype=torch.bfloat16)
        kc = torch.zeros(64, Hkv, 16, D, device="cuda", dtype=torch.bfloat16)
        vc = torch.zeros(64, Hkv, D, 16, device="cuda", dtype=torch.bfloat16)
        if name.startswith("fused"):
            ops.linear_rope_kv(x, w, None, pos, cs, slots, q, kc, vc, Hq, Hkv, D)
        else:
            qkv = ops.linear(x, w)
            ops.rope_kv_write(qkv, pos, cs, slots, q, kc, vc, Hq, Hkv, D, True, 1.0, 1.0)
        res[name] = q
    ws = ops.native().gemm_splitk_ws_floats(M, N, K)
    for a, b in (("fused", "fused2"), ("unfused", "unfused2"), ("fused", "unfused")):
        d = (res[a].float() - res[b].float()).abs()
        nz = (d > 0).nonzero()
        print(M, a, b, "ws_floats", ws, "maxdiff", d.max().item(), "ndiff", int((d > 0).sum()),
              "rows", sorted(set(nz[:, 0].tolist()))[:10], "heads", sorted(set(nz[:, 1].tolist()))[:10], flush=True)
