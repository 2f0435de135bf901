"""Micro-benchmarks of the gfx950 kernels vs the PyTorch/hipBLASLt baseline on the same data.

Interleaved rounds in one process (cdna_hip_programming §5.4 rule 24), random operands
(rule 25). Prints one JSON line per case; use --out to also write them to a file.
"""
from __future__ import annotations

import argparse
import sys
import os
import json
import math
import time

import torch

from generativeaiexamples_amd import ops
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from blas_ab import blas_linear  # noqa: E402


def timeit(fn, iters=20, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    ts.sort()
    return ts[len(ts) // 2]


def bench_gemm(rows, shapes):
    for M, N, K, tag in shapes:
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = (torch.randn(N, K, device="cuda") / math.sqrt(K)).to(torch.bfloat16)
        t_ours = timeit(lambda: ops.linear(x, w))
        t_blas = timeit(lambda: torch.matmul(x, w.t()))
        fl = 2 * M * N * K
        by = 2 * (M * K + N * K + M * N)
        rows.append(dict(op="gemm", tag=tag, M=M, N=N, K=K, ours_ms=t_ours, hipblaslt_ms=t_blas,
                         ours_tflops=fl / t_ours / 1e9, hipblaslt_tflops=fl / t_blas / 1e9,
                         ours_gbs=by / t_ours / 1e6, speedup=t_blas / t_ours))


def bench_decode_gemm(rows, shapes):
    """Decode GEMMs: split-K weight-streaming kernel vs the skinny kernel vs hipBLASLt (weight bytes / time)."""
    nat = ops.native()
    for M, N, K, tag in shapes:
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = (torch.randn(N, K, device="cuda") / math.sqrt(K)).to(torch.bfloat16)
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        ws = torch.empty(nat.gemm_splitk_ws_floats(M, N, K), device="cuda", dtype=torch.float32)
        t_sk = timeit(lambda: nat.gemm_splitk(x, w, out, None, None, 0, ws))
        t_sn = timeit(lambda: nat.gemm(x, w, out, None, None, 0, 1))
        t_bl = timeit(lambda: torch.matmul(x, w.t()))
        wb = N * K * 2
        rows.append(dict(op="decode_gemm", tag=tag, M=M, N=N, K=K, splitk_ms=t_sk, skinny_ms=t_sn, hipblaslt_ms=t_bl,
                         splitk_tbs=wb / t_sk / 1e9, skinny_tbs=wb / t_sn / 1e9, hipblaslt_tbs=wb / t_bl / 1e9,
                         speedup_vs_blas=t_bl / t_sk))


def bench_psw(rows, shapes):
    """Decode GEMM: plain split-K kernel vs the same on fragment-shuffled weights vs hipBLASLt."""
    for M, N, K, name in shapes:
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        # a pool of weights larger than the 256 MB Infinity Cache, cycled, so every call streams from HBM
        ncopy = max(2, -(-(640 << 20) // (N * K * 2)))
        ws_ = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(ncopy)]
        sh_ = [ops.shuffle_fragments(w) for w in ws_]
        w = ws_[0]
        nat = ops.native()
        ws = torch.empty(nat.gemm_splitk_ws_floats(M, N, K), dtype=torch.float32, device="cuda")
        y0 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        y1 = torch.empty_like(y0)
        it = [0]

        def nxt(pool):
            it[0] = (it[0] + 1) % ncopy
            return pool[it[0]]
        t0 = timeit(lambda: nat.gemm_splitk(x, nxt(ws_), y0, None, None, 0, ws, False), iters=50)
        t1 = timeit(lambda: nat.gemm_splitk(x, nxt(sh_), y1, None, None, 0, ws, True), iters=50)
        tb = timeit(lambda: torch.mm(x, nxt(ws_).t()), iters=50)
        nat.gemm_splitk(x, sh_[0], y1, None, None, 0, ws, True)
        err = (y1.float() - (x.float() @ w.float().t())).abs().max().item()
        by = N * K * 2
        rows.append(dict(op="decode_gemm_psw", name=name, M=M, N=N, K=K, plain_us=t0 * 1e3, psw_us=t1 * 1e3,
                         blas_us=tb * 1e3, psw_tbps=by / t1 / 1e9, plain_tbps=by / t0 / 1e9, max_err=err))
        del ws_, sh_


def bench_dec_hbm(rows, shapes, rounds=5):
    """Decode GEMMs as the engine runs them: weights streamed from HBM (a pool of copies larger than the
    256 MB Infinity Cache, cycled), the fused epilogue included. Arms, interleaved per round: native
    split-K on the natural [N, K] layout, native on fragment-shuffled weights, hipBLASLt + the framework's
    epilogue kernel. (M, N, K, act, out_dtype, name)."""
    nat = ops.native()
    for M, N, K, act, odt, name in shapes:
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        ncopy = max(2, -(-(640 << 20) // (N * K * 2)))
        ws_ = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(ncopy)]
        sh_ = [ops.shuffle_fragments(w) for w in ws_] if N % 16 == 0 else None
        ncol = N // 2 if act == "swiglu" else N
        out = torch.empty(M, ncol, device="cuda", dtype=odt)
        wsp = torch.empty(max(1, nat.gemm_splitk_ws_floats(M, N, K)), dtype=torch.float32, device="cuda")
        epi = ops.EPI[act]
        it = [0]

        def nxt(pool):
            it[0] = (it[0] + 1) % ncopy
            return pool[it[0]]
        arms = {"native": lambda: nat.gemm_splitk(x, nxt(ws_), out, None, None, epi, wsp, False),
                "blas": lambda: blas_linear(x, nxt(ws_), None, act, odt)}
        if sh_ is not None:
            arms["native_psw"] = lambda: nat.gemm_splitk(x, nxt(sh_), out, None, None, epi, wsp, True)
        ts = {k: [] for k in arms}
        for _ in range(rounds):
            for k, f in arms.items():
                ts[k].append(timeit(f, iters=30) * 1e3)
        nat.gemm_splitk(x, ws_[0], out, None, None, epi, wsp, False)
        ref_ = blas_linear(x, ws_[0], None, act, odt)
        err = (out.float() - ref_.float()).abs().max().item()
        by = N * K * 2
        r = dict(op="dec_hbm", name=name, M=M, N=N, K=K, act=act, max_err_vs_blas=err)
        for k, v in ts.items():
            v.sort()
            r[f"{k}_us"] = v[len(v) // 2]
            r[f"{k}_tbs"] = by / (v[len(v) // 2] * 1e3)
        r["native_vs_blas"] = r["blas_us"] / r["native_us"]
        rows.append(r)
        print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
        del ws_, sh_


def bench_fp8(rows, shapes):
    """fp8 GEMM (block-scaled MFMA) alone and with the fused per-token quantiser, vs bf16 hipBLASLt and
    (when this torch build has it) hipBLASLt fp8 via torch._scaled_mm."""
    for M, N, K, tag in shapes:
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = (torch.randn(N, K, device="cuda") / math.sqrt(K)).to(torch.bfloat16)
        W = ops.Fp8Weight.quantize(w)
        xq, sx = ops.quant_fp8(x)
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        nat = ops.native()
        t_gemm = timeit(lambda: nat.gemm_fp8(xq, W.q, sx, W.scale, out, None, None, 0, 0))
        t_lin = timeit(lambda: ops.linear_fp8(x, W))
        t_bf16 = timeit(lambda: torch.matmul(x, w.t()))
        t_sm = None
        try:
            one = torch.ones((), device="cuda")
            t_sm = timeit(lambda: torch._scaled_mm(xq, W.q.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16))
        except Exception:
            pass
        fl = 2 * M * N * K
        rows.append(dict(op="gemm_fp8", tag=tag, M=M, N=N, K=K, gemm_ms=t_gemm, linear_ms=t_lin, bf16_blas_ms=t_bf16,
                         scaled_mm_ms=t_sm, gemm_tflops=fl / t_gemm / 1e9, linear_tflops=fl / t_lin / 1e9,
                         bf16_blas_tflops=fl / t_bf16 / 1e9,
                         scaled_mm_tflops=(fl / t_sm / 1e9) if t_sm else None))


def bench_prefill(rows, B, S, Hq, Hkv, D):
    nb = B * ((S + 15) // 16)
    kc = torch.randn(nb, Hkv, 16, D, device="cuda", dtype=torch.bfloat16)
    vc = torch.randn(nb, Hkv, D, 16, device="cuda", dtype=torch.bfloat16)
    bt = torch.arange(nb, device="cuda", dtype=torch.int32).reshape(B, -1)
    q = torch.randn(B * S, Hq, D, device="cuda", dtype=torch.bfloat16)
    cu = torch.arange(0, B * S + 1, S, device="cuda", dtype=torch.int32)
    ctx = torch.full((B,), S, device="cuda", dtype=torch.int32)
    tiles = ops.build_prefill_tiles([S] * B, Hq, Hkv, "cuda", head_dim=D)
    t = timeit(lambda: ops.attention_prefill(q, kc, vc, bt, cu, ctx, 1 / math.sqrt(D), True, tiles=tiles))
    qs = q.view(B, S, Hq, D).transpose(1, 2)
    ks = torch.randn(B, Hkv, S, D, device="cuda", dtype=torch.bfloat16).repeat_interleave(Hq // Hkv, 1)
    vs = torch.randn(B, Hkv, S, D, device="cuda", dtype=torch.bfloat16).repeat_interleave(Hq // Hkv, 1)
    t_sdpa = timeit(lambda: torch.nn.functional.scaled_dot_product_attention(qs, ks, vs, is_causal=True))
    fl = 4 * B * Hq * S * S * D / 2
    rows.append(dict(op="attn_prefill", B=B, S=S, Hq=Hq, Hkv=Hkv, D=D, ours_ms=t, sdpa_ms=t_sdpa,
                     ours_tflops=fl / t / 1e9, sdpa_tflops=fl / t_sdpa / 1e9))


def bench_decode(rows, B, ctx, Hq, Hkv, D, split=None):
    nbps = (ctx + 15) // 16
    nb = B * nbps
    kc = torch.randn(nb, Hkv, 16, D, device="cuda", dtype=torch.bfloat16)
    vc = torch.randn(nb, Hkv, D, 16, device="cuda", dtype=torch.bfloat16)
    bt = torch.randperm(nb, device="cuda").int().reshape(B, nbps)
    q = torch.randn(B, Hq, D, device="cuda", dtype=torch.bfloat16)
    cl = torch.full((B,), ctx, device="cuda", dtype=torch.int32)
    ws = ops.DecodeWorkspace(B, Hq, D, ctx, "cuda", split_keys=split)
    t = timeit(lambda: ops.attention_decode(q, kc, vc, bt, cl, 1 / math.sqrt(D), ws=ws))
    by = 2 * B * ctx * Hkv * D * 2
    rows.append(dict(op="attn_decode", B=B, ctx=ctx, Hq=Hq, Hkv=Hkv, D=D, split=ws.split_for(B, Hkv, ctx), ours_ms=t,
                     ours_gbs=by / t / 1e6))


def bench_misc(rows):
    x = torch.randn(8192, 4096, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(4096, device="cuda", dtype=torch.bfloat16)
    r = torch.randn_like(x)
    t = timeit(lambda: ops.rms_norm(x, w, 1e-5, r))
    rows.append(dict(op="rmsnorm_residual", T=8192, D=4096, ours_ms=t, ours_gbs=4 * x.numel() * 2 / t / 1e6))
    logits = torch.randn(64, 128256, device="cuda")
    temp = torch.full((64,), 0.2, device="cuda")
    tp = torch.full((64,), 0.7, device="cuda")
    tk = torch.zeros(64, dtype=torch.int32, device="cuda")
    sd = torch.arange(64, device="cuda", dtype=torch.int64)
    t = timeit(lambda: ops.sample(logits, temp, tp, tk, sd, 0))
    rows.append(dict(op="sample_top_p", B=64, V=128256, ours_ms=t))
    X = torch.randn(1_000_000, 1024, device="cuda", dtype=torch.bfloat16)
    bias = torch.zeros(1_000_000, device="cuda")
    for nq in (1, 16, 64):
        Q = torch.randn(nq, 1024, device="cuda", dtype=torch.bfloat16)
        t = timeit(lambda: ops.sim_topk(Q, X, bias, 1_000_000, 4), iters=10)
        t_ref = timeit(lambda: torch.topk(Q @ X.t(), 4, dim=-1), iters=10)
        rows.append(dict(op="sim_topk", nq=nq, N=1_000_000, D=1024, k=4, ours_ms=t, torch_ms=t_ref,
                         ours_gbs=X.numel() * 2 / t / 1e6))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--only", default="gemm,prefill,decode,misc")
    a = ap.parse_args()
    rows = []
    only = set(a.only.split(","))
    if "gemm" in only:
        shapes = [
            (4096, 6144, 4096, "llama8b qkv prefill"), (4096, 28672, 4096, "llama8b gate_up prefill"),
            (4096, 4096, 14336, "llama8b down prefill"), (8192, 8192, 8192, "square 8k"),
            (64, 6144, 4096, "qkv decode b64"), (64, 28672, 4096, "gate_up decode b64"),
            (64, 4096, 14336, "down decode b64"), (64, 128256, 4096, "lm_head decode b64"),
            (1, 6144, 4096, "qkv decode b1"), (128, 4096, 4096, "o decode b128"),
            (16384, 1024, 1024, "e5 qkv-ish"), (16384, 4096, 1024, "e5 ffn up"),
        ]
        bench_gemm(rows, shapes)
    if "decode_gemm" in only:
        sh = []
        for M in (1, 16, 32, 64):
            sh += [(M, 6144, 4096, f"qkv b{M}"), (M, 4096, 4096, f"o b{M}"), (M, 28672, 4096, f"gate_up b{M}"),
                   (M, 4096, 14336, f"down b{M}")]
        sh += [(64, 128256, 4096, "lm_head b64")]
        bench_decode_gemm(rows, sh)
    if "psw" in only:
        sh = []
        for M in (1, 16, 64):
            sh += [(M, 6144, 4096, f"qkv b{M}"), (M, 4096, 4096, f"o b{M}"), (M, 28672, 4096, f"gate_up b{M}"),
                   (M, 4096, 14336, f"down b{M}")]
        bench_psw(rows, sh)
    if "dec_hbm" in only:
        bf, f32 = torch.bfloat16, torch.float32
        sh = []
        for M in (64, 1):
            sh += [(M, 6144, 4096, None, bf, f"qkv b{M}"), (M, 4096, 4096, None, bf, f"o b{M}"),
                   (M, 28672, 4096, "swiglu", bf, f"gate_up+swiglu b{M}"), (M, 4096, 14336, None, bf, f"down b{M}"),
                   (M, 128256, 4096, None, f32, f"lm_head b{M}")]
        bench_dec_hbm(rows, sh)
    if "dec_hbm_tp8" in only:  # one rank of Llama-3-70B at TP = 8, batch 64
        bf, f32 = torch.bfloat16, torch.float32
        bench_dec_hbm(rows, [(64, 1280, 8192, None, bf, "70b/tp8 qkv b64"), (64, 8192, 1024, None, bf, "70b/tp8 o b64"),
                             (64, 7168, 8192, "swiglu", bf, "70b/tp8 gate_up+swiglu b64"),
                             (64, 8192, 3584, None, bf, "70b/tp8 down b64"),
                             (64, 16032, 8192, None, f32, "70b/tp8 lm_head b64")], rounds=3)
    if "fp8" in only:
        bench_fp8(rows, [(4096, 6144, 4096, "qkv prefill"), (4096, 28672, 4096, "gate_up prefill"),
                         (4096, 4096, 14336, "down prefill"), (8192, 8192, 8192, "square 8k"),
                         (1601 * 8, 4096, 1024, "clip-L mlp up b8"), (64, 28672, 4096, "gate_up decode b64")])
    if "prefill" in only:
        bench_prefill(rows, 4, 2048, 32, 8, 128)
        bench_prefill(rows, 7, 2406, 32, 8, 128)  # one headline 16K prefill chunk: 7 RAG prompts of 2406 tokens
        bench_prefill(rows, 64, 512, 16, 16, 64)
        bench_prefill(rows, 4, 2048, 16, 16, 256)  # Gemma-7B attention shape
    if "decode_sweep" in only:
        for sp in (128, 256, 512, 1024, 2048):
            bench_decode(rows, 64, 2600, 32, 8, 128, sp)
    if "decode" in only:
        bench_decode(rows, 64, 2304, 32, 8, 128)
        bench_decode(rows, 1, 2304, 32, 8, 128)
        bench_decode(rows, 128, 4096, 32, 8, 128)
    if "misc" in only:
        bench_misc(rows)
    f = open(a.out, "w") if a.out else None
    for r in rows:
        line = json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()})
        print(line, flush=True)
        if f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
