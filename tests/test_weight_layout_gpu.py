"""The one weight layout on the GPU: every kernel that reads a fragment-ordered weight (ops.to_fragment_layout_).

* the prefill / mid-M GEMMs (skinny, 128x128 tiled, the 256x256 part-ring and double-slot walks at 256 / 192 rows,
  stream-K, the split walk, auto) are BITWISE equal on the fragment-ordered and the row-major copy of one weight -
  same MFMAs in the same order, only the B staging addresses differ - for the plain, bias, residual and SwiGLU
  epilogues, partial N tiles included;
* the prefill QKV GEMM with the RoPE / paged-KV epilogue likewise (q_out and both caches);
* the batch <= 4 GEMV (gemv.hip gemv_frag_kernel: whole-column workgroups, K split over waves) against the plain
  PyTorch fp32 reference for every epilogue, normalised input and the QKV + RoPE form;
* an engine on the one layout allocates no decode copies and generates the same greedy tokens as the two-layout
  engine at batch 8 (prefill GEMMs bitwise equal, the same split-K decode kernels).
"""
import math

import pytest
import torch

from generativeaiexamples_amd import ops
from generativeaiexamples_amd.ops import reference as R

pytestmark = pytest.mark.gpu

EPI = {"none": 0, "bias": 1, "residual": 3, "swiglu": 4}


def _pair(N, K, dev, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    w = (torch.randn(N, K, device=dev, generator=g) / math.sqrt(K)).to(torch.bfloat16)
    f = w.clone()
    assert ops.to_fragment_layout_(f) and ops.is_frag(f)
    return w, f


@pytest.mark.parametrize("force,M,N,K", [
    (1, 100, 1024, 4096),     # skinny
    (2, 300, 1040, 4096),     # 128x128 tiled, partial n tile
    (10, 2406, 4096, 1024),   # part ring
    (10, 700, 1040, 2048),    # part ring, partial n / m tiles
    (9, 2406, 6144, 4096),    # double-slot, 256 rows
    (13, 2406, 4096, 1024),   # double-slot, 192 rows
    (11, 512, 4096, 14336),   # stream-K
    (12, 2406, 4096, 14336),  # split walk
    (0, 1100, 2048, 4096),    # auto
])
@pytest.mark.parametrize("epi", ["none", "bias", "residual", "swiglu"])
def test_gemm_fragment_weight_bitwise(cuda, force, M, N, K, epi):
    if epi == "swiglu" and N % 32:
        pytest.skip("SwiGLU interleave needs N % 32 == 0")
    w, f = _pair(N, K, cuda, M + N + K)
    x = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    bias = torch.randn(N, device=cuda).to(torch.bfloat16) if epi == "bias" else None
    res = torch.randn(M, N, device=cuda).to(torch.bfloat16) if epi == "residual" else None
    cols = N // 2 if epi == "swiglu" else N
    a = torch.empty(M, cols, device=cuda, dtype=torch.bfloat16)
    b = torch.empty_like(a)
    nat = ops.native()
    nat.gemm(x, w, a, bias, res, EPI[epi], force, False)
    nat.gemm(x, f, b, bias, res, EPI[epi], force, True)
    torch.cuda.synchronize()
    assert torch.equal(a, b), f"force {force} {epi}: max diff {(a.float() - b.float()).abs().max():.3g}"


def test_gemm_fragment_weight_fp32_out(cuda):
    w, f = _pair(2048, 4096, cuda, 5)
    x = torch.randn(1500, 4096, device=cuda).to(torch.bfloat16)
    a = torch.empty(1500, 2048, device=cuda, dtype=torch.float32)
    b = torch.empty_like(a)
    ops.native().gemm(x, w, a, None, None, 0, 0, False)
    ops.native().gemm(x, f, b, None, None, 0, 0, True)
    assert torch.equal(a, b)


def test_linear_routes_fragment_weights(cuda):
    """ops.linear on a fragment-ordered weight: prefill (M > 64) equals the row-major weight bitwise; decode
    (M <= 64) takes the split-K kernel on the weight itself."""
    w, f = _pair(4096, 4096, cuda, 7)
    for M in (2406, 200, 17):
        x = torch.randn(M, 4096, device=cuda).to(torch.bfloat16)
        ya, yb = ops.linear(x, w), ops.linear(x, f)
        if M > 64:
            assert torch.equal(ya, yb), M
        else:
            want = x.float() @ w.float().t()
            assert (yb.float() - want).abs().max() <= 2e-2 + 1e-2 * want.abs().max(), M


def test_prefill_qkv_rope_kv_fragment_weight_bitwise(cuda):
    Hq, Hkv, D, K, M = 32, 8, 128, 4096, 2406
    w, f = _pair((Hq + 2 * Hkv) * D, K, cuda, 3)
    x = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    cs = ops.rope_cos_sin(8192, D, 500000.0, device=cuda)
    pos = torch.arange(M, dtype=torch.int32, device=cuda)
    slots = torch.arange(M, dtype=torch.int32, device=cuda)
    nb = (M + 15) // 16
    outs = []
    for wt in (w, f):
        q = torch.zeros(M, Hq, D, device=cuda, dtype=torch.bfloat16)
        kc = torch.zeros(nb, Hkv, 16, D, device=cuda, dtype=torch.bfloat16)
        vc = torch.zeros(nb, Hkv, D, 16, device=cuda, dtype=torch.bfloat16)
        ops.linear_rope_kv(x, wt, None, pos, cs, slots, q, kc, vc, Hq, Hkv, D)
        outs.append((q, kc, vc))
    torch.cuda.synchronize()
    for a, b, what in zip(outs[0], outs[1], ("q", "k cache", "v cache")):
        assert torch.equal(a, b), what


def _rms_ref(x, g, eps):
    xf = x.float()
    return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * g.float()).to(torch.bfloat16).float()


@pytest.mark.parametrize("M", [1, 2, 3, 4])
@pytest.mark.parametrize("N,K,epi,normed", [(6144, 4096, "plain", True), (4096, 4096, "residual", False),
                                           (28672, 4096, "swiglu", True), (4096, 14336, "residual", False),
                                           (128256, 4096, "f32", True), (2048, 8192, "plain", False)])
def test_gemv_fragment_weight_matches_fp32(cuda, M, N, K, epi, normed):
    torch.manual_seed(M * 5 + N + K)
    x = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    w, f = _pair(N, K, cuda, M + N)
    g = (torch.rand(K, device=cuda) + 0.5).to(torch.bfloat16) if normed else None
    res = torch.randn(M, N, device=cuda).to(torch.bfloat16) if epi == "residual" else None
    res0 = res.clone() if res is not None else None
    y = ops.gemv(x, f, gamma=g, eps=1e-5, epi=epi, res=res)
    xf = _rms_ref(x, g, 1e-5) if normed else x.float()
    acc = xf @ w.float().t()
    if epi == "f32":
        want, got = acc, y
    elif epi == "residual":
        want, got = acc.to(torch.bfloat16).float() + res0.float(), res.float()
    elif epi == "swiglu":
        gu = acc.view(M, -1, 2, 16)
        want, got = (torch.nn.functional.silu(gu[:, :, 0]) * gu[:, :, 1]).reshape(M, -1), y.float()
    else:
        want, got = acc, y.float()
    err = (got - want).abs()
    tol = 2e-2 + 1e-2 * want.abs()
    assert (err <= tol).all(), f"{epi} M={M} {N}x{K}: max err {err.max():.4g}"


@pytest.mark.parametrize("M", [1, 4])
def test_gemv_rope_kv_fragment_weight(cuda, M):
    torch.manual_seed(21 + M)
    Hq, Hkv, D, K = 32, 8, 128, 4096
    res = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    g = (torch.rand(K, device=cuda) + 0.5).to(torch.bfloat16)
    w, f = _pair((Hq + 2 * Hkv) * D, K, cuda, 9)
    cs = ops.rope_cos_sin(8192, D, 500000.0, device=cuda)
    pos = torch.tensor([5, 700, 2600, 4095][:M], dtype=torch.int32, device=cuda)
    slots = torch.tensor([3 * 16 + 5, 7 * 16 + 0, -1, 9 * 16 + 15][:M], dtype=torch.int32, device=cuda)
    kc = torch.zeros(12, Hkv, 16, D, device=cuda, dtype=torch.bfloat16)
    vc = torch.zeros(12, Hkv, D, 16, device=cuda, dtype=torch.bfloat16)
    q = torch.zeros(M, Hq, D, device=cuda, dtype=torch.bfloat16)
    ops.gemv_rope_kv(res, f, g, 1e-5, pos, cs, slots, q, kc, vc, Hq, Hkv)
    qkv = (_rms_ref(res, g, 1e-5) @ w.float().t()).to(torch.bfloat16).cpu()
    q2 = torch.zeros(M, Hq, D, dtype=torch.bfloat16)
    kc2, vc2 = torch.zeros_like(kc.cpu()), torch.zeros_like(vc.cpu())
    R.rope_kv_write(qkv, pos.cpu(), cs.cpu(), slots.cpu(), q2, kc2, vc2, Hq, Hkv, D, True)
    for a, b, what in ((q.cpu(), q2, "q"), (kc.cpu(), kc2, "k cache"), (vc.cpu(), vc2, "v cache")):
        err = (a.float() - b.float()).abs().max().item()
        assert err <= 3e-2 * max(1.0, b.float().abs().max().item()), (what, err)


def test_engine_one_layout_same_tokens_no_copies(cuda, monkeypatch):
    """8B widths, 2 layers: the fragment-layout engine keeps no decode copies (the two-layout engine adds one per
    projection) and generates the two-layout engine's greedy tokens at batch 8."""
    from generativeaiexamples_amd.engine import EngineConfig, LLMEngine, SamplingParams
    from generativeaiexamples_amd.engine.tokenizer import llama3_byte_tokenizer
    from generativeaiexamples_amd.models import LlamaConfig, LlamaModel

    cfg = LlamaConfig.llama3_8b(num_layers=2)
    tok = llama3_byte_tokenizer(cfg.vocab_size)
    g = torch.Generator().manual_seed(2)
    prompts = [torch.randint(1000, 120000, (80 + 29 * i,), generator=g).tolist() for i in range(8)]
    outs, extra = {}, {}
    for layout in ("dual", "fragment"):
        monkeypatch.setenv("GAI_WEIGHT_LAYOUT", layout)
        m = LlamaModel(cfg, device=cuda).random_init(5)
        # the bytes the preshuffle reports it added (allocator deltas are not evidence: a GC pass freeing an
        # earlier test's tensors in between would make them negative)
        extra[layout] = m.preshuffle_decode_weights(in_place=layout == "fragment")
        eng = LLMEngine(m, tok, EngineConfig(max_num_seqs=8, max_batched_tokens=4096, max_model_len=512,
                                             use_graphs=True, decode_steps=4, prefix_cache=False,
                                             graph_batch_sizes=(8,), kv_memory_fraction=0.05))
        assert all(ops.is_frag(m.w[f"l{i}.{k}"]) == (layout == "fragment")
                   for i in range(2) for k in ("qkv", "o", "gate_up", "down"))
        copies = [k for k, v in m.w.items() if getattr(v, "_gai_psw", None) is not None]
        assert (not copies) if layout == "fragment" else len(copies) == 2 * 4 + 1, copies
        reqs = eng.generate(prompts, SamplingParams(temperature=0.0, max_tokens=6, ignore_eos=True))
        outs[layout] = [r.output_ids for r in reqs]
        eng.close()
        del eng, m, reqs
    proj = 2 * (6144 * 4096 + 4096 * 4096 + 28672 * 4096 + 4096 * 14336) * 2 + 128256 * 4096 * 2
    assert extra["fragment"] == 0
    assert extra["dual"] == proj
    assert outs["fragment"] == outs["dual"]


def test_engine_memory_released_without_gc(cuda):
    """`del engine, model` returns the device memory at once - no reference cycle keeps the weights, the KV cache or
    the captured graphs alive until a GC pass (a second engine sizes its KV cache from free memory)."""
    import gc
    import weakref

    from generativeaiexamples_amd.engine import EngineConfig, LLMEngine, SamplingParams
    from generativeaiexamples_amd.engine.tokenizer import llama3_byte_tokenizer
    from generativeaiexamples_amd.models import LlamaConfig, LlamaModel

    cfg = LlamaConfig.llama3_8b(num_layers=2)
    tok = llama3_byte_tokenizer(cfg.vocab_size)
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    base = torch.cuda.memory_allocated(cuda)
    gc.disable()
    try:
        for close in (False, True):
            m = LlamaModel(cfg, device=cuda).random_init(1)
            eng = LLMEngine(m, tok, EngineConfig(max_num_seqs=8, max_batched_tokens=2048, max_model_len=512,
                                                 use_graphs=True, decode_steps=4, prefix_cache=False,
                                                 graph_batch_sizes=(4, 8), kv_memory_fraction=0.02))
            eng.capture_graphs()
            eng.generate([[5, 6, 7, 8] * 20] * 3, SamplingParams(temperature=0.0, max_tokens=9, ignore_eos=True))
            assert torch.cuda.memory_allocated(cuda) > base + (1 << 30)
            wm, we = weakref.ref(m), weakref.ref(eng)
            if close:
                eng.close()
            del eng, m
            assert wm() is None and we() is None, "model / engine kept alive by a reference cycle"
            torch.cuda.synchronize()
            # small per-device caches of the op layer (tail counters, workspaces) may stay
            assert torch.cuda.memory_allocated(cuda) - base < (64 << 20), torch.cuda.memory_allocated(cuda) - base
    finally:
        gc.enable()


def test_gemv_fragment_k_split_opt_in(cuda):
    """GAI_GEMV_FRAG_KS = 2 (read once per process, so in a child): the cross-workgroup K split of the fragment GEMV
    (write-through partials + ticket, the last workgroup sums in K order) matches the unsplit kernel's reference."""
    import os
    import subprocess
    import sys

    code = (
        "import torch, math\n"
        "from tests.test_weight_layout_gpu import test_gemv_fragment_weight_matches_fp32 as t, "
        "test_gemv_rope_kv_fragment_weight as r\n"
        "d = torch.device('cuda:0')\n"
        "for M in (1, 4):\n"
        "    t(d, M, 2048, 8192, 'plain', False)\n"
        "    t(d, M, 6144, 4096, 'plain', True)\n"
        "    t(d, M, 28672, 4096, 'swiglu', True)\n"
        "    r(d, M)\n"
        "print('split ok')\n")
    env = dict(os.environ, GAI_GEMV_FRAG_KS="2")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=110,
                         cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert out.returncode == 0 and "split ok" in out.stdout, out.stderr[-2000:]


def test_checkpoint_roundtrip_on_fragment_layout(cuda):
    """export_hf_state hands out row-major weights, and load_hf_state into a model an engine already rewrote stores
    them fragment-ordered again: reloading the export leaves every weight bitwise unchanged."""
    from generativeaiexamples_amd.models import LlamaConfig, LlamaModel

    cfg = LlamaConfig.llama3_8b(num_layers=1)
    m = LlamaModel(cfg, device=cuda).random_init(3)
    nat = {k: v.clone() for k, v in m.w.items()}
    m.preshuffle_decode_weights(in_place=True)
    assert ops.is_frag(m.w["l0.gate_up"]) and ops.is_frag(m.w["lm_head"])
    sd = m.export_hf_state()
    for k, v in m.w.items():
        assert torch.equal(ops.natural_weight(v), nat[k]), k
    before = {k: v.clone() for k, v in m.w.items()}
    m.load_hf_state(sd)
    for k, v in m.w.items():
        assert torch.equal(v, before[k]), k
    assert ops.is_frag(m.w["l0.qkv"])


@pytest.mark.parametrize("M", [1, 2, 4])
def test_gemv_k_parts_and_swiglu_staging(cuda, M):
    """Batch-1 rebalanced decode forms (gemv.hip): QKV as K-part fp32 slabs [ks, M, N] (the RMSNorm staged in), and
    the down projection staging bf16(silu(g) * u) from the fp32 gate_up GEMV's [gate16 | up16] interleave."""
    torch.manual_seed(40 + M)
    D, N, I = 4096, 6144, 14336
    res = torch.randn(M, D, device=cuda).to(torch.bfloat16)
    g = (torch.rand(D, device=cuda) + 0.5).to(torch.bfloat16)
    w, f = _pair(N, D, cuda, 3)
    slabs = ops.gemv(res, f, gamma=g, eps=1e-5, epi="part", ks=2)
    assert slabs.shape == (2, M, N) and slabs.dtype == torch.float32
    xf = _rms_ref(res, g, 1e-5)
    for h in range(2):
        want = xf[:, h * 2048:(h + 1) * 2048] @ w.float()[:, h * 2048:(h + 1) * 2048].t()
        err = (slabs[h] - want).abs()
        assert (err <= 1e-2 + 1e-3 * want.abs()).all(), (h, err.max().item())
    # gate_up as fp32 GEMV, then down with the SwiGLU in its staging
    wgu, fgu = _pair(2 * I, D, cuda, 4)
    wd, fd = _pair(D, I, cuda, 5)
    gu = ops.gemv(res, fgu, gamma=g, eps=1e-5, epi="f32")
    want_gu = xf @ wgu.float().t()
    assert ((gu - want_gu).abs() <= 1e-2 + 1e-3 * want_gu.abs()).all()
    r = torch.randn(M, D, device=cuda).to(torch.bfloat16)
    r0 = r.clone()
    ops.gemv(None, fd, epi="residual", res=r, swi=gu)
    q = gu.view(M, -1, 2, 16)
    act = (torch.nn.functional.silu(q[:, :, 0]) * q[:, :, 1]).reshape(M, -1).to(torch.bfloat16).float()
    want = (act @ wd.float().t()).to(torch.bfloat16).float() + r0.float()
    err = (r.float() - want).abs()
    assert (err <= 3e-2 + 1e-2 * want.abs()).all(), err.max().item()
    # the same fused pair against the swiglu-epilogue route, which it replaces at batch 1
    g2 = ops.gemv(res, fgu, gamma=g, eps=1e-5, epi="swiglu")
    r2 = r0.clone()
    ops.gemv(g2, fd, epi="residual", res=r2)
    assert (r2.float() - r.float()).abs().max().item() <= 3e-2 * max(1.0, r.float().abs().max().item())


def test_batch1_rebalanced_decode_same_as_five_launch_path(cuda, monkeypatch):
    """8B widths, 2 layers, batch 1 on the graph-captured decode: the rebalanced launches (QKV K-part slabs folded
    into the attention launch; fp32 gate_up + SwiGLU in down's staging) give the same greedy tokens as the
    gemv_rope_kv / swiglu-epilogue path, and actually ran (the fold taken every layer)."""
    from generativeaiexamples_amd.engine import EngineConfig, LLMEngine, SamplingParams
    from generativeaiexamples_amd.engine.tokenizer import llama3_byte_tokenizer
    from generativeaiexamples_amd.models import LlamaConfig, LlamaModel
    from generativeaiexamples_amd.models import llama as L

    cfg = LlamaConfig.llama3_8b(num_layers=2)
    m = LlamaModel(cfg, device=cuda).random_init(11)
    tok = llama3_byte_tokenizer(cfg.vocab_size)
    prompt = torch.randint(1000, 120000, (300,), generator=torch.Generator().manual_seed(8)).tolist()
    folds = {"n": 0}
    orig = ops.gemv_qkv_partials

    def spy(*a, **k):
        r = orig(*a, **k)
        folds["n"] += r is not None
        return r

    monkeypatch.setattr(ops, "gemv_qkv_partials", spy)
    outs = {}
    for on in (True, False):
        monkeypatch.setattr(L, "_GEMV_B1", on)
        eng = LLMEngine(m, tok, EngineConfig(max_num_seqs=2, max_batched_tokens=2048, max_model_len=512,
                                             use_graphs=True, decode_steps=4, prefix_cache=False,
                                             graph_batch_sizes=(1,), kv_memory_fraction=0.05))
        eng.capture_graphs(max_bs=1)
        outs[on] = eng.generate([prompt], SamplingParams(temperature=0.0, max_tokens=12, ignore_eos=True))[0].output_ids
        eng.close()
        del eng
    assert folds["n"] >= 2, "the QKV fold never applied"
    # fp32 sums split in two K parts round differently from the one-part sums: check the rebalanced path's tokens
    # against the dense fp32 forward (near-ties may legitimately pick the other token), and that the paths agree
    from tests.test_headline_numerics_gpu import _fp32_logits

    out = outs[True]
    seq = torch.tensor(prompt + out, device=cuda)
    lg = _fp32_logits(m, seq, torch.arange(len(prompt) - 1, len(prompt) + 11, device=cuda))
    top, scale = lg.max(-1).values, lg.abs().max(-1).values.clamp_min(1.0)
    mine = lg[torch.arange(12, device=cuda), torch.tensor(out, device=cuda)]
    assert bool((mine >= top - 0.02 * scale).all()), (mine - top).tolist()
    assert sum(a == b for a, b in zip(outs[True], outs[False])) >= 10, outs

