"""Small-batch decode GEMV (csrc/kernels/gemv.hip) against plain PyTorch fp32 references: every epilogue (plain,
residual in place, SwiGLU interleave, fp32 logits) with and without the staged RMSNorm, the QKV + RoPE + paged
K / V^T store form, and an 8B-width engine decode at batch 1..4 (graph-captured, the GEMV path) whose greedy
tokens must be the dense fp32 forward's argmax up to bf16 near-ties."""
import math

import pytest
import torch

from generativeaiexamples_amd import ops
from generativeaiexamples_amd.ops import reference as R

pytestmark = pytest.mark.gpu


def _rms_ref(x, g, eps):
    xf = x.float()
    return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * g.float()).to(torch.bfloat16).float()


@pytest.mark.parametrize("M", [1, 2, 3, 4])
@pytest.mark.parametrize("N,K,epi,normed", [(6144, 4096, "plain", True), (4096, 4096, "residual", False),
                                           (28672, 4096, "swiglu", True), (4096, 14336, "residual", False),
                                           (128256, 4096, "f32", True), (2048, 8192, "plain", False)])
def test_gemv_matches_fp32(cuda, M, N, K, epi, normed):
    torch.manual_seed(M * 7 + N + K)
    x = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    W = (torch.randn(N, K, device=cuda) / math.sqrt(K)).to(torch.bfloat16)
    g = (torch.rand(K, device=cuda) + 0.5).to(torch.bfloat16) if normed else None
    res = torch.randn(M, N, device=cuda).to(torch.bfloat16) if epi == "residual" else None
    res0 = res.clone() if res is not None else None
    y = ops.gemv(x, W, gamma=g, eps=1e-5, epi=epi, res=res)
    xf = _rms_ref(x, g, 1e-5) if normed else x.float()
    acc = xf @ W.float().t()
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
    # the oracle the CPU path uses agrees too (rounding conventions)
    if epi != "residual":
        r = R.gemv(x.cpu(), W.cpu(), g.cpu() if g is not None else None, 1e-5, epi)
        assert (r.float() - got.cpu()).abs().max() <= 3e-2 + 1e-2 * r.float().abs().max()


@pytest.mark.parametrize("M", [1, 4])
def test_gemv_rope_kv_matches_reference(cuda, M):
    torch.manual_seed(11 + M)
    Hq, Hkv, D, K = 32, 8, 128, 4096
    N = (Hq + 2 * Hkv) * D
    res = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    g = (torch.rand(K, device=cuda) + 0.5).to(torch.bfloat16)
    W = (torch.randn(N, K, device=cuda) / math.sqrt(K)).to(torch.bfloat16)
    cs = ops.rope_cos_sin(8192, D, 500000.0, device=cuda)
    pos = torch.tensor([5, 700, 2600, 4095][:M], dtype=torch.int32, device=cuda)
    slots = torch.tensor([3 * 16 + 5, 7 * 16 + 0, -1, 9 * 16 + 15][:M], dtype=torch.int32, device=cuda)
    kc = torch.zeros(12, Hkv, 16, D, device=cuda, dtype=torch.bfloat16)
    vc = torch.zeros(12, Hkv, D, 16, device=cuda, dtype=torch.bfloat16)
    q = torch.zeros(M, Hq, D, device=cuda, dtype=torch.bfloat16)
    ops.gemv_rope_kv(res, W, g, 1e-5, pos, cs, slots, q, kc, vc, Hq, Hkv)
    qkv = (_rms_ref(res, g, 1e-5) @ W.float().t()).to(torch.bfloat16).cpu()
    q2 = torch.zeros(M, Hq, D, dtype=torch.bfloat16)
    kc2, vc2 = torch.zeros_like(kc.cpu()), torch.zeros_like(vc.cpu())
    R.rope_kv_write(qkv, pos.cpu(), cs.cpu(), slots.cpu(), q2, kc2, vc2, Hq, Hkv, D, True)
    for a, b, what in ((q.cpu(), q2, "q"), (kc.cpu(), kc2, "k cache"), (vc.cpu(), vc2, "v cache")):
        err = (a.float() - b.float()).abs().max().item()
        assert err <= 3e-2 * max(1.0, b.float().abs().max().item()), (what, err)


def test_batch1_to_4_decode_on_gemv_path_matches_fp32(cuda, monkeypatch):
    """8B widths, 2 layers: prompts prefilled, then graph-captured decode at batch 1..4 (the GEMV path: five
    launches per layer); greedy tokens vs the dense fp32 forward."""
    from generativeaiexamples_amd.engine import EngineConfig, LLMEngine, SamplingParams
    from generativeaiexamples_amd.engine.tokenizer import llama3_byte_tokenizer
    from generativeaiexamples_amd.models import LlamaConfig, LlamaModel
    from tests.test_headline_numerics_gpu import _fp32_logits

    cfg = LlamaConfig.llama3_8b(num_layers=2)
    m = LlamaModel(cfg, device=cuda).random_init(9)
    tok = llama3_byte_tokenizer(cfg.vocab_size)
    g = torch.Generator().manual_seed(4)
    calls = {"n": 0}
    orig = m._forward_gemv

    def spy(*a, **k):
        calls["n"] += 1
        return orig(*a, **k)

    monkeypatch.setattr(m, "_forward_gemv", spy)
    for bs in (1, 3, 4):
        prompts = [torch.randint(1000, 120000, (100 + 37 * i,), generator=g).tolist() for i in range(bs)]
        eng = LLMEngine(m, tok, EngineConfig(max_num_seqs=4, max_batched_tokens=2048, max_model_len=512,
                                             use_graphs=True, decode_steps=4, prefix_cache=False,
                                             graph_batch_sizes=(1, 2, 4), kv_memory_fraction=0.05))
        eng.capture_graphs(max_bs=4)
        reqs = eng.generate(prompts, SamplingParams(temperature=0.0, max_tokens=8, ignore_eos=True))
        for p, r in zip(prompts, reqs):
            out = r.output_ids
            assert len(out) == 8
            seq = torch.tensor(p + out, device=cuda)
            rows = torch.arange(len(p) - 1, len(p) + 7, device=cuda)
            lg = _fp32_logits(m, seq, rows)
            top = lg.max(-1).values
            scale = lg.abs().max(-1).values.clamp_min(1.0)
            mine = lg[torch.arange(8, device=cuda), torch.tensor(out, device=cuda)]
            assert bool((mine >= top - 0.02 * scale).all()), (bs, (mine - top).tolist())
    assert calls["n"] > 0, "the batch <= 4 decode never took the GEMV path"
