"""Numerics of the REAL headline path: a 2-layer model at Llama-3-8B width (d 4096, GQA
32/8, head_dim 128, FFN 14336, vocab 128256) takes 2 x 4096-token prompts + 62 short ones through ONE
16K-token prefill chunk (the persistent w4d / w4r GEMMs with the fused RoPE + paged-KV epilogue, chunked
varlen flash attention), then 16 tokens of HIP-graph multi-step decode at batch 64 (decode GEMMs, split-K
tails, paged decode attention, split-row sampler, pipelined runs). Every greedy token of the long prompts
must be the argmax of a dense fp32 GPU forward of the same weights up to bf16 near-ties, and the first token's
logit row must match it closely. Also the Llama-3-70B GEMM shapes (K 8192 / 28672, N 10240 / 57344) against
the fp32 product."""
import math

import pytest
import torch

from generativeaiexamples_amd import ops
from generativeaiexamples_amd.engine import EngineConfig, LLMEngine, SamplingParams
from generativeaiexamples_amd.models import LlamaConfig, LlamaModel

pytestmark = pytest.mark.gpu


def _fp32_logits(m: LlamaModel, ids: torch.Tensor, rows: torch.Tensor) -> torch.Tensor:
    """Dense causal fp32 forward on the GPU; logits [len(rows), vocab] at the given positions."""
    c, dev = m.cfg, ids.device
    w = {k: ops.natural_weight(v).float() for k, v in m.w.items()}
    T, hd = ids.numel(), c.head_dim
    h = w["embed"][ids.long()]
    cs = m.cos_sin[:T].float()
    cos, sin = cs[:, None, : hd // 2], cs[:, None, hd // 2:]

    def rope(t):
        a, b = t[..., : hd // 2], t[..., hd // 2:]
        return torch.cat([a * cos - b * sin, b * cos + a * sin], -1)

    def rms(x, g):
        return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + c.rms_eps) * g

    for i in range(c.num_layers):
        p = f"l{i}."
        x = rms(h, w[p + "attn_norm"])
        qkv = (x @ w[p + "qkv"].t()).view(T, m.hq + 2 * m.hkv, hd)
        q, k, v = qkv[:, : m.hq], qkv[:, m.hq: m.hq + m.hkv], qkv[:, m.hq + m.hkv:]
        q, k = rope(q), rope(k)
        rep = m.hq // m.hkv
        k, v = k.repeat_interleave(rep, 1), v.repeat_interleave(rep, 1)
        o = torch.nn.functional.scaled_dot_product_attention(q.transpose(0, 1), k.transpose(0, 1), v.transpose(0, 1),
                                                             is_causal=True, scale=m.scale)
        h = h + o.transpose(0, 1).reshape(T, -1) @ w[p + "o"].t()
        x = rms(h, w[p + "mlp_norm"])
        gu = (x @ w[p + "gate_up"].t()).view(T, -1, 2, 16)  # [gate16 | up16] interleave of the fused weight
        g, u = gu[:, :, 0].reshape(T, -1), gu[:, :, 1].reshape(T, -1)
        h = h + (torch.nn.functional.silu(g) * u) @ w[p + "down"].t()
    x = rms(h[rows], w["norm"])
    return x @ w["lm_head"].t()


def test_llama3_8b_width_prefill_and_graph_decode_match_fp32(cuda):
    torch.manual_seed(0)
    cfg = LlamaConfig.llama3_8b(num_layers=2)
    m = LlamaModel(cfg, device=cuda).random_init(7)
    from generativeaiexamples_amd.engine.tokenizer import llama3_byte_tokenizer

    tok = llama3_byte_tokenizer(cfg.vocab_size)
    g = torch.Generator().manual_seed(1)
    long = [torch.randint(1000, 120000, (4096,), generator=g).tolist() for _ in range(2)]
    short = [torch.randint(1000, 120000, (128,), generator=g).tolist() for _ in range(62)]
    eng = LLMEngine(m, tok, EngineConfig(max_num_seqs=64, max_batched_tokens=16384, prefill_chunk=16384,
                                         max_model_len=4096 + 64, use_graphs=True, decode_steps=8, prefix_cache=False,
                                         kv_memory_fraction=0.1))
    eng.capture_graphs(max_bs=64)
    sp = SamplingParams(temperature=0.0, max_tokens=16, ignore_eos=True)
    reqs = eng.generate(long + short, sp)
    assert eng.stats["prefill_tokens"] == 2 * 4096 + 62 * 128
    assert eng.stats["graph_steps"] > 0 and eng.stats["multi_step_runs"] > 0
    for p, r in zip(long, reqs[:2]):
        out = r.output_ids
        assert len(out) == 16
        seq = torch.tensor(p + out, device=cuda)
        rows = torch.arange(len(p) - 1, len(p) + 15, device=cuda)
        lg = _fp32_logits(m, seq, rows)
        top = lg.max(-1).values
        scale = lg.abs().max(-1).values.clamp_min(1.0)
        mine = lg[torch.arange(16, device=cuda), torch.tensor(out, device=cuda)]
        assert bool((mine >= top - 0.02 * scale).all()), (mine - top).tolist()
        exact = int((lg.argmax(-1).cpu() == torch.tensor(out)).sum())
        assert exact >= 14, exact


@pytest.mark.parametrize("N,K", [(10240, 8192), (57344, 8192), (8192, 28672), (8192, 8192)])
@pytest.mark.parametrize("M", [64, 16384])
def test_llama3_70b_gemm_shapes(cuda, M, N, K):
    """Llama-3-70B (TP 1) projections: QKV N 10240, gate_up N 57344 (SwiGLU), down K 28672, O; decode (M 64) and
    prefill (M 16K) kernels; 256 sampled rows vs the fp32 product."""
    torch.manual_seed(M + N + K)
    x = torch.randn(M, K, device=cuda, dtype=torch.bfloat16)
    w = (torch.randn(N, K, device=cuda) / math.sqrt(K)).to(torch.bfloat16)
    act = "swiglu" if N == 57344 else None
    y = ops.linear(x, w, act=act)
    rows = torch.randperm(M, device=cuda)[:256] if M > 256 else torch.arange(M, device=cuda)
    r = x[rows].float() @ w.float().t()
    if act:
        r = r.view(len(rows), -1, 2, 16)
        r = (torch.nn.functional.silu(r[:, :, 0]) * r[:, :, 1]).reshape(len(rows), -1)
    err = (y[rows].float() - r).abs()
    tol = 3e-2 + 2e-2 * r.abs()
    assert (err <= tol).all(), f"{M}x{N}x{K}: max err {err.max():.4g}, {(err > tol).sum()} bad"
