"""Gemma (head_dim 256, GeGLU), StarCoder2 (LayerNorm + biases + tanh-GELU MLP) and Qwen3 (q/k norm) on the
gfx950 kernels: engine prefill logits vs the CPU fp32 reference of the same weights, and graph decode."""
import pytest
import torch

from generativeaiexamples_amd import ops
from generativeaiexamples_amd.engine import EngineConfig, LLMEngine, SamplingParams
from generativeaiexamples_amd.engine.tokenizer import small_byte_tokenizer
from generativeaiexamples_amd.models import LlamaConfig, LlamaModel

pytestmark = pytest.mark.gpu

FAMILIES = {
    "gemma-d256": dict(arch="gemma", mlp="geglu", embed_scale=True, tie_embeddings=True, num_heads=4,
                       num_kv_heads=1, head_dim=256),
    "gemma-mha-d256": dict(arch="gemma", mlp="geglu", embed_scale=True, tie_embeddings=True, num_heads=2,
                           num_kv_heads=2, head_dim=256),
    "starcoder2": dict(arch="starcoder2", norm="layernorm", mlp="gelu_tanh", qkv_bias=True, o_bias=True,
                       mlp_bias=True, num_heads=8, num_kv_heads=2, head_dim=128, hidden_size=512),
    "qwen3": dict(arch="qwen3", qk_norm=True),
}


def _pair(cuda, kw):
    cfg = LlamaConfig.tiny(**kw)
    g = LlamaModel(cfg, device=cuda).random_init(7)
    c = LlamaModel(cfg, device="cpu")
    for k in c.w:
        c.w[k].copy_(ops.natural_weight(g.w[k]).cpu())
    return g, c


@pytest.mark.parametrize("name", list(FAMILIES))
def test_family_prefill_logits_match_cpu(cuda, name):
    g, c = _pair(cuda, FAMILIES[name])
    tok = small_byte_tokenizer(512)
    prompts = [list(range(3, 3 + n)) for n in (9, 70, 130)]
    outs = []
    for m in (g, c):
        eng = LLMEngine(m, tok, EngineConfig(num_blocks=64, max_model_len=512, use_graphs=False))
        for p in prompts:
            eng.add_request(p, SamplingParams(temperature=0.0, max_tokens=1))
        b = eng.sched.schedule()
        fb, _ = eng._make_batch(b)
        outs.append(m.forward(fb, eng.kv, eng.decode_ws).float().cpu())
    err = (outs[0] - outs[1]).abs().max().item()
    assert err < 0.05 * outs[1].abs().max().item() + 0.05, (name, err)


@pytest.mark.parametrize("name", list(FAMILIES))
def test_family_graph_decode_matches_eager(cuda, name):
    g, _ = _pair(cuda, FAMILIES[name])
    tok = small_byte_tokenizer(512)
    prompts = [list(range(5, 5 + n)) for n in (7, 33, 3)]
    sp = SamplingParams(temperature=0.0, max_tokens=20, ignore_eos=True)
    res = []
    for graphs, steps in ((False, 1), (True, 8)):
        eng = LLMEngine(g, tok, EngineConfig(num_blocks=128, max_model_len=512, use_graphs=graphs,
                                             graph_batch_sizes=(1, 2, 4), decode_steps=steps))
        res.append([r.output_ids for r in eng.generate(prompts, sp)])
    assert res[0] == res[1], name
