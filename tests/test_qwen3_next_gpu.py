"""Qwen3-Next on gfx950: the gated-DeltaNet decode kernel (in-place slot-pool state update) vs the
fp32 recurrence, and the tiny hybrid model served by the engine (bf16, HIP kernels) vs its CPU fp32
copy, eager vs HIP-graph decode."""
import pytest
import torch

from generativeaiexamples_amd import ops
from generativeaiexamples_amd.engine import EngineConfig, LLMEngine, SamplingParams
from generativeaiexamples_amd.engine.tokenizer import small_byte_tokenizer
from generativeaiexamples_amd.models.qwen3_next import Qwen3NextConfig, Qwen3NextModel, gdn_recurrent_step

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dk,dv", [(128, 128), (64, 256)])
def test_gdn_decode_kernel(cuda, dk, dv):
    torch.manual_seed(0)
    B, H, NS = 5, 4, 9
    q = torch.nn.functional.normalize(torch.randn(B, H, dk, device=cuda), dim=-1) * dk ** -0.5
    k = torch.nn.functional.normalize(torch.randn(B, H, dk, device=cuda), dim=-1)
    v = torch.randn(B, H, dv, device=cuda)
    g = -torch.rand(B, H, device=cuda)
    beta = torch.rand(B, H, device=cuda)
    state = torch.randn(NS, H, dk, dv, device=cuda) * 0.1
    slots = torch.tensor([7, 0, 3, 8, 5], dtype=torch.int32, device=cuda)
    want_o, want_S = gdn_recurrent_step(q, k, v, g, beta, state[slots.long()])
    before = state.clone()
    out = torch.empty(B, H, dv, device=cuda)
    ops.native().gdn_decode(q, k, v, g, beta, state, slots, out)
    assert torch.allclose(out, want_o, atol=1e-4, rtol=1e-4)
    assert torch.allclose(state[slots.long()], want_S, atol=1e-4, rtol=1e-4)
    untouched = [s for s in range(NS) if s not in slots.tolist()]
    assert torch.equal(state[untouched], before[untouched])


def _pair(cuda):
    cfg = Qwen3NextConfig.tiny()
    g = Qwen3NextModel(cfg, device=cuda).random_init(3)
    c = Qwen3NextModel(cfg, device="cpu", dtype=torch.float32)
    for k in c.w:
        c.w[k].copy_(ops.natural_weight(g.w[k]).float().cpu())
    return g, c


def test_qwen3_next_gpu_matches_cpu(cuda):
    g, c = _pair(cuda)
    tok = small_byte_tokenizer(512)
    prompts = [list(range(3, 3 + n)) for n in (9, 40, 100)]
    outs = []
    for m in (g, c):
        eng = LLMEngine(m, tok, EngineConfig(num_blocks=64, max_model_len=512, use_graphs=False))
        for p in prompts:
            eng.add_request(p, SamplingParams(temperature=0.0, max_tokens=1))
        fb, _ = eng._make_batch(eng.sched.schedule())
        outs.append(m.forward(fb, eng.kv, eng.decode_ws).float().cpu())
    err = (outs[0] - outs[1]).abs().max().item()
    assert err < 0.05 * outs[1].abs().max().item() + 0.05, err


def test_qwen3_next_graph_decode_equals_eager(cuda):
    g, _ = _pair(cuda)
    tok = small_byte_tokenizer(512)
    sp = SamplingParams(temperature=0.0, max_tokens=10, ignore_eos=True)
    prompts = [list(range(5, 5 + n)) for n in (7, 30, 64)]
    res = []
    for graphs in (False, True):
        eng = LLMEngine(g, tok, EngineConfig(num_blocks=128, max_model_len=512, use_graphs=graphs,
                                             graph_batch_sizes=(1, 2, 4)))
        res.append([r.output_ids for r in eng.generate(prompts, sp)])
        if graphs:
            assert eng.stats["graph_steps"] > 0
    assert res[0] == res[1]
    assert not g.slot_of
