"""Decoder families beyond Llama (Gemma / CodeGemma, StarCoder2, Qwen2.5, Qwen3) on the CPU reference path:
HF-checkpoint parity against ``transformers`` (random tiny configs, no download) and engine consistency
(paged KV + chunked prefill + continuous batching) against the dense oracle."""
import pytest
import torch

from generativeaiexamples_amd.engine import EngineConfig, LLMEngine, SamplingParams
from generativeaiexamples_amd.engine.tokenizer import small_byte_tokenizer
from generativeaiexamples_amd.models import LlamaConfig, LlamaModel

transformers = pytest.importorskip("transformers")

TINY = dict(vocab_size=512, hidden_size=256, intermediate_size=512, num_layers=2, num_heads=4, num_kv_heads=2,
            head_dim=64, max_position=1024, bos_token_id=1, eos_token_ids=(2,))


def _hf_pair(arch):
    """(HF model in fp32 with bf16-representable weights, our LlamaConfig) for a tiny config of `arch`."""
    common = dict(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                  num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=1024)
    if arch == "gemma":
        hf = transformers.GemmaForCausalLM(transformers.GemmaConfig(head_dim=64, hidden_activation="gelu_pytorch_tanh",
                                                                    rms_norm_eps=1e-6, **common))
        ours = LlamaConfig.tiny(arch="gemma", mlp="geglu", embed_scale=True, tie_embeddings=True, rms_eps=1e-6,
                                rope_theta=10000.0)
    elif arch == "starcoder2":
        hf = transformers.Starcoder2ForCausalLM(transformers.Starcoder2Config(
            hidden_act="gelu_pytorch_tanh", use_bias=True, norm_epsilon=1e-5, sliding_window=None,
            tie_word_embeddings=False, rope_theta=10000.0, **common))
        ours = LlamaConfig.tiny(arch="starcoder2", norm="layernorm", mlp="gelu_tanh", qkv_bias=True, o_bias=True,
                                mlp_bias=True, rope_theta=10000.0)
    elif arch == "qwen2":
        hf = transformers.Qwen2ForCausalLM(transformers.Qwen2Config(rms_norm_eps=1e-6, tie_word_embeddings=False,
                                                                    rope_theta=10000.0, **common))
        ours = LlamaConfig.tiny(arch="qwen2", qkv_bias=True, rms_eps=1e-6, rope_theta=10000.0)
    else:
        hf = transformers.Qwen3ForCausalLM(transformers.Qwen3Config(head_dim=64, rms_norm_eps=1e-6,
                                                                    tie_word_embeddings=False, rope_theta=10000.0,
                                                                    **common))
        ours = LlamaConfig.tiny(arch="qwen3", qk_norm=True, rms_eps=1e-6, rope_theta=10000.0)
    torch.manual_seed(0)
    with torch.no_grad():
        for n, p in hf.named_parameters():
            if "norm" in n and n.endswith("weight"):
                p.copy_(0.1 * torch.randn_like(p) + (0.0 if arch == "gemma" else 1.0))
            elif n.endswith("bias"):
                p.copy_(0.05 * torch.randn_like(p))
            else:
                p.copy_(0.05 * torch.randn_like(p))
            p.copy_(p.to(torch.bfloat16).float())
    return hf.float().eval(), ours


@pytest.mark.parametrize("arch", ["gemma", "starcoder2", "qwen2", "qwen3"])
def test_family_matches_transformers(arch):
    hf, cfg = _hf_pair(arch)
    m = LlamaModel(cfg, device="cpu")
    m.load_hf_state({k: v.detach() for k, v in hf.state_dict().items()})
    ids = torch.randint(3, 500, (37,), generator=torch.Generator().manual_seed(1))
    with torch.no_grad():
        ref = hf(ids[None]).logits[0].float()
    ours = m.reference_forward(ids)
    # Gemma's (1 + w) norm weights are folded into bf16 at load: allow that rounding
    tol = 3e-2 if arch == "gemma" else 1e-2
    err = (ours - ref).abs().max().item()
    assert err < tol * ref.abs().max().item(), (arch, err)
    # export round-trips to the HF layout
    sd = m.export_hf_state()
    for k, v in hf.state_dict().items():
        if k in sd:
            torch.testing.assert_close(sd[k].float(), v.float(), rtol=0, atol=2e-2 if "norm" in k else 0)


@pytest.mark.parametrize("kw", [dict(arch="gemma", mlp="geglu", embed_scale=True, tie_embeddings=True),
                                dict(arch="starcoder2", norm="layernorm", mlp="gelu_tanh", qkv_bias=True,
                                     o_bias=True, mlp_bias=True),
                                dict(arch="qwen3", qk_norm=True)])
def test_family_engine_greedy_consistent(kw):
    cfg = LlamaConfig.tiny(**kw)
    m = LlamaModel(cfg, device="cpu").random_init(5)
    tok = small_byte_tokenizer(512)
    eng = LLMEngine(m, tok, EngineConfig(max_num_seqs=4, max_batched_tokens=64, prefill_chunk=24, num_blocks=64,
                                         max_model_len=512, use_graphs=False))
    prompts = [list(range(10, 10 + n)) for n in (5, 41)]
    reqs = eng.generate(prompts, SamplingParams(temperature=0.0, max_tokens=5, ignore_eos=True))
    for p, r in zip(prompts, reqs):
        assert len(r.output_ids) == 5
        for i, t in enumerate(r.output_ids):
            lg = m.reference_forward(torch.tensor(p + r.output_ids[:i]))[-1]
            assert lg[t] >= lg.max() - 0.02 * max(1.0, float(lg.abs().max())), (kw["arch"], i)


def test_family_lora_forward_backward():
    """The SFT forward (training/forward.py) runs the same families: loss is finite and LoRA grads flow."""
    from generativeaiexamples_amd.training.forward import lm_loss
    from generativeaiexamples_amd.training.lora import LoRAAdapter, LoRAConfig

    for kw in (dict(arch="starcoder2", norm="layernorm", mlp="gelu_tanh", qkv_bias=True, o_bias=True, mlp_bias=True),
               dict(arch="gemma", mlp="geglu", embed_scale=True, tie_embeddings=True)):
        m = LlamaModel(LlamaConfig.tiny(**kw), device="cpu").random_init(2)
        for k in m.w:
            m.w[k] = m.w[k].float()
        ad = LoRAAdapter(m, LoRAConfig(r=4, targets=("qkv", "o", "fc", "gate_up", "down")))
        for v in ad.params.values():
            if v.shape[0] != 4:
                torch.nn.init.normal_(v.data, std=0.01)
        ids = torch.randint(3, 500, (2, 24))
        labels = ids.clone()
        labels[:, :8] = -100
        loss = lm_loss(m, ad, ids, labels)
        loss.backward()
        assert torch.isfinite(loss)
        assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in ad.parameters())
        target = "fc" if kw["mlp"] == "gelu_tanh" else "gate_up"
        assert f"l0.{target}.A" in ad.params
