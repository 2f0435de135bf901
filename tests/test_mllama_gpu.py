"""Llama-3.2-Vision on the HIP kernels: vision encoder vs fp32 reference, engine with HIP-graph decode
and cross-attention, fp8 weights, and the real 11B geometry's vision encoder."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from generativeaiexamples_amd import ops
from generativeaiexamples_amd.engine import EngineConfig, LLMEngine, SamplingParams
from generativeaiexamples_amd.engine.tokenizer import small_byte_tokenizer
from generativeaiexamples_amd.models.mllama import MllamaConfig, MllamaModel, MllamaVisionConfig

pytestmark = pytest.mark.gpu


def _img(seed, h=70, w=130):
    return np.random.RandomState(seed).randint(0, 255, (h, w, 3), dtype=np.uint8)


def test_tiny_vision_encoder(cuda):
    m = MllamaModel(MllamaConfig.tiny(), device="cuda").random_init(seed=4)
    im = m.preprocess(_img(0))
    st = m.encode_images([im])[0]
    ref = m._reference_vision(im, {k: ops.natural_weight(v).float().cpu() for k, v in m.w.items()})
    assert ((st.float().cpu() - ref).norm() / ref.norm()) < 0.03


def test_padded_head_dim_vision_layer(cuda):
    """head_dim 80 -> padded 128 attention (the 11B geometry) on a 2-layer encoder."""
    cfg = MllamaConfig.tiny(vision=MllamaVisionConfig(hidden_size=1280, num_layers=2, num_global_layers=1,
                                                      num_heads=16, intermediate_size=512, image_size=112,
                                                      intermediate_layers=(1,)))
    m = MllamaModel(cfg, device="cuda").random_init(seed=5)
    im = m.preprocess(_img(1, 100, 100))
    st = m.encode_images([im])[0]
    ref = m._reference_vision(im, {k: ops.natural_weight(v).float().cpu() for k, v in m.w.items()})
    assert ((st.float().cpu() - ref).norm() / ref.norm()) < 0.03


@pytest.mark.parametrize("graphs", [False, True])
def test_engine_cross_attention_greedy(cuda, graphs):
    m = MllamaModel(MllamaConfig.tiny(), device="cuda").random_init(seed=4)
    eng = LLMEngine(m, small_byte_tokenizer(m.cfg.vocab_size),
                    EngineConfig(max_num_seqs=8, max_batched_tokens=512, max_model_len=512, use_graphs=graphs))
    if graphs:
        eng.capture_graphs(max_bs=8)
    prompt = [1] + list(range(10, 50))
    ims = [m.preprocess(_img(s)) for s in range(3)]
    reqs = [eng.add_request(prompt, SamplingParams(temperature=0, max_tokens=6), images=[ims[i]]) for i in range(3)]
    reqs.append(eng.add_request(prompt, SamplingParams(temperature=0, max_tokens=6)))
    while eng.has_work():
        eng.step()
    if graphs:
        assert eng.stats["graph_steps"] > 0
    for r, im in zip(reqs, ims + [None]):
        ids = prompt + r.output_ids[:-1]
        ref = m.reference_forward(torch.tensor(ids), im)[len(prompt) - 1:]
        agree = sum(int(ref[t].argmax()) == r.output_ids[t] for t in range(len(r.output_ids)))
        assert agree >= len(r.output_ids) - 1, (r.output_ids, ref.argmax(-1).tolist())
    assert not m.cross.seqs


def test_fp8_mllama_runs(cuda):
    m = MllamaModel(MllamaConfig.tiny(), device="cuda").random_init(seed=4)
    im = m.preprocess(_img(3))
    st16 = m.encode_images([im])[0].float()
    m.quantize_fp8()
    st8 = m.encode_images([im])[0].float()
    assert F.cosine_similarity(st8.flatten(), st16.flatten(), dim=0) > 0.97


def test_llama32_11b_vision_encoder_geometry(cuda):
    """Real 11B vision geometry (32+8 layers, 1280 hidden, 4 tiles of 560 px) with random weights."""
    cfg = MllamaConfig.llama32_11b_vision()
    cfg.text = cfg.text.__class__.tiny(num_layers=4, hidden_size=4096, num_heads=32, num_kv_heads=8, head_dim=128,
                                       intermediate_size=512)
    cfg.cross_layers = (1, 3)
    m = MllamaModel(cfg, device="cuda").random_init(seed=1)
    im = m.preprocess(_img(4, 900, 1200))
    st = m.encode_images([im])[0]
    assert st.shape == (im.num_tiles * 1601, 4096) and torch.isfinite(st.float()).all()
