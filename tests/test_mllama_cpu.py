"""Llama-3.2-Vision (tiny geometry) through the engine on CPU vs its dense fp32 reference."""
import numpy as np
import torch

from generativeaiexamples_amd.engine import EngineConfig, LLMEngine, SamplingParams
from generativeaiexamples_amd.engine.tokenizer import small_byte_tokenizer
from generativeaiexamples_amd.models.mllama import MllamaConfig, MllamaModel


def _model():
    return MllamaModel(MllamaConfig.tiny(), device="cpu").random_init(seed=4)


def test_preprocess_tiles_and_aspect_ratio():
    m = _model()
    im = m.preprocess(np.zeros((40, 200, 3), dtype=np.uint8))  # very wide -> one row of tiles
    w, h = m.mcfg.vision.aspect_ratios[im.aspect_ratio_id - 1]
    assert h == 1 and w >= 2 and im.pixels.shape == (im.num_tiles, 3, 56, 56)


def test_vision_encoder_matches_reference():
    m = _model()
    im = m.preprocess(np.random.RandomState(0).randint(0, 255, (70, 130, 3), dtype=np.uint8))
    st = m.encode_images([im])[0]
    ref = m._reference_vision(im, {k: v.float() for k, v in m.w.items()})
    assert st.shape == ref.shape
    assert ((st.float() - ref).norm() / ref.norm()) < 0.02


def test_engine_with_and_without_image_matches_reference():
    m = _model()
    im = m.preprocess(np.random.RandomState(1).randint(0, 255, (60, 60, 3), dtype=np.uint8))
    eng = LLMEngine(m, small_byte_tokenizer(m.cfg.vocab_size),
                    EngineConfig(max_num_seqs=4, max_batched_tokens=256, max_model_len=512, use_graphs=False))
    prompt = [1] + list(range(10, 40))
    r_img = eng.add_request(prompt, SamplingParams(temperature=0, max_tokens=1), images=[im])
    r_txt = eng.add_request(prompt, SamplingParams(temperature=0, max_tokens=1))
    while eng.has_work():
        eng.step()
    for r, image in ((r_img, im), (r_txt, None)):
        ref = m.reference_forward(torch.tensor(prompt), image)[-1]
        top = ref.topk(2)
        if float(top.values[0] - top.values[1]) > 0.05:  # skip bf16 near-ties
            assert r.output_ids[0] == int(top.indices[0])
    assert not m.cross.seqs and len(m.cross.free) == m.cross.pad_block  # cross blocks released
