"""Constrained decoding on the GPU: the token_mask HIP kernel against the reference, and guided
generation through the engine's captured decode graphs (guided rows run single-step)."""
import json

import numpy as np
import pytest
import torch

from generativeaiexamples_amd import ops
from generativeaiexamples_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("V", [512, 128256, 1000])
def test_token_mask_kernel(cuda, V):
    torch.manual_seed(V)
    B, R = 7, 4
    W = (V + 31) // 32
    logits = torch.randn(B, V, device=cuda)
    rows = torch.tensor([6, 0, 3, 2], dtype=torch.int32, device=cuda)
    mask = torch.randint(-2**31, 2**31 - 1, (R, W), dtype=torch.int32, device=cuda)
    mask[1] = -1  # all allowed
    want = ref.token_mask(logits.cpu().clone(), rows.cpu(), mask.cpu())
    got = ops.token_mask(logits.clone(), rows, mask)
    assert torch.equal(torch.isinf(got).cpu(), torch.isinf(want))
    fin = torch.isfinite(want)
    assert torch.equal(got.cpu()[fin], want[fin])


def test_engine_guided_gpu(cuda):
    from generativeaiexamples_amd.engine import EngineConfig, LLMEngine, SamplingParams
    from generativeaiexamples_amd.engine.guided import Guide, validate
    from generativeaiexamples_amd.engine.tokenizer import llama3_byte_tokenizer
    from generativeaiexamples_amd.models import LlamaConfig, LlamaModel

    schema = {"type": "object", "properties": {"city": {"type": "string", "maxLength": 10},
                                               "temp_c": {"type": "number"},
                                               "tags": {"type": "array", "items": {"enum": ["a", "b"]}, "maxItems": 4}},
              "required": ["city", "temp_c"]}
    tok = llama3_byte_tokenizer()
    cfg = LlamaConfig.tiny(vocab_size=128256)
    model = LlamaModel(cfg, device=cuda).random_init(3)
    eng = LLMEngine(model, tok, EngineConfig(max_num_seqs=8, num_blocks=256, max_model_len=1024))
    eng.capture_graphs(max_bs=8)
    g = Guide.json_schema(schema, tok)
    prompts = [tok.encode(f"weather {i}") for i in range(6)]
    ps = [SamplingParams(temperature=1.0, top_p=1.0, max_tokens=40 + 20 * i, guided=g, seed=i) for i in range(5)]
    ps.append(SamplingParams(temperature=0.0, max_tokens=30, ignore_eos=True))  # unguided neighbour
    reqs = eng.generate(prompts, ps)
    for r in reqs[:5]:
        assert validate(json.loads(r.text), schema), r.text
    assert len(reqs[5].output_ids) == 30
    assert eng.stats["graph_steps"] > 0
