"""Multi-LoRA serving: unmerged per-request adapters reproduce the merged-weights model, requests for
different adapters and the base model share batches, and /v1 routes a model name to its adapter."""
import copy

import torch

from generativeaiexamples_amd.engine import EngineConfig, LLMEngine, SamplingParams
from generativeaiexamples_amd.engine.tokenizer import small_byte_tokenizer
from generativeaiexamples_amd.models.llama import LlamaConfig, LlamaModel
from generativeaiexamples_amd.parallel.dist import DistContext
from generativeaiexamples_amd.training.lora import LoRAAdapter, LoRAConfig


def _model():
    return LlamaModel(LlamaConfig.tiny(num_layers=2), device="cpu", dist_ctx=DistContext(),
                      dtype=torch.float32).random_init(seed=3)


def _adapter(m, seed):
    ad = LoRAAdapter(m, LoRAConfig(r=4, alpha=8, targets=("qkv", "o")), seed=seed)
    with torch.no_grad():
        for j, (k, v) in enumerate(ad.params.items()):
            if k.endswith(".B"):
                v.normal_(0, 0.5, generator=torch.Generator().manual_seed(seed * 100 + j))
    return ad


def _run(m, reqs):
    eng = LLMEngine(m, small_byte_tokenizer(512), EngineConfig(max_num_seqs=8, max_model_len=256, use_graphs=False))
    out = [eng.add_request(p, SamplingParams(temperature=0, max_tokens=6), lora=l) for p, l in reqs]
    while eng.has_work():
        eng.step()
    return [r.output_ids for r in out]


def test_unmerged_adapters_match_merged_models(tmp_path):
    base = _model()
    a1, a2 = _adapter(base, 1), _adapter(base, 2)
    a1.save(str(tmp_path / "a1"))
    served = copy.deepcopy(base)
    served.add_lora("a1", str(tmp_path / "a1"))
    served.add_lora("a2", a2)
    prompts = [[1] + list(range(20 + i, 40 + i)) for i in range(3)]
    mixed = _run(served, [(prompts[0], "a1"), (prompts[1], None), (prompts[2], "a2"), (prompts[0], None)])
    m1, m2 = copy.deepcopy(base), copy.deepcopy(base)
    a1.merge_into(m1)
    a2.merge_into(m2)
    assert mixed[0] == _run(m1, [(prompts[0], None)])[0]
    assert mixed[2] == _run(m2, [(prompts[2], None)])[0]
    assert mixed[1] == _run(base, [(prompts[1], None)])[0]
    assert mixed[3] == _run(base, [(prompts[0], None)])[0]
    assert mixed[0] != mixed[3]  # the adapter changes the output


def test_openai_routes_adapter_by_model_name(tmp_path):
    from fastapi.testclient import TestClient

    from generativeaiexamples_amd.serving.hub import HubSpec, ServiceHub
    from generativeaiexamples_amd.serving.openai_api import create_openai_app

    hub = ServiceHub.build(HubSpec(llm="tiny-llama", embedder=None, reranker=None, device="cpu", served_llm_name="base",
                                   max_num_seqs=4, max_model_len=256))
    eng = hub.llm("base").engine
    ad = _adapter(eng.model, 5)
    ad.save(str(tmp_path / "ad"))
    hub.shutdown()
    hub = ServiceHub.build(HubSpec(llm="tiny-llama", embedder=None, reranker=None, device="cpu", served_llm_name="base",
                                   max_num_seqs=4, max_model_len=256, lora_adapters={"my-lora": str(tmp_path / "ad")}))
    with TestClient(create_openai_app(hub)) as c:
        body = {"messages": [{"role": "user", "content": "hello there"}], "max_tokens": 6, "temperature": 0}
        base_txt = c.post("/v1/chat/completions", json=dict(body, model="base")).json()["choices"][0]["message"]
        lora_txt = c.post("/v1/chat/completions", json=dict(body, model="my-lora")).json()["choices"][0]["message"]
        ids = {m["id"] for m in c.get("/v1/models").json()["data"]}
    hub.shutdown()
    assert "my-lora" in ids
    assert base_txt != lora_txt
