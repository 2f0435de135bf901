"""Medical-device training assistant example (E7) through the chain server on tiny CPU models."""
import json
import os

import pytest

from generativeaiexamples_amd.examples.medical_device import parse_gt_qa_txt


def test_parse_gt_qa_txt():
    txt = ("Example 1:\nQuestion: How do I prime the pump?\nAnswer: Open the clamp.\nThen press PRIME.\n\n"
           "Example 2:\nQuestion: What does alarm E3 mean?\nAnswer: Occlusion downstream.\n")
    qa = parse_gt_qa_txt(txt)
    assert [q["question"] for q in qa] == ["How do I prime the pump?", "What does alarm E3 mean?"]
    assert qa[0]["gt_answer"] == "Open the clamp.\nThen press PRIME."


@pytest.fixture()
def client(tmp_path):
    env = {"APP_ENGINE_LLM": "tiny-llama", "APP_ENGINE_EMBEDDER": "tiny-e5", "APP_ENGINE_DEVICE": "cpu",
           "APP_ENGINE_RERANKER": "tiny-reranker", "APP_RETRIEVER_SCORETHRESHOLD": "-1",
           "EXAMPLE_PATH": "industries/healthcare/medical_device_training_assistant", "UPLOAD_DIR": str(tmp_path / "up"),
           "GAI_LAZY_EXAMPLE": "1", "APP_CONFIG_FILE": str(tmp_path / "none.json")}
    old = {k: os.environ.get(k) for k in list(env) + ["PROMPT_CONFIG_FILE"]}
    os.environ.update(env)
    os.environ.pop("PROMPT_CONFIG_FILE", None)
    from fastapi.testclient import TestClient

    from generativeaiexamples_amd.chain_server import server, utils, vectorstore
    utils.get_config.cache_clear()
    utils.get_prompts.cache_clear()
    utils.set_hub(None)
    vectorstore.reset_stores()
    server.app.state.example = None
    with TestClient(server.app) as c:
        yield c
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    utils.get_config.cache_clear()
    utils.get_prompts.cache_clear()
    utils.set_hub(None)


def test_medical_device_chain(client):
    manual = ("Infusion pump model X instructions for use. To prime the pump open the clamp and press PRIME. " * 20)
    r = client.post("/documents", files={"file": ("pump_ifu.txt", manual.encode(), "text/plain")})
    assert r.status_code == 200, r.text
    body = {"messages": [{"role": "user", "content": "How do I prime the pump?"}], "use_knowledge_base": True,
            "max_tokens": 6, "temperature": 0.1}
    r = client.post("/generate", json=body)
    assert r.status_code == 200
    frames = [json.loads(f[6:]) for f in r.text.split("\n\n") if f.startswith("data: ")]
    text = "".join(f["choices"][0]["message"]["content"] for f in frames)
    assert "Sources: pump_ifu.txt" in text
    assert type(server_example()).__name__ == "MedicalDeviceAssistant"


def server_example():
    from generativeaiexamples_amd.chain_server import server
    return server.example()
