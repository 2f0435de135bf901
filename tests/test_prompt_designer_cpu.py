"""Prompt designer (SURVEY §2.9 llm-prompt-design-helper): the reference's per-model YAML (read with yaml.safe_load
from the reference tree), message building with few-shot turns and context, streaming / comparing models, and the
playground routes."""
import os
import zlib

import pytest
import torch

from generativeaiexamples_amd.chain_server.connectors import Embeddings
from generativeaiexamples_amd.chain_server.vectorstore import VectorStore
from generativeaiexamples_amd.playground.prompt_designer import PromptConfigStore, PromptDesigner, build_messages

REF_CFG = "/root/reference/community/llm-prompt-design-helper/config.yaml"


class _Emb(Embeddings):
    dim = 32

    def embed_tensor(self, texts, input_type):
        out = torch.zeros(len(texts), self.dim)
        for i, t in enumerate(texts):
            for w in t.lower().split():
                out[i, zlib.crc32(w.strip(".,?").encode()) % self.dim] += 1.0
        return torch.nn.functional.normalize(out + 1e-3, dim=-1)


class _LLM:
    def __init__(self, name, log):
        self.name, self.log = name, log

    def stream(self, messages, **kw):
        self.log.append((self.name, messages, kw))
        yield f"[{self.name}] "
        yield messages[-1]["content"].upper()


@pytest.mark.skipif(not os.path.exists(REF_CFG), reason="reference tree not present")
def test_reads_reference_config_shape(tmp_path):
    st = PromptConfigStore(REF_CFG)
    assert "meta/llama3-70b-instruct" in st.models() and "default" not in st.models()
    s = st.get("nvidia/nemotron-4-340b-instruct")
    assert s["temperature"] == 0.1 and s["max_tokens"] == 1024 and s["few_shot_examples"] == []
    assert st.get("unknown/model")["temperature"] == 0.0  # inherits default
    out = tmp_path / "cfg.yaml"
    st.save(str(out))
    assert PromptConfigStore(str(out)).get("meta/llama3-70b-instruct") == st.get("meta/llama3-70b-instruct")


def test_build_messages_and_update(tmp_path):
    st = PromptConfigStore(str(tmp_path / "p.yaml"))
    shots = [{"role": "user", "content": "2+2?"}, {"role": "assistant", "content": "4"}, {"role": "bad", "content": 1}]
    s = st.update("m", {"system_prompt": "Be terse.", "few_shot_examples": shots, "temperature": 0.3})
    assert len(s["few_shot_examples"]) == 2 and os.path.exists(tmp_path / "p.yaml")
    with pytest.raises(ValueError):
        st.update("m", {"exec": "x"})
    msgs = build_messages(s, "3+3?", context=["ctx A"], history=[{"role": "user", "content": "hi"},
                                                                   {"role": "system", "content": "ignored"}])
    assert msgs[0]["role"] == "system" and "ctx A" in msgs[0]["content"] and msgs[0]["content"].startswith("Be terse.")
    assert [m["content"] for m in msgs[1:]] == ["2+2?", "4", "hi", "3+3?"]
    assert PromptConfigStore(str(tmp_path / "p.yaml")).get("m")["temperature"] == 0.3


def test_designer_stream_compare_and_routes(tmp_path):
    from fastapi.testclient import TestClient

    from generativeaiexamples_amd.playground.app import create_app

    log = []
    st = PromptConfigStore(str(tmp_path / "p.yaml"))
    st.update("a", {"temperature": 0.5, "seed": 7})
    ctx = VectorStore("pd", _Emb(), device="cpu")
    d = PromptDesigner(st, llm_for=lambda m, s: _LLM(m, log), context_store=ctx)
    assert d.add_context(["The MI355X has 288 GB of HBM3E."]) == 1
    assert "".join(d.stream("a", "memory?", use_context=True)) == "[a] MEMORY?"
    name, msgs, kw = log[-1]
    assert "288 GB" in msgs[0]["content"] and kw["temperature"] == 0.5 and kw["seed"] == 7
    assert d.compare(["a", "b"], "hello") == {"a": "[a] HELLO", "b": "[b] HELLO"}

    c = TestClient(create_app(server_url="http://127.0.0.1:1", designer=d))
    assert c.get("/prompt-design").status_code == 200
    r = c.get("/api/prompt/config", params={"model": "a"}).json()
    assert r["settings"]["temperature"] == 0.5 and r["models"] == ["a"]
    assert c.put("/api/prompt/config", json={"model": "b", "settings": {"max_tokens": 64}}).json()["settings"][
        "max_tokens"] == 64
    assert c.put("/api/prompt/config", json={"model": "b", "settings": {"nope": 1}}).status_code == 400
    assert c.post("/api/prompt/generate", json={"model": "b", "input": "x"}).text == "[b] X"
    assert c.post("/api/prompt/compare", json={"models": ["a", "b"], "input": "y"}).json() == {"a": "[a] Y",
                                                                                             "b": "[b] Y"}
    assert c.post("/api/prompt/context", json={"texts": ["more text"]}).json() == {"chunks": 1}
