"""Chain-server API contract on the CPU plumbing configuration (tiny random-init models): every route,
SSE framing, validation ranges (422), sanitisation, upload / list / search / delete."""
import importlib
import json
import os

import pytest


@pytest.fixture(scope="module")
def client(tmp_path_factory):
    tmp = tmp_path_factory.mktemp("cs")
    env = {"APP_ENGINE_LLM": "tiny-llama", "APP_ENGINE_EMBEDDER": "tiny-e5", "APP_ENGINE_DEVICE": "cpu",
           "APP_ENGINE_RERANKER": "tiny-reranker", "APP_RETRIEVER_SCORETHRESHOLD": "-1",
           "EXAMPLE_PATH": "basic_rag/langchain", "UPLOAD_DIR": str(tmp / "up"), "GAI_LAZY_EXAMPLE": "1",
           "PROMPT_CONFIG_FILE": str(tmp / "none.yaml"), "APP_CONFIG_FILE": str(tmp / "none.json")}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
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
    utils.set_hub(None)


def _sse(resp):
    frames = [ln for ln in resp.text.split("\n\n") if ln.strip()]
    out = []
    for f in frames:
        assert f.startswith("data: "), f
        out.append(json.loads(f[6:]))
    return out


def test_health(client):
    r = client.get("/health")
    assert r.status_code == 200 and r.json() == {"message": "Service is up."}


def test_upload_list_search_delete(client):
    txt = ("MI355X accelerators have 288 GB of HBM3E memory. " * 30 + "\n\n" +
           "CDNA4 wavefronts are 64 lanes wide and MFMA units do matrix math. " * 30)
    r = client.post("/documents", files={"file": ("notes.txt", txt.encode(), "text/plain")})
    assert r.status_code == 200, r.text
    assert r.json() == {"message": "File uploaded successfully"}
    r = client.get("/documents")
    assert r.status_code == 200 and "notes.txt" in r.json()["documents"]
    r = client.post("/search", json={"query": "How much memory?", "top_k": 2})
    assert r.status_code == 200, r.text
    chunks = r.json()["chunks"]
    assert 1 <= len(chunks) <= 2 and chunks[0]["filename"] == "notes.txt"
    assert set(chunks[0]) == {"content", "filename", "score"}
    r = client.delete("/documents", params={"filename": "notes.txt"})
    assert r.status_code == 200 and "deleted successfully" in r.json()["message"]
    assert "notes.txt" not in client.get("/documents").json()["documents"]


def test_generate_sse_framing(client):
    client.post("/documents", files={"file": ("kb.md", b"# Title\n\nThe answer is forty two. " * 20, "text/markdown")})
    body = {"messages": [{"role": "user", "content": "What is the answer?"}], "use_knowledge_base": True,
            "max_tokens": 8, "temperature": 0.2, "top_p": 0.7}
    r = client.post("/generate", json=body)
    assert r.status_code == 200
    assert r.headers["content-type"].startswith("text/event-stream")
    frames = _sse(r)
    assert frames[-1]["choices"][0]["finish_reason"] == "[DONE]"
    assert frames[-1]["choices"][0]["message"] == {"role": "assistant", "content": ""}
    for f in frames:
        assert set(f) == {"id", "choices"}
        assert f["choices"][0]["index"] == 0
    body["use_knowledge_base"] = False
    frames = _sse(client.post("/generate", json=body))
    assert frames[-1]["choices"][0]["finish_reason"] == "[DONE]"


@pytest.mark.parametrize("patch", [{"temperature": 0.05}, {"temperature": 1.5}, {"top_p": 0.0}, {"max_tokens": 2000},
                                   {"use_knowledge_base": "maybe"}, {"messages": [{"role": "robot", "content": "x"}]}])
def test_generate_validation_422(client, patch):
    body = {"messages": [{"role": "user", "content": "hi"}], "use_knowledge_base": False}
    body.update(patch)
    r = client.post("/generate", json=body)
    assert r.status_code == 422
    d = r.json()["detail"]
    assert isinstance(d, list) and all("input" not in e for e in d)


def test_search_validation(client):
    assert client.post("/search", json={"query": "x", "top_k": 26}).status_code == 422


def test_sanitize():
    from generativeaiexamples_amd.chain_server.sanitize import clean

    assert clean("<script>alert(1)</script>hello") == "alert(1)hello"
    assert clean("<b>bold</b> & co") == "<b>bold</b> &amp; co"
    assert clean("a < b") == "a &lt; b"


def test_config_env_precedence(tmp_path, monkeypatch):
    from generativeaiexamples_amd.chain_server.configuration import AppConfig

    f = tmp_path / "c.yaml"
    f.write_text("retriever:\n  topK: 7\n")
    monkeypatch.setenv("APP_RETRIEVER_TOPK", "9")
    monkeypatch.setenv("APP_RETRIEVER_SCORETHRESHOLD", "0.5")
    monkeypatch.setenv("APP_TEXTSPLITTER_CHUNKSIZE", "300")
    c = AppConfig.from_file(str(f))
    assert c.retriever.top_k == 7            # file beats env
    assert c.retriever.score_threshold == 0.5  # env fills missing keys
    assert c.text_splitter.chunk_size == 300
    assert c.vector_store.nlist == 64          # default
