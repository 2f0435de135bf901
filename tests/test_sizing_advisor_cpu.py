"""Sizing advisor on the RAG-Blueprint-2.x API (SURVEY §2.9 vgpu-sizing-advisor): collections / documents / task
ingestion, streaming generate with citations and usage, search, structured MI355X recommendations, GPU detection and
the test / apply configuration event streams - scripted LLM, hashing embedder, CPU."""
import json
import os
import time
import zlib

import pytest
import torch

from generativeaiexamples_amd.chain_server.connectors import Embeddings
from generativeaiexamples_amd.community.sizing_advisor import CollectionManager, create_ingestor_app, create_rag_app
from generativeaiexamples_amd.community.sizing_advisor.deploy import gpu_code
from generativeaiexamples_amd.community.sizing_advisor.rag_server import REWRITE_SYSTEM, _structured_config
from generativeaiexamples_amd.rag.guardrails import Guardrails

DOCS = {"falcon.txt": "The Falcon sensor measures grid losses in Norway. It was released by Contoso Labs.",
        "mi355x.txt": "An MI355X GPU has 288 GB of HBM3E memory and 8 TB/s of bandwidth."}


class _HashEmb(Embeddings):
    dim = 64

    def embed_tensor(self, texts, input_type):
        out = torch.zeros(len(texts), self.dim)
        for i, t in enumerate(texts):
            for w in t.lower().split():
                out[i, zlib.crc32(w.strip(".,?").encode()) % self.dim] += 1.0
        return torch.nn.functional.normalize(out + 1e-3, dim=-1)


class _LLM:
    def __init__(self, structured='{"model": "llama3-70b", "num_gpus": null, "concurrency": 32, '
                                  '"prompt_tokens": 2000, "response_tokens": 200, "dtype": "bf16", '
                                  '"kv_dtype": "fp8", "reasoning": "70B needs room for KV."}'):
        self.structured, self.seen = structured, []

    def invoke(self, messages, **kw):
        self.seen.append(messages)
        if messages[0]["content"] == REWRITE_SYSTEM:
            return "falcon sensor grid losses\nextra line"
        if "recommend a GPU deployment" in messages[0]["content"]:
            return self.structured
        return "ok"

    def stream(self, messages, **kw):
        self.seen.append(messages)
        yield from ["Hello", " there", "!"]


@pytest.fixture()
def servers(tmp_path):
    from fastapi.testclient import TestClient

    mgr = CollectionManager(_HashEmb(), str(tmp_path / "uploads"), device="cpu")
    llm = _LLM()
    gr = Guardrails(input_rails={"topic": lambda t: "forbidden" not in t})
    rag = create_rag_app(lambda model: llm, mgr, guardrails=gr, models=lambda: ["local-llm"],
                         measure_fn=lambda preset, **kw: {"model": preset, "tpot_ms": 5.0, **kw},
                         launch_fn=lambda preset, **kw: iter([{"status": "starting", "preset": preset, **kw},
                                                              {"status": "ready"}]),
                         detect_fn=lambda: {"gpu_model": "MI355X", "gpu_count": 1, "gpu_memory_mb": 294896})
    return TestClient(create_ingestor_app(mgr)), TestClient(rag), mgr, llm


def _upload(ing, names, method="post", **data):
    files = [("documents", (n, DOCS[n].encode(), "text/plain")) for n in names]
    body = {"collection_name": "kb", "blocking": True, "split_options": {"chunk_size": 200, "chunk_overlap": 0}}
    body.update(data)
    return getattr(ing, method)("/documents", files=files, data={"data": json.dumps(body)})


def _sse(resp):
    return [json.loads(line[6:]) for line in resp.text.split("\n\n") if line.startswith("data: ")]


def test_collections_and_documents(servers):
    ing, _, mgr, _ = servers
    assert ing.get("/health").json()["message"] == "Ingestion Service is up."
    r = ing.post("/collections", params={"collection_names": ["kb", "bad name!"]}).json()
    assert r["successful"] == ["kb"] and r["failed"][0]["collection_name"] == "bad name!"
    assert ing.post("/collections", json=["other"]).json()["successful"] == ["other"]
    r = _upload(ing, ["falcon.txt", "mi355x.txt"]).json()
    assert r["total_documents"] == 2 and len(r["documents"]) == 2 and r["failed_documents"] == []
    dup = _upload(ing, ["falcon.txt"]).json()
    assert dup["documents"] == [] and "already exists" in dup["failed_documents"][0]["error_message"]
    assert _upload(ing, ["falcon.txt"], method="patch").json()["documents"] == [{"document_name": "falcon.txt"}]
    task = _upload(ing, ["mi355x.txt"], method="patch", blocking=False).json()
    for _ in range(200):
        st = ing.get("/status", params={"task_id": task["task_id"]}).json()
        if st["state"] != "PENDING":
            break
        time.sleep(0.02)
    assert st["state"] == "FINISHED" and st["result"]["documents"] == [{"document_name": "mi355x.txt"}]
    assert ing.get("/status", params={"task_id": "nope"}).json()["state"] == "UNKNOWN"
    docs = ing.get("/documents", params={"collection_name": "kb"}).json()
    assert docs["total_documents"] == 2
    cols = {c["collection_name"]: c["num_entities"] for c in ing.get("/collections").json()["collections"]}
    assert cols["kb"] == 2 and cols["other"] == 0
    r = ing.delete("/documents", params={"collection_name": "kb", "document_names": ["falcon.txt"]}).json()
    assert r["total_documents"] == 1
    assert ing.get("/documents", params={"collection_name": "kb"}).json()["documents"] == [
        {"document_name": "mi355x.txt"}]
    assert ing.delete("/collections", params={"collection_names": ["other", "ghost"]}).json()["total_failed"] == 1
    # a collection name is a directory under the upload dir: path-like names are refused before anything is written
    r = _upload(ing, ["falcon.txt"], collection_name="../escape")
    assert r.status_code == 400 and not os.path.exists(os.path.join(mgr.upload_dir, "..", "escape"))
    with pytest.raises(ValueError):
        mgr.save_upload("../x", "a.txt", b"")


def test_generate_stream_citations_usage(servers):
    ing, rag, _, llm = servers
    _upload(ing, ["falcon.txt", "mi355x.txt"])
    body = {"messages": [{"role": "user", "content": "What does the Falcon sensor measure?"}], "collection_name": "kb",
            "reranker_top_k": 1, "model": "m"}
    chunks = _sse(rag.post("/generate", json=body))
    assert "".join(c["choices"][0]["delta"]["content"] for c in chunks) == "Hello there!"
    first, last = chunks[0], chunks[-1]
    assert first["citations"]["total_results"] == 1
    assert first["citations"]["results"][0]["document_name"] == "falcon.txt"
    assert last["choices"][0]["finish_reason"] == "stop" and last["usage"]["completion_tokens"] == 2
    assert last["usage"]["total_tokens"] == last["usage"]["prompt_tokens"] + 2
    assert "Falcon sensor measures grid losses" in llm.seen[-1][0]["content"]  # context in the system prompt
    assert chunks[-2]["choices"][0]["message"]["content"] == "Hello there!"
    # alias, no knowledge base, citations off
    body.update(use_knowledge_base=False)
    c2 = _sse(rag.post("/chat/completions", json=body))
    assert c2[0]["citations"]["total_results"] == 0
    # guardrails: the input rail blocks the request
    body.update(use_knowledge_base=True, enable_guardrails=True,
                messages=[{"role": "user", "content": "a forbidden question"}])
    assert "can't respond" in "".join(c["choices"][0]["delta"]["content"] for c in _sse(rag.post("/generate",
                                                                                                  json=body)))


def test_search_and_query_rewriting(servers):
    ing, rag, _, llm = servers
    _upload(ing, ["falcon.txt", "mi355x.txt"])
    r = rag.post("/search", json={"query": "MI355X GPU HBM3E memory bandwidth", "collection_name": "kb",
                                  "reranker_top_k": 1}).json()
    assert r["results"][0]["document_name"] == "mi355x.txt" and r["results"][0]["score"] > 0
    r = rag.post("/search", json={"query": "what does it measure?", "collection_name": "kb", "reranker_top_k": 1,
                                  "enable_query_rewriting": True,
                                  "messages": [{"role": "user", "content": "tell me about the falcon sensor"}]}).json()
    assert r["results"][0]["document_name"] == "falcon.txt"
    assert any(m[0]["content"] == REWRITE_SYSTEM for m in llm.seen)
    assert rag.post("/search", json={"query": "x", "collection_name": "missing"}).json()["total_results"] == 0


def test_structured_recommendation(servers):
    _, rag, _, _ = servers
    out = rag.post("/generate_structured", json={"messages": [{"role": "user", "content": "Serve a 70B model"}],
                                                 "use_knowledge_base": False}).json()
    so = out["structured_output"]
    assert so["configuration"]["model"] == "llama3-70b" and so["configuration"]["kv_dtype"] == "fp8"
    assert so["parameters"]["tp"] >= 1 and so["parameters"]["fits"] and so["description"] == "70B needs room for KV."
    cfg, _ = _structured_config("no json here", "serve mixtral-8x7b in fp8 for 100 concurrent users on 4 GPUs",
                                ["llama3-8b", "mixtral-8x7b"])
    assert (cfg.model, cfg.concurrency, cfg.num_gpus, cfg.dtype) == ("mixtral-8x7b", 100, 4, "fp8")
    cfg, _ = _structured_config('{"model": "gpt-9", "num_gpus": 3}', "hi", ["llama3-8b"])
    assert cfg.model == "llama3-8b" and cfg.num_gpus is None


def test_models_gpu_and_configuration_events(servers, tmp_path):
    ing, rag, _, _ = servers
    models = {m["id"]: m for m in rag.get("/available-models").json()["models"]}
    assert models["llama3-8b"]["size"] == "8.0B" and "tiny-llama" not in models
    assert rag.get("/detect-gpu").json()["gpu_model"] == "MI355X"
    cfg = {"configuration": {"model": "llama3-8b", "concurrency": 16, "prompt_tokens": 512, "response_tokens": 64}}
    ev = _sse(rag.post("/test-configuration", json=cfg))
    assert [e["status"] for e in ev] == ["planning", "plan", "measuring", "done"]
    assert ev[-1]["measured"]["concurrency"] == 16 and ev[-1]["estimated"]["tpot_ms"] > 0
    ev = _sse(rag.post("/test-configuration", json={**cfg, "measure": False}))
    assert ev[-1]["status"] == "done" and "measured" not in ev[-1]
    assert _sse(rag.post("/test-configuration", json={"configuration": {"model": "nope"}}))[-1]["status"] == "error"
    ev = _sse(rag.post("/apply-configuration", json={**cfg, "port": 9100}))
    assert ev[0]["preset"] == "llama3-8b" and ev[0]["port"] == 9100 and ev[-1]["status"] == "ready"
    assert rag.post("/apply-configuration", json={"configuration": {"model": "nope"}}).status_code == 400
    _upload(ing, ["falcon.txt"])
    got = rag.get("/api/download-citation", params={"source": "falcon.txt", "collection_name": "kb"})
    assert got.status_code == 200 and got.content == DOCS["falcon.txt"].encode()
    assert rag.get("/api/download-citation", params={"source": "../../etc/passwd", "collection_name": "kb"}
                   ).status_code == 404


def test_one_measurement_at_a_time(tmp_path):
    import threading

    from fastapi.testclient import TestClient

    started, release = threading.Event(), threading.Event()

    def measure(preset, **kw):
        started.set()
        release.wait(10)
        return {"model": preset, **kw}

    app = create_rag_app(lambda model: None, CollectionManager(_HashEmb(), str(tmp_path / "u"), device="cpu"),
                         measure_fn=measure, detect_fn=lambda: {"gpu_model": "MI355X"})
    c = TestClient(app)
    cfg = {"configuration": {"model": "llama3-8b", "concurrency": 4, "prompt_tokens": 128, "response_tokens": 16}}
    first = {}
    t = threading.Thread(target=lambda: first.update(r=_sse(c.post("/test-configuration", json=cfg))))
    t.start()
    assert started.wait(10)
    assert _sse(c.post("/test-configuration", json=cfg))[-1]["status"] == "busy"
    release.set()
    t.join(10)
    assert first["r"][-1]["status"] == "done"
    assert _sse(c.post("/test-configuration", json=cfg))[-1]["status"] == "done"  # the lock was released


def test_no_gpu_paths(tmp_path):
    from fastapi.testclient import TestClient

    mgr = CollectionManager(_HashEmb(), str(tmp_path / "u"), device="cpu")
    rag = TestClient(create_rag_app(lambda m: _LLM(), mgr, detect_fn=lambda: None))
    assert rag.get("/detect-gpu").status_code == 404
    ev = _sse(rag.post("/test-configuration", json={"configuration": {"model": "llama3-8b"}}))
    assert ev[-1]["status"] == "skipped"
    assert gpu_code("AMD Instinct MI355X") == "MI355X" and gpu_code("AMD Instinct MI300X") == "MI300X"


def test_persisted_collections_reopen(tmp_path):
    mgr = CollectionManager(_HashEmb(), str(tmp_path / "u"), persist_dir=str(tmp_path / "p"), device="cpu")
    p = mgr.save_upload("kb", "falcon.txt", DOCS["falcon.txt"].encode())
    assert mgr.ingest("kb", [p])["documents"] == [{"document_name": "falcon.txt"}]
    again = CollectionManager(_HashEmb(), str(tmp_path / "u"), persist_dir=str(tmp_path / "p"), device="cpu")
    assert again.list()["collections"] == [{"collection_name": "kb", "num_entities": 1}]
    assert again.search("kb", "Falcon sensor", 1)[0][0].metadata["filename"] == "falcon.txt"


def test_launch_server_reports_exit():
    from generativeaiexamples_amd.community.sizing_advisor.deploy import launch_server

    ev = list(launch_server("llama3-8b", port=9199, python="/bin/false", poll_s=0.05, timeout_s=10))
    assert ev[0]["status"] == "starting" and "--llm llama3-8b" in ev[0]["command"]
    assert ev[-1]["status"] == "error" and "exited with code 1" in ev[-1]["message"]
