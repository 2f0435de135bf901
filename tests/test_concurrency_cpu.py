"""Concurrent clients against the /v1 server ("Python stress tests with concurrent clients
against async endpoints"): 16 threads mix streaming chat, embeddings and ranking on one uvicorn server;
every request must succeed and greedy chat answers must equal the answers of the same prompts run
serially (continuous batching must not mix up sequences)."""
import socket
import threading
import time

import httpx
import pytest


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def server():
    import uvicorn

    from generativeaiexamples_amd.serving.hub import HubSpec, ServiceHub
    from generativeaiexamples_amd.serving.openai_api import create_openai_app

    hub = ServiceHub.build(HubSpec(llm="tiny-llama", embedder="tiny-e5", reranker="tiny-reranker", device="cpu",
                                   served_llm_name="m", max_num_seqs=16, max_model_len=512))
    port = _port()
    cfg = uvicorn.Config(create_openai_app(hub), host="127.0.0.1", port=port, log_level="warning")
    srv = uvicorn.Server(cfg)
    th = threading.Thread(target=srv.run, daemon=True)
    th.start()
    for _ in range(200):
        try:
            if httpx.get(f"http://127.0.0.1:{port}/v1/health/ready").status_code == 200:
                break
        except httpx.HTTPError:
            time.sleep(0.05)
    yield f"http://127.0.0.1:{port}"
    srv.should_exit = True
    th.join(10)
    hub.shutdown()


def _chat(url, i):
    body = {"model": "m", "messages": [{"role": "user", "content": f"question number {i} about kernels"}],
            "max_tokens": 8, "temperature": 0, "stream": i % 2 == 0}
    r = httpx.post(url + "/v1/chat/completions", json=body, timeout=120)
    r.raise_for_status()
    if body["stream"]:
        import json
        txt = ""
        for ln in r.text.split("\n\n"):
            if ln.startswith("data: ") and ln != "data: [DONE]":
                ch = json.loads(ln[6:])["choices"]
                if ch:
                    txt += ch[0]["delta"].get("content") or ""
        return txt
    return r.json()["choices"][0]["message"]["content"]


def test_concurrent_mixed_clients(server):
    serial = {i: _chat(server, i) for i in range(8)}
    results, errors = {}, []

    def worker(k):
        try:
            for j in range(3):
                i = (k + j) % 8
                kind = (k + j) % 3
                if kind == 0:
                    results[(k, j)] = (i, _chat(server, i))
                elif kind == 1:
                    r = httpx.post(server + "/v1/embeddings", json={"model": "tiny-e5", "input": [f"doc {k} {j}"] * 3,
                                                                     "input_type": "passage"}, timeout=60)
                    r.raise_for_status()
                    assert len(r.json()["data"]) == 3
                else:
                    r = httpx.post(server + "/v1/ranking", json={"model": "tiny-reranker", "query": {"text": "q"},
                                                                  "passages": [{"text": f"p{n}"} for n in range(5)]},
                                   timeout=60)
                    r.raise_for_status()
                    assert len(r.json()["rankings"]) == 5
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(k,)) for k in range(16)]
    for t in th:
        t.start()
    for t in th:
        t.join(300)
    assert not errors, errors[:3]
    for i, txt in results.values():
        assert txt == serial[i], (i, txt, serial[i])
    assert httpx.get(server + "/v1/health/ready").status_code == 200
