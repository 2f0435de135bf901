"""Elastic serving: the replica router re-queues an in-flight chat completion when its replica
fails and resumes it on another one from the tokens already delivered; the supervisor restarts a TP group
whose follower rank died and the group rejoins the rotation.

Greedy decoding makes the resumed stream checkable: it must equal an uninterrupted completion."""
import json
import os
import socket
import sys
import threading
import time

import pytest

sys.path.insert(0, os.path.dirname(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _Server:
    """A FastAPI app served by uvicorn on a background thread (a replica reachable over real HTTP)."""

    def __init__(self, app):
        import uvicorn

        self.port = _free_port()
        self.server = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=self.port, log_level="warning"))
        self.thread = threading.Thread(target=self.server.run, daemon=True)
        self.thread.start()
        deadline = time.time() + 30
        while not self.server.started and time.time() < deadline:
            time.sleep(0.05)
        assert self.server.started

    @property
    def url(self):
        return f"http://127.0.0.1:{self.port}"

    def stop(self):
        self.server.should_exit = True
        self.thread.join(timeout=10)


def _stream_text(resp_text):
    text, reason, ids = [], None, []
    for ln in resp_text.split("\n\n"):
        if not ln.startswith("data: ") or ln == "data: [DONE]":
            continue
        obj = json.loads(ln[6:])
        assert "error" not in obj, obj
        for ch in obj.get("choices", []):
            text.append((ch.get("delta") or {}).get("content") or "")
            reason = ch.get("finish_reason") or reason
        ids += (obj.get("nvext") or {}).get("token_ids", [])
    return "".join(text), reason, ids


MSGS = [{"role": "user", "content": "tell me about elastic serving"}]


@pytest.fixture(scope="module")
def ckpt(tmp_path_factory):
    from _dist_workers import write_tiny_llama_ckpt

    p = str(tmp_path_factory.mktemp("elastic") / "tiny")
    write_tiny_llama_ckpt(p)
    return p


def _hub(ckpt):
    from generativeaiexamples_amd.serving.hub import HubSpec, ServiceHub

    return ServiceHub.build(HubSpec(llm="tiny-llama", llm_weights=ckpt, embedder=None, device="cpu", dtype="float32",
                                    max_num_seqs=8, max_model_len=512, max_batched_tokens=64, use_graphs=False))


def test_router_requeues_on_replica_failure(ckpt):
    from fastapi.testclient import TestClient

    from generativeaiexamples_amd.parallel.fault import RankFailure
    from generativeaiexamples_amd.serving.openai_api import create_openai_app
    from generativeaiexamples_amd.serving.router import create_router_app

    hub_a, hub_b = _hub(ckpt), _hub(ckpt)
    a, b = _Server(create_openai_app(hub_a)), _Server(create_openai_app(hub_b))
    try:
        body = {"messages": MSGS, "max_tokens": 40, "temperature": 0, "ignore_eos": True, "stream": True}
        import httpx

        ref = httpx.post(b.url + "/v1/chat/completions", json=body, timeout=60)
        ref_text, ref_reason, _ = _stream_text(ref.text)
        assert ref_reason == "length" and ref_text

        # replica A's engine fails after a few steps (a dead TP peer / watchdog: RankFailure inside step)
        eng = hub_a.llm().engine
        orig, calls = eng.step, {"n": 0}

        def failing_step():
            calls["n"] += 1
            if calls["n"] == 4:
                raise RankFailure("collective 'tp_all_reduce' failed on rank 0: injected")
            return orig()

        eng.step = failing_step
        with TestClient(create_router_app([a.url, b.url], health_interval=0.2, requeue_timeout=30)) as rc:
            r = rc.post("/v1/chat/completions", json=dict(body, nvext={"return_token_ids": True}))
            assert r.status_code == 200
            text, reason, ids = _stream_text(r.text)
            assert calls["n"] >= 4, "replica A never ran"
            assert text == ref_text and reason == "length"
            assert len(ids) == 40  # every token exactly once across the two replicas
            reps = {x["url"]: x for x in rc.get("/v1/replicas").json()["data"]}
            assert not reps[a.url]["healthy"] and reps[b.url]["healthy"]
            assert b"gai_router_requeued_total 1.0" in rc.get("/metrics").content
            # non-streaming client through the router: served by the healthy replica, usage intact
            j = rc.post("/v1/chat/completions", json=dict(body, stream=False)).json()
            assert j["choices"][0]["message"]["content"] == ref_text
            assert j["usage"]["completion_tokens"] == 40
            assert rc.get("/v1/health/ready").status_code == 200
    finally:
        a.stop()
        b.stop()
        hub_a.shutdown()
        hub_b.shutdown()


def test_resume_continues_a_completion(ckpt):
    """The replica-side half: resume_token_ids extend the prompt and count against max_tokens."""
    from fastapi.testclient import TestClient

    from generativeaiexamples_amd.serving.openai_api import create_openai_app

    hub = _hub(ckpt)
    try:
        with TestClient(create_openai_app(hub)) as c:
            body = {"messages": MSGS, "max_tokens": 20, "temperature": 0, "ignore_eos": True, "stream": True,
                    "nvext": {"return_token_ids": True}}
            full, _, ids = _stream_text(c.post("/v1/chat/completions", json=body).text)
            assert len(ids) == 20
            head, _, _ = _stream_text(c.post("/v1/chat/completions", json=dict(body, max_tokens=7)).text)
            r = c.post("/v1/chat/completions", json=dict(body, nvext={"return_token_ids": True,
                                                                      "resume_token_ids": ids[:7],
                                                                      "resume_text_chars": len(head)}))
            tail, reason, tids = _stream_text(r.text)
            assert tids == ids[7:] and reason == "length"
            assert head + tail == full
    finally:
        hub.shutdown()


def test_supervisor_restarts_tp_group_and_router_resumes(ckpt, tmp_path):
    """TP=2 replica (two processes, gloo): the follower rank dies mid-request, the group is torn down and
    restarted by the supervisor, and the router finishes the request on the restarted group."""
    from fastapi.testclient import TestClient

    from generativeaiexamples_amd.serving.router import create_router_app
    from generativeaiexamples_amd.serving.supervisor import ReplicaSupervisor

    args = ["--llm", "tiny-llama", "--llm-weights", ckpt, "--embedder", "", "--device", "cpu", "--dtype", "float32",
            "--no-graphs", "--max-num-seqs", "8", "--max-model-len", "512"]
    sup = ReplicaSupervisor(args, replicas=1, tp=2, base_port=_free_port(), assign_gpus=False, backoff_s=0.2,
                            env={"GAI_DIST_BACKEND": "gloo", "GAI_DIST_TIMEOUT_S": "60", "GAI_RANK_STOP_GRACE_S": "5",
                                 "OMP_NUM_THREADS": "2"},
                            first_env={0: {"FI_KILL_RANK": "1", "FI_KILL_AT_CALL": "40"}}, log_dir=str(tmp_path))
    sup.start()
    try:
        with TestClient(create_router_app(sup.urls, health_interval=0.3, requeue_timeout=180)) as rc:
            deadline = time.time() + 180
            while rc.get("/v1/health/ready").status_code != 200:
                assert time.time() < deadline, "replica never became ready"
                time.sleep(0.5)
            body = {"messages": MSGS, "max_tokens": 40, "temperature": 0, "ignore_eos": True, "stream": True,
                    "nvext": {"return_token_ids": True}}
            text, reason, ids = _stream_text(rc.post("/v1/chat/completions", json=body).text)
            assert reason == "length" and len(ids) == 40
            assert sup.reps[0].generation == 1 and sup.reps[0].exit_codes and sup.reps[0].exit_codes[0] != 0
            # the restarted group serves the same request uninterrupted: identical greedy completion
            text2, _, ids2 = _stream_text(rc.post("/v1/chat/completions", json=body).text)
            assert ids2 == ids and text2 == text
    finally:
        sup.stop()
