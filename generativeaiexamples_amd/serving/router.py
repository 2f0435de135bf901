"""Replica router: one OpenAI/NIM-compatible front over N data-parallel model-server replicas, with health
tracking and re-queue of in-flight requests when a replica fails (SURVEY §5.3 failure recovery).

The reference keeps its NIM containers alive with the orchestrator's restart policy
(RAG/examples/local_deploy/docker-compose-vectordb.yaml:90 ``restart``, nims.yaml health checks); a request
that was running inside a container that died is simply lost. Here each replica is a model server
(``python -m generativeaiexamples_amd.serving``, itself a TP group of one process per GPU) and this router:

* routes every request to the healthy replica with the fewest requests in flight;
* polls ``/v1/health/ready`` and marks a replica down on a failed poll, a refused connection, a 5xx, an
  in-band stream error or a stream that ends before ``[DONE]`` - a replica whose engine watchdog fired or
  whose TP peer died drops out of routing at once, and comes back when its health poll passes again
  (serving/supervisor.py restarts dead replicas);
* re-queues in-flight chat completions: upstream calls always stream with ``nvext.return_token_ids``, so
  the router knows every token the client already has; on failure it re-issues the request to another
  (or the restarted) replica with ``nvext.resume_token_ids`` / ``resume_text_chars``, the replica appends
  those tokens to the prompt and continues - the client sees one uninterrupted stream (for greedy
  decoding, token-identical to a run without the failure);
* retries idempotent calls (completions that have not streamed yet, embeddings, ranking) on another
  replica.

``python -m generativeaiexamples_amd.serving.router --upstream http://h:8001 --upstream http://h:8002`` fronts
existing servers; ``--replicas R --tp T -- <server args>`` also starts and supervises them.
"""
from __future__ import annotations

import asyncio
import json
import logging
import time
import uuid
from dataclasses import dataclass
from typing import Any, AsyncIterator, Dict, List, Optional

import httpx
from fastapi import FastAPI, Request
from fastapi.responses import JSONResponse, Response, StreamingResponse

from prometheus_client import CollectorRegistry, Counter, Gauge, generate_latest

log = logging.getLogger(__name__)


@dataclass
class Replica:
    url: str
    healthy: bool = False
    in_flight: int = 0
    failures: int = 0
    last_change: float = 0.0

    def set(self, ok: bool, why: str = ""):
        if ok != self.healthy:
            self.last_change = time.time()
            log.warning("replica %s is %s%s", self.url, "up" if ok else "DOWN", f" ({why})" if why else "")
        self.healthy = ok
        if not ok:
            self.failures += 1


class UpstreamFailure(Exception):
    pass


class Router:
    def __init__(self, urls: List[str], health_interval: float = 1.0, requeue_timeout: float = 120.0,
                 max_attempts: int = 8, request_timeout: float = 600.0):
        self.replicas = [Replica(u.rstrip("/")) for u in urls]
        self.health_interval = health_interval
        self.requeue_timeout = requeue_timeout
        self.max_attempts = max_attempts
        self.client = httpx.AsyncClient(timeout=httpx.Timeout(request_timeout, connect=5.0))
        self._task: Optional[asyncio.Task] = None
        self._changed = asyncio.Event()
        reg = self.registry = CollectorRegistry()
        self.m_requeued = Counter("gai_router_requeued_total", "in-flight requests re-issued after a failure",
                                  registry=reg)
        self.m_failures = Counter("gai_router_replica_failures_total", "replica failures seen by the router",
                                  registry=reg)
        self.m_healthy = Gauge("gai_router_healthy_replicas", "replicas currently routable", registry=reg)
        self.m_requests = Counter("gai_router_requests_total", "requests routed", registry=reg)

    # ---------------------------------------------------------------- health
    async def check(self, r: Replica):
        try:
            resp = await self.client.get(r.url + "/v1/health/ready", timeout=2.0)
            ok = resp.status_code == 200
        except httpx.HTTPError as e:
            ok, resp = False, e
        self._mark(r, ok, "" if ok else f"health: {getattr(resp, 'status_code', resp)!s}")

    def _mark(self, r: Replica, ok: bool, why: str = ""):
        was = r.healthy
        r.set(ok, why)
        if was and not ok:
            self.m_failures.inc()
        self.m_healthy.set(sum(x.healthy for x in self.replicas))
        if ok and not was:
            self._changed.set()

    async def _health_loop(self):
        while True:
            await asyncio.gather(*(self.check(r) for r in self.replicas))
            await asyncio.sleep(self.health_interval)

    async def start(self):
        await asyncio.gather(*(self.check(r) for r in self.replicas))
        self._task = asyncio.create_task(self._health_loop())

    async def stop(self):
        if self._task:
            self._task.cancel()
        await self.client.aclose()

    async def pick(self, exclude: Optional[Replica] = None) -> Replica:
        """Healthy replica with the fewest requests in flight; waits (up to requeue_timeout) for one."""
        deadline = time.monotonic() + self.requeue_timeout
        while True:
            live = [r for r in self.replicas if r.healthy]
            if exclude is not None and len(live) > 1:
                live = [r for r in live if r is not exclude] or live
            if live:
                return min(live, key=lambda r: r.in_flight)
            left = deadline - time.monotonic()
            if left <= 0:
                raise UpstreamFailure("no healthy replica")
            self._changed.clear()
            try:
                await asyncio.wait_for(self._changed.wait(), timeout=min(left, self.health_interval))
            except asyncio.TimeoutError:
                await asyncio.gather(*(self.check(r) for r in self.replicas))

    # ---------------------------------------------------------------- chat with resume
    async def chat_events(self, body: Dict[str, Any]) -> AsyncIterator[Dict[str, Any]]:
        """Upstream chat chunks (dicts) of one logical completion, across replica failures."""
        tokens: List[int] = []
        sent_chars = 0
        max_tokens = body.get("max_completion_tokens") or body.get("max_tokens")
        client_ids = bool((body.get("nvext") or {}).get("return_token_ids"))
        attempt, last = 0, None
        while True:
            attempt += 1
            if attempt > self.max_attempts:
                raise UpstreamFailure(f"gave up after {self.max_attempts} attempts")
            rep = await self.pick(exclude=last)
            up = dict(body, stream=True)
            up.pop("max_completion_tokens", None)
            nv = dict(up.get("nvext") or {}, return_token_ids=True)
            if tokens:
                nv.update(resume_token_ids=tokens, resume_text_chars=sent_chars)
                if max_tokens is not None:
                    up["max_tokens"] = int(max_tokens)  # the replica subtracts the resumed tokens
            elif max_tokens is not None:
                up["max_tokens"] = int(max_tokens)
            up["nvext"] = nv
            rep.in_flight += 1
            done = False
            try:
                async with self.client.stream("POST", rep.url + "/v1/chat/completions", json=up) as resp:
                    if resp.status_code >= 500:
                        raise UpstreamFailure(f"HTTP {resp.status_code}")
                    if resp.status_code != 200:  # client error: not the replica's fault, pass it through
                        err = json.loads(await resp.aread() or b"{}")
                        yield {"__status__": resp.status_code, "body": err}
                        return
                    async for line in resp.aiter_lines():
                        if not line.startswith("data: "):
                            continue
                        data = line[6:]
                        if data == "[DONE]":
                            done = True
                            break
                        obj = json.loads(data)
                        if "error" in obj:
                            raise UpstreamFailure(str(obj["error"]))
                        ids = (obj.pop("nvext", None) or {}).get("token_ids", [])
                        tokens.extend(ids)
                        for ch in obj.get("choices", []):
                            sent_chars += len((ch.get("delta") or {}).get("content") or "")
                        if obj.get("usage"):  # counts of this replica's part only: report the whole completion
                            u = obj["usage"]
                            u["completion_tokens"] = len(tokens)
                            u["total_tokens"] = u.get("prompt_tokens", 0) + len(tokens)
                        if client_ids and ids:
                            obj["nvext"] = {"token_ids": ids}
                        yield obj
                if not done:
                    raise UpstreamFailure("stream ended before [DONE]")
                return
            except (UpstreamFailure, httpx.HTTPError, json.JSONDecodeError) as e:
                self._mark(rep, False, f"chat: {e}")
                self.m_requeued.inc()
                last = rep
                log.warning("re-queueing chat completion after %d tokens (%s)", len(tokens), e)
            finally:
                rep.in_flight -= 1

    async def forward(self, path: str, body: Dict[str, Any]) -> Response:
        """Idempotent POST, retried on another replica when one fails."""
        last = None
        for _ in range(self.max_attempts):
            rep = await self.pick(exclude=last)
            rep.in_flight += 1
            try:
                resp = await self.client.post(rep.url + path, json=body)
                if resp.status_code >= 500:
                    raise UpstreamFailure(f"HTTP {resp.status_code}")
                return Response(resp.content, status_code=resp.status_code,
                                media_type=resp.headers.get("content-type", "application/json"))
            except (UpstreamFailure, httpx.HTTPError) as e:
                self._mark(rep, False, f"{path}: {e}")
                self.m_requeued.inc()
                last = rep
            finally:
                rep.in_flight -= 1
        raise UpstreamFailure(f"gave up after {self.max_attempts} attempts")


def _err(status: int, msg: str):
    return JSONResponse(status_code=status, content={"error": {"message": msg, "type": "router_error", "code": status},
                                                     "object": "error", "message": msg})


def create_router_app(urls: List[str], **kw) -> FastAPI:
    router = Router(urls, **kw)
    app = FastAPI(title="generativeaiexamples_amd replica router")
    app.state.router = router

    @app.on_event("startup")
    async def _start():
        await router.start()

    @app.on_event("shutdown")
    async def _stop():
        await router.stop()

    @app.get("/v1/health/ready")
    async def ready():
        if not any(r.healthy for r in router.replicas):
            return JSONResponse(status_code=503, content={"object": "health.response", "message": "No ready replica."})
        return {"object": "health.response", "message": "Service is ready."}

    @app.get("/v1/health/live")
    async def live():
        return {"object": "health.response", "message": "Service is live."}

    @app.get("/v1/replicas")
    async def replicas():
        return {"data": [{"url": r.url, "healthy": r.healthy, "in_flight": r.in_flight, "failures": r.failures}
                         for r in router.replicas]}

    @app.get("/metrics")
    async def metrics():
        return Response(generate_latest(router.registry), media_type="text/plain; version=0.0.4")

    @app.get("/v1/models")
    async def models():
        try:
            rep = await router.pick()
            resp = await router.client.get(rep.url + "/v1/models")
            return Response(resp.content, status_code=resp.status_code, media_type="application/json")
        except (UpstreamFailure, httpx.HTTPError) as e:
            return _err(503, str(e))

    @app.post("/v1/chat/completions")
    async def chat(request: Request):
        body = await request.json()
        router.m_requests.inc()
        stream = bool(body.get("stream"))
        if not stream:
            body = dict(body, stream_options={"include_usage": True})
        rid = f"chatcmpl-{uuid.uuid4().hex}"
        events = router.chat_events(body)
        try:
            first = await events.__anext__()
        except StopAsyncIteration:
            return _err(502, "empty upstream response")
        except UpstreamFailure as e:
            return _err(503, str(e))
        if "__status__" in first:
            return JSONResponse(status_code=first["__status__"], content=first["body"])

        async def chunks():
            yield first
            async for ev in events:
                yield ev

        if stream:
            async def sse():
                role_sent = False
                try:
                    async for ev in chunks():
                        ev["id"] = rid
                        for ch in ev.get("choices", []):
                            if "role" in (ch.get("delta") or {}):
                                if role_sent:  # a resumed stream starts with its own role chunk
                                    ch["delta"].pop("role")
                                    if not ch["delta"] and not ch.get("finish_reason"):
                                        ev = None
                                        break
                                role_sent = True
                        if ev is not None:
                            yield f"data: {json.dumps(ev)}\n\n"
                except UpstreamFailure as e:
                    yield f"data: {json.dumps({'error': {'message': str(e)}})}\n\n"
                yield "data: [DONE]\n\n"

            return StreamingResponse(sse(), media_type="text/event-stream")
        # non-streaming client: assemble the message from the (resumable) upstream stream
        text, reason, usage, ntok, msg, model, created = [], None, None, 0, None, body.get("model"), int(time.time())
        try:
            async for ev in chunks():
                model, created = ev.get("model", model), ev.get("created", created)
                if ev.get("usage"):
                    usage = ev["usage"]
                for ch in ev.get("choices", []):
                    d = ch.get("delta") or {}
                    if d.get("tool_calls") is not None:
                        msg = d
                    if d.get("content"):
                        text.append(d["content"])
                    if ch.get("finish_reason"):
                        reason = ch["finish_reason"]
                ntok += len((ev.get("nvext") or {}).get("token_ids", []))
        except UpstreamFailure as e:
            return _err(503, str(e))
        if msg is None or msg.get("tool_calls") is None:
            msg = {"role": "assistant", "content": "".join(text)}
        out = {"id": rid, "object": "chat.completion", "created": created, "model": model,
               "choices": [{"index": 0, "message": msg, "logprobs": None, "finish_reason": reason}]}
        if usage:
            out["usage"] = usage
        return out

    async def _fwd(path: str, request: Request):
        body = await request.json()
        router.m_requests.inc()
        if path == "/v1/completions" and body.get("stream"):
            body = dict(body, stream=False)  # buffered through the router so it can be retried
            try:
                resp = await router.forward(path, body)
            except UpstreamFailure as e:
                return _err(503, str(e))
            if resp.status_code != 200:
                return resp
            j = json.loads(resp.body)

            async def sse():
                for ch in j.get("choices", []):
                    yield f"data: {json.dumps(dict(j, choices=[ch]))}\n\n"
                yield "data: [DONE]\n\n"

            return StreamingResponse(sse(), media_type="text/event-stream")
        try:
            return await router.forward(path, body)
        except UpstreamFailure as e:
            return _err(503, str(e))

    def _route(path: str):
        async def handler(request: Request):
            return await _fwd(path, request)

        return handler

    for p in ("/v1/completions", "/v1/embeddings", "/v1/ranking", "/v1/retrieval/nvidia/reranking"):
        app.post(p)(_route(p))
    return app


def main():
    import argparse

    import uvicorn

    ap = argparse.ArgumentParser(description="replica router (+ optional supervisor of the replicas)")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8000)
    ap.add_argument("--upstream", action="append", default=[], help="URL of an existing model server (repeat)")
    ap.add_argument("--replicas", type=int, default=0, help="start and supervise this many model servers")
    ap.add_argument("--tp", type=int, default=1, help="tensor-parallel degree of each supervised replica")
    ap.add_argument("--base-port", type=int, default=8001)
    ap.add_argument("--health-interval", type=float, default=1.0)
    ap.add_argument("--requeue-timeout", type=float, default=300.0)
    ap.add_argument("server_args", nargs=argparse.REMAINDER, help="-- then model-server arguments")
    a = ap.parse_args()
    logging.basicConfig(level=logging.INFO)
    sup = None
    urls = list(a.upstream)
    if a.replicas:
        from .supervisor import ReplicaSupervisor

        args = a.server_args[1:] if a.server_args[:1] == ["--"] else a.server_args
        sup = ReplicaSupervisor(args, replicas=a.replicas, tp=a.tp, base_port=a.base_port)
        sup.start()
        urls += sup.urls
    if not urls:
        ap.error("give --upstream URLs and/or --replicas N")
    try:
        uvicorn.run(create_router_app(urls, health_interval=a.health_interval, requeue_timeout=a.requeue_timeout),
                    host=a.host, port=a.port, log_level="info")
    finally:
        if sup is not None:
            sup.stop()


if __name__ == "__main__":
    main()
