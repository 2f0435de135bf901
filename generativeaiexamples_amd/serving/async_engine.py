"""Asynchronous front of the generator engine for HTTP serving.

A single background thread owns the GPU and runs ``LLMEngine.step()`` whenever there is work;
HTTP handlers only enqueue requests and await per-request ``asyncio.Queue`` s that the engine
thread feeds through ``loop.call_soon_threadsafe``. The event loop therefore never blocks on
GPU work (fixes the reference's event-loop blocking), and a client
disconnect aborts its request (frees its KV blocks) immediately.
"""
from __future__ import annotations

import asyncio
import collections
import concurrent.futures
import faulthandler
import logging
import os
import sys
import threading
import time
import uuid
from dataclasses import dataclass
from typing import AsyncIterator, Dict, Iterator, List, Optional

from ..engine.llm_engine import LLMEngine, RequestOutput
from ..engine.sampling import SamplingParams
from ..utils.metrics import METRICS
from ..utils.streams import RETRIEVAL_GATE


@dataclass
class StreamItem:
    delta: str
    token_id: int
    finished: bool
    finish_reason: Optional[str]


log = logging.getLogger(__name__)


def _settle(fut: concurrent.futures.Future, res=None, exc: Optional[BaseException] = None) -> None:
    """Complete ``fut`` unless it is already done (cancelled by its awaiting task): never raises."""
    try:
        if exc is not None:
            fut.set_exception(exc)
        else:
            fut.set_result(res)
    except concurrent.futures.InvalidStateError:
        pass


class AsyncLLMEngine:
    """``watchdog_s`` (env GAI_WATCHDOG_S, default 300): a step running longer than this (hung kernel or
    collective) marks the engine unhealthy - /v1/health/ready turns 503 so a router drains it - dumps
    every thread's stack and fails the waiting requests instead of leaving clients hanging."""

    def __init__(self, engine: LLMEngine, watchdog_s: Optional[float] = None):
        self.engine = engine
        self.queues: Dict[str, tuple] = {}
        self.cv = threading.Condition()
        self.running = True
        self.healthy = True
        self.error: Optional[BaseException] = None
        self.watchdog_s = watchdog_s if watchdog_s is not None else float(os.environ.get("GAI_WATCHDOG_S", "300"))
        self.admission_wait_s = float(os.environ.get("GAI_ADMISSION_WAIT_MS", "25")) / 1000.0
        self._step_started: Optional[float] = None
        self._hung = False  # the watchdog fired on the running step: nothing reaches the engine thread now
        # (request id, generated tokens, finish reason) of recently finished requests (benchmarks, tests)
        self.completed: collections.deque = collections.deque(maxlen=4096)
        # per finished streamed request, perf_counter timestamps (CLOCK_MONOTONIC: comparable across processes):
        # submit (generate() entered), first_token (engine sampled it), first_yield (first item handed to the
        # caller); the served benchmark splits client TTFT into retrieval / queue+prefill / delivery
        self.timings: collections.deque = collections.deque(maxlen=4096)
        self.inbox: collections.deque = collections.deque()  # (fn, args, kwargs, future) run between steps
        self._stop = threading.Event()
        self.thread = threading.Thread(target=self._loop, daemon=True, name="llm-engine")
        self.thread.start()
        self.watchdog = threading.Thread(target=self._watch, daemon=True, name="llm-watchdog")
        self.watchdog.start()

    def _fail_all(self, e: BaseException, inbox: bool = False):
        for rid, (loop, q) in list(self.queues.items()):
            loop.call_soon_threadsafe(q.put_nowait, e)
        self.queues.clear()
        if inbox:  # a hung step never drains the inbox: fail the admissions waiting in it too
            with self.cv:
                pending, self.inbox = list(self.inbox), collections.deque()
            for _, _, _, fut in pending:
                _settle(fut, exc=e)

    def _watch(self):
        period = max(0.05, min(1.0, self.watchdog_s / 4))
        while not self._stop.wait(period):
            t = self._step_started
            if t is not None and self.healthy and time.perf_counter() - t > self.watchdog_s:
                err = TimeoutError(f"engine step exceeded the {self.watchdog_s:.1f}s watchdog")
                self.error, self.healthy, self._hung = err, False, True
                log.error("%s; dumping thread stacks", err)
                faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
                self._fail_all(err, inbox=True)

    @property
    def tokenizer(self):
        return self.engine.tok

    def _call(self, fn, *args, **kw) -> concurrent.futures.Future:
        """Run ``fn`` on the engine thread between steps. Request admission and aborts go through here: the
        engine holds its lock for a whole step (a prefill chunk waits ~0.2 s on the GPU), and an event-loop
        thread blocked on that lock stalls every open SSE stream (served first-frame delay 0.5 s p50)."""
        fut: concurrent.futures.Future = concurrent.futures.Future()
        if self._hung:  # the engine thread is stuck in a step: fail now instead of waiting forever
            _settle(fut, exc=self.error or RuntimeError("engine step hung"))
            return fut
        with self.cv:
            self.inbox.append((fn, args, kw, fut))
            self.cv.notify()
        return fut

    def _drain(self):
        while True:
            with self.cv:
                if not self.inbox:
                    return
                fn, args, kw, fut = self.inbox.popleft()
            # a caller that went away (asyncio cancellation of the wrapped future) is skipped, never half-applied
            if not fut.set_running_or_notify_cancel():
                continue
            try:
                res = fn(*args, **kw)
            except BaseException as e:  # noqa: BLE001 - delivered to the caller
                _settle(fut, exc=e)
            else:
                _settle(fut, res=res)

    def _loop(self):
        eng = self.engine
        while self.running:
            with self.cv:
                while self.running and not self.inbox and not eng.has_work():
                    self.cv.wait(0.05)
            if not self.running:
                break
            self._safe_drain()
            if not eng.has_work():
                continue
            self._admission_wait(eng)
            self._safe_drain()  # requests that arrived during the wait join this step
            try:
                t0 = self._step_started = time.perf_counter()
                outs = eng.step()
                self._step_started = None
                self._hung = False
                METRICS.observe_step(time.perf_counter() - t0, len(outs), eng)
            except BaseException as e:  # engine failure: fail every pending request, keep serving health
                self._step_started = None
                self.error, self.healthy = e, False
                self._fail_all(e)
                continue
            for o in outs:
                ent = self.queues.get(o.request_id)
                if ent is None:
                    continue
                loop, q = ent
                loop.call_soon_threadsafe(q.put_nowait, o)
                if o.finished:
                    self.queues.pop(o.request_id, None)

    def _safe_drain(self):
        try:
            self._drain()
        except BaseException:  # noqa: BLE001 - one bad inbox item must not end the engine thread
            log.exception("engine inbox item failed")

    def _admission_wait(self, eng) -> None:
        """Before a step that would only start prefill for newly queued prompts (nothing running, nothing in
        flight), give query-path work still pending in this process (utils.streams.RETRIEVAL_GATE) up to
        ``admission_wait_s`` (env GAI_ADMISSION_WAIT_MS, default 25) to finish, so concurrent arrivals share
        that prefill. Never delays decode steps of running sequences."""
        if self.admission_wait_s <= 0 or not RETRIEVAL_GATE.busy():
            return
        sched = getattr(eng, "sched", None)
        if sched is None or getattr(eng, "_pending", None) is not None or sched.num_running() > 0:
            return
        RETRIEVAL_GATE.wait_idle(self.admission_wait_s)

    async def generate(self, prompt_ids: List[int], params: SamplingParams,
                       request_id: Optional[str] = None, images: Optional[list] = None,
                       lora: Optional[str] = None) -> AsyncIterator[StreamItem]:
        rid = request_id or f"cmpl-{uuid.uuid4().hex}"
        loop = asyncio.get_running_loop()
        q: asyncio.Queue = asyncio.Queue()
        self.queues[rid] = (loop, q)
        t0 = time.perf_counter()
        first = True
        try:
            req = await asyncio.wrap_future(self._call(self.engine.add_request, prompt_ids, params, rid, images=images,
                                                       lora=lora))
        except BaseException:
            self.queues.pop(rid, None)
            raise
        METRICS.requests_total.inc()
        METRICS.prompt_tokens.inc(len(prompt_ids))
        if req.finished:  # zero-budget request
            self.queues.pop(rid, None)
            yield StreamItem("", -1, True, req.finish_reason)
            return
        t_yield = None
        try:
            while True:
                o = await q.get()
                if isinstance(o, BaseException):
                    raise RuntimeError(f"engine failure: {o!r}")
                assert isinstance(o, RequestOutput)
                if first:
                    t_yield = time.perf_counter()
                    METRICS.ttft.observe(t_yield - t0)
                    first = False
                METRICS.generation_tokens.inc()
                yield StreamItem(o.delta, o.token_id, o.finished, o.finish_reason)
                if o.finished:
                    METRICS.e2e.observe(time.perf_counter() - t0)
                    self.completed.append((rid, len(req.output_ids), o.finish_reason))
                    self.timings.append({"submit": t0, "first_token": req.first_token_time, "first_yield": t_yield})
                    return
        finally:
            if rid in self.queues:  # client went away or error: free the sequence now (on the engine thread)
                self.queues.pop(rid, None)
                self._call(self.engine.abort, rid)

    def generate_sync(self, prompt_ids: List[int], params: SamplingParams,
                      request_id: Optional[str] = None, images: Optional[list] = None) -> Iterator[StreamItem]:
        """Blocking streaming API for worker threads (chain-server example pipelines)."""
        import queue as _q

        rid = request_id or f"cmpl-{uuid.uuid4().hex}"
        q: _q.Queue = _q.Queue()

        class _Shim:  # duck-types the (loop, queue) pair used by the engine thread
            @staticmethod
            def call_soon_threadsafe(fn, item):
                q.put(item)

        self.queues[rid] = (_Shim, q)
        t0 = time.perf_counter()
        try:
            req = self._call(self.engine.add_request, prompt_ids, params, rid, images=images).result()
        except BaseException:
            self.queues.pop(rid, None)
            raise
        METRICS.requests_total.inc()
        if req.finished:
            self.queues.pop(rid, None)
            yield StreamItem("", -1, True, req.finish_reason)
            return
        first = True
        try:
            while True:
                o = q.get()
                if isinstance(o, BaseException):
                    raise RuntimeError(f"engine failure: {o!r}")
                if first:
                    METRICS.ttft.observe(time.perf_counter() - t0)
                    first = False
                yield StreamItem(o.delta, o.token_id, o.finished, o.finish_reason)
                if o.finished:
                    self.completed.append((rid, len(req.output_ids), o.finish_reason))
                    return
        finally:
            if rid in self.queues:
                self.queues.pop(rid, None)
                self._call(self.engine.abort, rid)

    async def complete(self, prompt_ids: List[int], params: SamplingParams, request_id: Optional[str] = None,
                       images: Optional[list] = None, lora: Optional[str] = None):
        text, ids, reason = [], [], None
        async for it in self.generate(prompt_ids, params, request_id, images, lora):
            text.append(it.delta)
            if it.token_id >= 0:
                ids.append(it.token_id)
            reason = it.finish_reason
        return "".join(text), ids, reason

    def shutdown(self):
        self.running = False
        with self.cv:
            pending, self.inbox = list(self.inbox), collections.deque()
            self.cv.notify_all()
        for _, _, _, fut in pending:
            _settle(fut, exc=RuntimeError("engine shut down"))
        self._stop.set()
        with self.cv:
            self.cv.notify_all()
        self.thread.join(timeout=30)
        self.watchdog.join(timeout=5)
