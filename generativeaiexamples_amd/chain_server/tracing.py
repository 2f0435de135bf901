"""Distributed tracing hooks (parity with RAG/src/chain_server/tracing.py and the OTel callback handlers
of RAG/tools/observability).

* Off by default; ``ENABLE_TRACING=true`` turns it on. Spans carry W3C ``traceparent`` context:
  incoming request headers are extracted (so playground -> chain-server traces join) and outgoing
  HTTP calls get the header injected.
* With ``opentelemetry`` installed spans go to its SDK (OTLP exporter to
  ``OTEL_EXPORTER_OTLP_ENDPOINT``); without it (this image) a built-in tracer records spans and
  exports them as OTLP/HTTP JSON to the same endpoint, or to a JSONL file
  (``GAI_TRACE_FILE``), so Jaeger / the collector pipeline of the reference still receive them.
* Engine-internal spans (queue wait, retrieval, first token) and ``first_token_time_ms`` (TTFT,
  the reference's opentelemetry_callback.py:230-245,282) are recorded by the pipelines.
"""
from __future__ import annotations

import contextvars
import functools
import json
import logging
import os
import random
import threading
import time
from contextlib import contextmanager
from typing import Any, Dict, Iterator, List, Optional

log = logging.getLogger(__name__)
ENABLED = os.environ.get("ENABLE_TRACING", "false").lower() == "true"
SERVICE = os.environ.get("OTEL_SERVICE_NAME", "chain-server")

_current: contextvars.ContextVar = contextvars.ContextVar("gai_span", default=None)


class Span:
    __slots__ = ("name", "trace_id", "span_id", "parent_id", "start", "end", "attributes", "events")

    def __init__(self, name: str, trace_id: str, parent_id: Optional[str]):
        self.name, self.trace_id, self.parent_id = name, trace_id, parent_id
        self.span_id = "%016x" % random.getrandbits(64)
        self.start, self.end = time.time_ns(), None
        self.attributes: Dict[str, Any] = {}
        self.events: List[dict] = []

    def set_attribute(self, k: str, v: Any):
        self.attributes[k] = v if isinstance(v, (int, float, bool, str)) else str(v)

    def add_event(self, name: str, attrs: Optional[dict] = None):
        self.events.append({"name": name, "time": time.time_ns(), "attributes": attrs or {}})

    @property
    def traceparent(self) -> str:
        return f"00-{self.trace_id}-{self.span_id}-01"

    def to_otlp(self) -> dict:
        def av(v):
            if isinstance(v, bool):
                return {"boolValue": v}
            if isinstance(v, int):
                return {"intValue": str(v)}
            if isinstance(v, float):
                return {"doubleValue": v}
            return {"stringValue": str(v)}

        return {"traceId": self.trace_id, "spanId": self.span_id, "parentSpanId": self.parent_id or "",
                "name": self.name, "kind": 1, "startTimeUnixNano": str(self.start),
                "endTimeUnixNano": str(self.end or time.time_ns()),
                "attributes": [{"key": k, "value": av(v)} for k, v in self.attributes.items()],
                "events": [{"name": e["name"], "timeUnixNano": str(e["time"]),
                            "attributes": [{"key": k, "value": av(v)} for k, v in e["attributes"].items()]}
                           for e in self.events]}


class _Exporter:
    def __init__(self):
        self.buf: List[Span] = []
        self.lock = threading.Lock()
        self.file = os.environ.get("GAI_TRACE_FILE")
        ep = os.environ.get("OTEL_EXPORTER_OTLP_ENDPOINT", "")
        self.http = (ep.rstrip("/") + "/v1/traces") if ep.startswith("http") else None

    def export(self, span: Span):
        with self.lock:
            self.buf.append(span)
            if len(self.buf) >= 32:
                self.flush_locked()

    def flush_locked(self):
        spans, self.buf = self.buf, []
        if not spans:
            return
        payload = {"resourceSpans": [{"resource": {"attributes": [
            {"key": "service.name", "value": {"stringValue": SERVICE}}]},
            "scopeSpans": [{"scope": {"name": "generativeaiexamples_amd"}, "spans": [s.to_otlp() for s in spans]}]}]}
        if self.file:
            with open(self.file, "a") as f:
                f.write(json.dumps(payload) + "\n")
        if self.http:
            try:
                import httpx

                httpx.post(self.http, json=payload, timeout=2.0)
            except Exception as e:  # tracing must never break serving
                log.debug("trace export failed: %s", e)

    def flush(self):
        with self.lock:
            self.flush_locked()


EXPORTER = _Exporter()


def extract(headers) -> Optional[tuple]:
    tp = headers.get("traceparent") if headers is not None else None
    if not tp:
        return None
    parts = tp.split("-")
    if len(parts) == 4 and len(parts[1]) == 32:
        return parts[1], parts[2]
    return None


@contextmanager
def span(name: str, headers=None, **attrs) -> Iterator[Optional[Span]]:
    if not ENABLED:
        yield None
        return
    parent = _current.get()
    remote = extract(headers) if parent is None else None
    if parent is not None:
        s = Span(name, parent.trace_id, parent.span_id)
    elif remote:
        s = Span(name, remote[0], remote[1])
    else:
        s = Span(name, "%032x" % random.getrandbits(128), None)
    for k, v in attrs.items():
        s.set_attribute(k, v)
    tok = _current.set(s)
    try:
        yield s
    finally:
        s.end = time.time_ns()
        _process_metrics(s)
        _current.reset(tok)
        EXPORTER.export(s)


_PROC = None


def _process_metrics(s: "Span"):
    """psutil process metrics at span end (the reference's LangChain callback records them, T5)."""
    global _PROC
    try:
        import psutil
        _PROC = _PROC or psutil.Process()
        s.set_attribute("process.memory.rss_bytes", int(_PROC.memory_info().rss))
        s.set_attribute("process.cpu.percent", float(_PROC.cpu_percent(None)))
        s.set_attribute("process.threads", int(_PROC.num_threads()))
    except Exception:  # noqa: BLE001 - metrics are best-effort
        pass


def inject(headers: dict) -> dict:
    s = _current.get()
    if s is not None:
        headers["traceparent"] = s.traceparent
    return headers


def instrumentation_wrapper(func):
    """Route decorator: opens a span per request, joining the caller's W3C trace context."""

    @functools.wraps(func)
    async def wrapper(*args, **kwargs):
        req = kwargs.get("request")
        with span(func.__name__, getattr(req, "headers", None)):
            return await func(*args, **kwargs)

    return wrapper


def traced(kind: str):
    """Decorator for component calls (callback-handler role, T5/T6): one span per call named
    ``<kind>.<function>`` with the call's scalar kwargs as attributes; result-size attribute when the
    result is a sized collection (retrieved documents, embeddings)."""

    def deco(func):
        @functools.wraps(func)
        def wrapper(*args, **kwargs):
            if not ENABLED:
                return func(*args, **kwargs)
            attrs = {f"{kind}.{k}": v for k, v in kwargs.items() if isinstance(v, (int, float, str, bool))}
            with span(f"{kind}.{func.__name__}", **attrs) as sp:
                out = func(*args, **kwargs)
                if sp is not None and hasattr(out, "__len__"):
                    sp.set_attribute(f"{kind}.result_count", len(out))
                    if kind == "retriever" and out and isinstance(out[0], tuple):
                        sp.set_attribute("retriever.scores", [float(x[1]) for x in out][:16])
                return out
        return wrapper
    return deco


async def traced_astream(name: str, it, **attrs):
    """Async twin of :func:`traced_stream` for streams iterated with ``async for``."""
    if not ENABLED:
        async for chunk in it:
            yield chunk
        return
    with span(name, **attrs) as s:
        t0, n = time.perf_counter(), 0
        async for chunk in it:
            if n == 0 and s is not None:
                s.set_attribute("first_token_time_ms", (time.perf_counter() - t0) * 1000.0)
            n += 1
            yield chunk
        if s is not None:
            s.set_attribute("completion_chunks", n)


def traced_stream(name: str, it: Iterator[str], **attrs) -> Iterator[str]:
    """Wraps a token stream; records first_token_time_ms (TTFT) and the token count."""
    if not ENABLED:
        yield from it
        return
    with span(name, **attrs) as s:
        t0, n = time.perf_counter(), 0
        for chunk in it:
            if n == 0 and s is not None:
                s.set_attribute("first_token_time_ms", (time.perf_counter() - t0) * 1000.0)
            n += 1
            yield chunk
        if s is not None:
            s.set_attribute("completion_chunks", n)
