"""Prometheus metrics (SURVEY §5.5 plan): TTFT / end-to-end histograms, token counters, step latency,
KV usage, embed / search / rerank latency. Exposed at ``GET /metrics`` by both servers."""
from __future__ import annotations

try:
    from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest

    _HAVE_PROM = True
except Exception:  # pragma: no cover
    _HAVE_PROM = False

_BUCKETS = (0.005, 0.01, 0.02, 0.05, 0.1, 0.2, 0.5, 1.0, 2.0, 5.0, 10.0, 30.0, 60.0)


class _Null:
    def inc(self, *a, **k):
        pass

    def observe(self, *a, **k):
        pass

    def set(self, *a, **k):
        pass

    def labels(self, *a, **k):
        return self


class Metrics:
    def __init__(self):
        if _HAVE_PROM:
            self.registry = CollectorRegistry()
            r = self.registry
            self.requests_total = Counter("gai_requests_total", "generation requests", registry=r)
            self.prompt_tokens = Counter("gai_prompt_tokens_total", "prompt tokens", registry=r)
            self.generation_tokens = Counter("gai_generation_tokens_total", "generated tokens", registry=r)
            self.ttft = Histogram("gai_ttft_seconds", "time to first token", buckets=_BUCKETS, registry=r)
            self.e2e = Histogram("gai_request_seconds", "end-to-end request latency", buckets=_BUCKETS, registry=r)
            self.step = Histogram("gai_engine_step_seconds", "engine step latency", buckets=_BUCKETS, registry=r)
            self.batch = Gauge("gai_batch_size", "sequences sampled in the last step", registry=r)
            self.kv_usage = Gauge("gai_kv_cache_usage", "fraction of KV blocks in use", registry=r)
            self.embed = Histogram("gai_embed_seconds", "embedding batch latency", buckets=_BUCKETS, registry=r)
            self.search = Histogram("gai_index_search_seconds", "vector search latency", buckets=_BUCKETS,
                                    registry=r)
            self.rerank = Histogram("gai_rerank_seconds", "rerank latency", buckets=_BUCKETS, registry=r)
            self.api_requests = Counter("api_requests_total", "HTTP API requests", ["route"], registry=r)
        else:  # pragma: no cover
            self.registry = None
            for n in ("requests_total", "prompt_tokens", "generation_tokens", "ttft", "e2e", "step", "batch",
                      "kv_usage", "embed", "search", "rerank", "api_requests"):
                setattr(self, n, _Null())

    def observe_step(self, dt: float, n: int):
        self.step.observe(dt)
        self.batch.set(n)

    def render(self) -> bytes:
        return generate_latest(self.registry) if self.registry is not None else b""


METRICS = Metrics()
