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
            self.tpot = Histogram("gai_tpot_seconds", "time per output token (decode step latency)",
                                  buckets=(0.002, 0.005, 0.01, 0.02, 0.05, 0.1, 0.2, 0.5), registry=r)
            self.prefill_tokens = Counter("gai_prefill_tokens_total", "prompt tokens prefilled", registry=r)
            self.decode_tokens = Counter("gai_decode_tokens_total", "tokens decoded", registry=r)
            self.queue = Gauge("gai_waiting_requests", "requests waiting for admission", registry=r)
            self.collective = Histogram("gai_collective_seconds", "host-observed collective latency", ["op"],
                                        buckets=(1e-5, 1e-4, 1e-3, 1e-2, 0.1, 1.0), registry=r)
            self.hbm_used = Gauge("gai_gpu_hbm_used_bytes", "HBM in use on the device (all processes)", ["gpu"],
                                  registry=r)
            self.hbm_total = Gauge("gai_gpu_hbm_total_bytes", "HBM capacity of the device", ["gpu"], registry=r)
            self.hbm_allocated = Gauge("gai_gpu_hbm_allocated_bytes", "HBM held by this process's tensors", ["gpu"],
                                       registry=r)
        else:  # pragma: no cover
            self.registry = None
            for n in ("requests_total", "prompt_tokens", "generation_tokens", "ttft", "e2e", "step", "batch",
                      "kv_usage", "embed", "search", "rerank", "api_requests", "tpot", "prefill_tokens",
                      "decode_tokens", "queue", "collective", "hbm_used", "hbm_total", "hbm_allocated"):
                setattr(self, n, _Null())

    def observe_step(self, dt: float, n: int, engine=None):
        self.step.observe(dt)
        self.batch.set(n)
        if engine is not None:  # token counters / KV usage / TPOT from the engine's running stats
            st = engine.stats
            last = getattr(engine, "_metrics_last", (0, 0))
            dp, dd = st["prefill_tokens"] - last[0], st["decode_tokens"] - last[1]
            engine._metrics_last = (st["prefill_tokens"], st["decode_tokens"])
            if dp:
                self.prefill_tokens.inc(dp)
            if dd:
                self.decode_tokens.inc(dd)
                if not dp:
                    self.tpot.observe(dt)
            try:
                sch = engine.sched
                self.kv_usage.set(1.0 - sch.num_free_blocks() / max(1, sch.num_blocks()))
                self.queue.set(sch.num_waiting())
            except Exception:  # pragma: no cover - scheduler without counters
                pass

    def update_hbm(self) -> None:
        """Per-GPU HBM gauges (used / total from the driver, allocated by this process's caching allocator)."""
        try:
            import torch

            if not torch.cuda.is_available():
                return
            for i in range(torch.cuda.device_count()):
                free, total = torch.cuda.mem_get_info(i)
                self.hbm_used.labels(gpu=str(i)).set(total - free)
                self.hbm_total.labels(gpu=str(i)).set(total)
                self.hbm_allocated.labels(gpu=str(i)).set(torch.cuda.memory_allocated(i))
        except Exception:  # pragma: no cover - device query failures never break /metrics
            pass

    def render(self) -> bytes:
        self.update_hbm()
        return generate_latest(self.registry) if self.registry is not None else b""


METRICS = Metrics()
