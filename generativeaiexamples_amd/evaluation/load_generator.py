"""Concurrent streaming load generator (the reference's API-client notebook measures tokens/s but never
increments its counter; this one measures).

Targets: the chain server (``POST /generate`` SSE frames with ``data: `` prefix) or any /v1 server
(``POST /v1/chat/completions`` with ``stream: true``). ``--concurrency`` client threads each loop over
questions until ``--requests`` complete; reports QPS, TTFT and inter-token latency percentiles and
streamed-chunks/s. ``python -m generativeaiexamples_amd.evaluation.load_generator --help``.
"""
from __future__ import annotations

import argparse
import json
import statistics
import threading
import time
from typing import Dict, List, Optional

import httpx


def _pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * len(xs)))] if xs else float("nan")


def one_request(http: httpx.Client, url: str, mode: str, question: str, max_tokens: int, model: str,
                use_kb: bool) -> Dict:
    if mode == "chain":
        body = {"messages": [{"role": "user", "content": question}], "use_knowledge_base": use_kb,
                "temperature": 0.2, "top_p": 0.7, "max_tokens": max_tokens}
        path = "/generate"
    else:
        body = {"model": model, "messages": [{"role": "user", "content": question}], "temperature": 0.2,
                "top_p": 0.7, "max_tokens": max_tokens, "stream": True}
        path = "/v1/chat/completions"
    t0 = time.perf_counter()
    stamps: List[float] = []
    with http.stream("POST", url + path, json=body) as r:
        r.raise_for_status()
        for line in r.iter_lines():
            if not line.startswith("data: ") or line == "data: [DONE]":
                continue
            fr = json.loads(line[6:])
            ch = (fr.get("choices") or [{}])[0]
            txt = (ch.get("message") or ch.get("delta") or {}).get("content")
            if txt:
                stamps.append(time.perf_counter())
    t1 = time.perf_counter()
    itl = [b - a for a, b in zip(stamps, stamps[1:])]
    return {"ttft": (stamps[0] - t0) if stamps else t1 - t0, "e2e": t1 - t0, "chunks": len(stamps), "itl": itl}


def run_load(url: str, mode: str = "chain", concurrency: int = 8, requests: int = 64, max_tokens: int = 256,
             model: str = "meta/llama3-8b-instruct", use_kb: bool = True, http: Optional[httpx.Client] = None,
             questions: Optional[List[str]] = None) -> Dict:
    from ..rag.synthetic import question
    qs = questions or [question(i) for i in range(requests)]
    url = url.rstrip("/")
    if not url.startswith("http"):
        url = "http://" + url
    results: List[Dict] = []
    lock = threading.Lock()
    counter = iter(range(requests))
    errors = []

    def worker():
        cl = http or httpx.Client(timeout=600)
        while True:
            with lock:
                i = next(counter, None)
            if i is None:
                return
            try:
                res = one_request(cl, url, mode, qs[i % len(qs)], max_tokens, model, use_kb)
                with lock:
                    results.append(res)
            except Exception as e:  # keep measuring; report the failure count
                with lock:
                    errors.append(repr(e))

    t0 = time.perf_counter()
    th = [threading.Thread(target=worker) for _ in range(concurrency)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    wall = time.perf_counter() - t0
    ttft = [r["ttft"] for r in results]
    itl = [x for r in results for x in r["itl"]]
    return {"requests": len(results), "errors": len(errors), "concurrency": concurrency, "wall_s": round(wall, 3),
            "qps": round(len(results) / wall, 3) if wall > 0 else None,
            "chunks_per_s": round(sum(r["chunks"] for r in results) / wall, 1) if wall > 0 else None,
            "ttft_p50_s": round(_pct(ttft, 0.5), 4), "ttft_p90_s": round(_pct(ttft, 0.9), 4),
            "itl_p50_ms": round(1000 * _pct(itl, 0.5), 2), "itl_p90_ms": round(1000 * _pct(itl, 0.9), 2),
            "e2e_mean_s": round(statistics.fmean(r["e2e"] for r in results), 3) if results else None,
            "first_error": errors[0] if errors else None}


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--url", default="http://localhost:8081")
    ap.add_argument("--mode", choices=["chain", "openai"], default="chain")
    ap.add_argument("--concurrency", type=int, default=8)
    ap.add_argument("--requests", type=int, default=64)
    ap.add_argument("--max-tokens", type=int, default=256)
    ap.add_argument("--model", default="meta/llama3-8b-instruct")
    ap.add_argument("--no-kb", action="store_true")
    a = ap.parse_args()
    print(json.dumps(run_load(a.url, a.mode, a.concurrency, a.requests, a.max_tokens, a.model, not a.no_kb)))


if __name__ == "__main__":
    main()
