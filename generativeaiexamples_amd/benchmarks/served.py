"""``bench.py --served``: the headline workload (BASELINE.json config 2) through the product path.

The reference's RAG product is the chain server's ``POST /generate`` streamed as SSE
(RAG/src/chain_server/server.py:313-404), driven by its evaluation client with temperature 0.2 /
top_p 0.7 / max_tokens 256 (RAG/tools/evaluation/rag_evaluator/llm_answer_generator.py:58-66), and
BASELINE.md's protocol measures TTFT at the client. Here every rank starts the chain server in-process
(uvicorn on 127.0.0.1, ``basic_rag`` example, ``APP_LLM_MODELENGINE=mi355x``: the engines built by
bench.py behind a ServiceHub, the same 1M-vector HBM index shard as the vector store) and one step =
``--batch`` concurrent HTTP clients, released together, each streaming one ``/generate`` answer:

  client POST -> validation -> worker thread: query embed + exact scan, coalesced with the concurrent
  queries (DynamicBatcher) on the high-priority retrieval stream -> rag prompt -> AsyncLLMEngine ->
  SSE frames awaited on the event loop -> client.

The HTTP clients run in a separate process (``served_client``, spawned before the GPU is initialised),
all streams of a wave on one asyncio loop. value = queries/s over all ranks; TTFT = client send -> first
non-empty ``data:`` frame. The per-query
relevant chunks are planted exactly as in the in-process bench (untimed), score_threshold is off and EOS
is ignored (``APP_LLM_IGNOREEOS``, asserted: every answer has exactly max_tokens tokens). Untimed
probes: a concurrency-1 run (TTFT, TPOT) and an open-loop Poisson run at 0.8x the measured rate.
"""
from __future__ import annotations

import asyncio
import json
import os
import random
import socket
import statistics
import threading
import time
from typing import Dict, List

import torch

from .common import log, percentile, sync


def _dev_sync():
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def _port(rank: int) -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _client_request(http, url: str, question: str, max_tokens: int) -> Dict:
    body = {"messages": [{"role": "user", "content": question}], "use_knowledge_base": True,
            "temperature": 0.2, "top_p": 0.7, "max_tokens": max_tokens}
    t0 = time.perf_counter()
    first = None
    n = 0
    with http.stream("POST", url + "/generate", json=body) as r:
        if r.status_code != 200:
            raise RuntimeError(f"/generate returned {r.status_code}")
        for ln in r.iter_lines():
            if not ln.startswith("data: "):
                continue
            fr = json.loads(ln[6:])
            ch = fr["choices"][0]
            if ch["message"]["content"]:
                n += 1
                if first is None:
                    first = time.perf_counter()
            if ch.get("finish_reason") == "[DONE]":
                break
    t1 = time.perf_counter()
    return {"t0": t0, "ttft": (first or t1) - t0, "e2e": t1 - t0, "chunks": n}


def _start_server(port: int):
    import anyio
    import uvicorn

    from ..chain_server import server

    server.app.state.example = None
    srv = uvicorn.Server(uvicorn.Config(server.app, host="127.0.0.1", port=port, log_level="warning",
                                        timeout_keep_alive=600))

    async def main():
        # retrieval / prompt building run in worker threads; streams are awaited on the loop
        anyio.to_thread.current_default_thread_limiter().total_tokens = 256
        await srv.serve()

    th = threading.Thread(target=lambda: asyncio.run(main()), daemon=True, name="chain-server")
    th.start()
    return srv, th


def run_served(args, ctx, st: dict) -> dict:
    import logging

    import httpx

    logging.getLogger("httpx").setLevel(logging.WARNING)

    from ..chain_server import utils, vectorstore
    from ..chain_server.connectors import LocalEmbeddings
    from ..rag import synthetic
    from ..serving.hub import ServiceHub

    rank, world = ctx.rank, ctx.world_size
    engine, embedder, index = st["engine"], st["embedder"], st["index"]
    llm_name, emb_name = "meta/llama3-8b-instruct", "nvidia/nv-embedqa-e5-v5"
    env = {"APP_LLM_MODELENGINE": "mi355x", "APP_LLM_MODELNAME": llm_name, "APP_LLM_IGNOREEOS": "true",
           "APP_EMBEDDINGS_MODELENGINE": "mi355x", "APP_EMBEDDINGS_MODELNAME": emb_name,
           "APP_RETRIEVER_TOPK": str(args.top_k), "APP_RETRIEVER_SCORETHRESHOLD": "-1",
           "APP_VECTORSTORE_HYBRID": "false", "EXAMPLE_PATH": "basic_rag/langchain", "GAI_LAZY_EXAMPLE": "1",
           "COLLECTION_NAME": "vector_db"}
    os.environ.update(env)
    utils.get_config.cache_clear()
    utils.get_prompts.cache_clear()
    hub = ServiceHub()
    hub.add_llm(llm_name, engine)
    hub.add_embedder(emb_name, embedder)
    hub.default_max_tokens = args.max_tokens
    utils.set_hub(hub)
    vectorstore.reset_stores()
    store = vectorstore.get_store("vector_db", LocalEmbeddings(embedder), "cosine", device=index.device)
    store.index = index  # the bench's 1M-vector shard (synthetic 506-token chunk documents)
    aeng = hub.llm(llm_name)

    port = _port(rank)
    srv, th = _start_server(port)
    url = f"http://127.0.0.1:{port}"
    for _ in range(600):
        try:
            if httpx.get(url + "/health", timeout=2).status_code == 200:
                break
        except httpx.HTTPError:
            time.sleep(0.05)
    B = args.batch
    from .served_client import start as start_clients

    clients = start_clients()  # spawned by bench.py before the GPU was initialised

    def wave(qids: List[int], delays=None) -> tuple:
        """All streams of the wave from the client process; (wall seconds, per-request results)."""
        qs = [synthetic.question(q) for q in qids]
        n_done = len(aeng.completed)
        t0 = time.perf_counter()
        out = clients.wave(url, qs, args.max_tokens, delays)
        dt = time.perf_counter() - t0
        done = list(aeng.completed)[n_done:]
        short = [n for _, n, _ in done if n != args.max_tokens]
        assert len(done) == len(qs) and not short, f"{len(short)} answers != max_tokens ({short[:4]}): work skipped"
        return dt, out["results"]

    def step(i: int):
        qids = [(i * world + rank) * B + j for j in range(B)]
        planted = st["plant"](qids, [synthetic.question(q) for q in qids])
        sync(ctx)
        dt, res = wave(qids)
        sync(ctx)
        st["unplant"](planted)
        return dt, res

    for w in range(args.warmup):
        dt, _ = step(10_000 + w)
        log(f"served warmup {w}: {dt:.2f}s")
    times, ttfts = [], []
    # client TTFT split (medians over the timed waves, ms): send -> engine submit (HTTP + retrieval + prompt),
    # submit -> first token sampled (queue + prefill), first token -> first SSE frame read by the client
    split = {"send_to_submit": [], "submit_to_first_token": [], "first_token_to_client": []}
    for s_ in range(args.steps):
        n_t = len(aeng.timings)
        dt, res = step(s_)
        times.append(dt)
        ttfts += [r["ttft"] for r in res]
        tms = list(aeng.timings)[n_t:]
        t_send = min(r["t0"] for r in res)
        for tm in tms:
            if tm["first_token"] is not None:
                split["submit_to_first_token"].append(tm["first_token"] - tm["submit"])
        split["send_to_submit"] += [tm["submit"] - t_send for tm in tms]
        firsts = sorted(r["t_first"] for r in res if r.get("t_first"))
        toks = sorted(tm["first_token"] for tm in tms if tm["first_token"] is not None)
        split["first_token_to_client"] += [a - b for a, b in zip(firsts, toks)]  # k-th first frame vs k-th token
        log(f"served step {s_}: {dt:.3f}s p50 TTFT {statistics.median(r['ttft'] for r in res):.3f}s")
    total = sum(times)
    if world > 1:
        total = max(ctx.all_gather_obj(total))
        ttfts = [x for part in ctx.all_gather_obj(ttfts) for x in part]
    qps = B * args.steps * world / total

    probes = {}
    if not args.no_probes:
        # concurrency 1 through the server: TTFT and per-token latency of a lone stream
        c1, tpot = [], []
        for i in range(args.probe_c1):
            qid = 900_000 + 1000 * rank + i
            planted = st["plant"]([qid], [synthetic.question(qid)])
            _dev_sync()
            n0 = len(aeng.completed)
            r = wave([qid])[1][0]
            st["unplant"](planted)
            c1.append(r["ttft"])
            ntok = aeng.completed[-1][1] if len(aeng.completed) > n0 else 0
            if ntok > 1:
                tpot.append((r["e2e"] - r["ttft"]) / (ntok - 1))
        # open loop: Poisson arrivals at 0.8x the measured per-rank rate
        rate = 0.8 * qps / world
        rng = random.Random(4242 + rank)
        arr, t = [], 0.0
        for _ in range(B):
            t += rng.expovariate(rate)
            arr.append(t)
        qids = [900_000 + 1000 * rank + 500 + j for j in range(B)]
        planted = st["plant"](qids, [synthetic.question(q) for q in qids])
        _dev_sync()
        span, out = wave(qids, delays=arr)
        st["unplant"](planted)
        pt = sorted(r["ttft"] for r in out)
        probes = {"p50_ttft_c1_s": round(statistics.median(c1), 4), "ttft_c1_s": [round(x, 4) for x in c1],
                  "tpot_c1_ms": round(1000 * statistics.median(tpot), 3) if tpot else None,
                  "decode_tok_s_c1": round(1.0 / statistics.median(tpot), 1) if tpot else None,
                  "poisson": {"rate_qps_per_gpu": round(rate, 3), "queries": B,
                              "achieved_qps_per_gpu": round(B / span, 3),
                              "p50_ttft_s": round(percentile(pt, 0.5), 4), "p90_ttft_s": round(percentile(pt, 0.9), 4)}}
        log(f"served probes: {probes}")
    srv.should_exit = True
    th.join(10)
    lcfg, bcfg = st["lcfg"], st["bcfg"]
    ttfts.sort()
    return {
        "metric": st["metric"], "value": round(qps, 4), "unit": "queries/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(1000 * total / args.steps, 2), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic (random-init weights of the named architectures; synthetic 506-token chunk corpus and "
                "questions; score_threshold off, EOS ignored)",
        "config": {"model": f"{lcfg.name} + {bcfg.name} + {args.index_size}-vector exact HBM index per GPU",
                   "global_batch": B * world, "seq_len": None, "parallelism": f"dp{world}",
                   "max_tokens": args.max_tokens, "top_k": args.top_k, "path": "served: POST /generate SSE",
                   "kv_cache_dtype": "bf16" if args.kv_cache_dtype == "auto" else "fp8_e4m3"},
        "p50_ttft_s": round(percentile(ttfts, 0.5), 4), "p90_ttft_s": round(percentile(ttfts, 0.9), 4),
        "served": True, "tokens_per_query": args.max_tokens, "planted_chunks": not args.no_plant,
        "ttft_split_p50_ms": {k: round(1000 * statistics.median(v), 1) for k, v in split.items() if v},
        "baseline_qps_single_stream_l40s": round(st["baseline_qps"], 4),
        "batch_vs_single_stream_baseline": round(qps / st["baseline_qps"], 3), **probes,
    }
