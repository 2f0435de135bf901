#!/usr/bin/env python
"""Headline benchmark: end-to-end RAG queries/sec + p50 TTFT (BASELINE.json config 2 on every GPU).

Per GPU: Llama-3-8B bf16 generator (TP=1, random-init weights of the real architecture),
e5-large-v2 bf16 embedder (random-init), and a 1M x 1024 exact HBM vector index shard over a
synthetic corpus of 506-token chunks. One timed *step* = one wave of ``--batch`` concurrent RAG
queries per GPU through the whole query path of the reference's basic_rag chain
(RAG/examples/basic_rag/langchain/chains.py rag_chain):

  query -> e5 "query: " embedding (all-gathered across ranks: embedder DP)
        -> exact top-4 search of every shard (candidates all-gathered + merged: index DP, RCCL)
        -> prompt = rag_template + "Context: <4 chunks>\n\nQuestion: <q>" (Llama-3 chat format)
        -> continuous-batching generation, temperature 0.2 / top_p 0.7, max_tokens 256 (the
           reference evaluation tool's generation settings, llm_answer_generator.py:63).

value = total queries/s over all ranks (weak scaling: --batch queries per GPU per step).
TTFT = query arrival (step start) -> first generated token, per query; p50/p90 reported.
vs_baseline: the reference publishes no RAG queries/s for any configuration, so the field is
null. Its only per-query figures are the single-stream L40S estimates of its sizing calculator (BASELINE.md row 2:
TTFT 0.062 s + 249 x 18.5 ms TPOT = 4.67 s per query = 0.2141 queries/s). The like-for-like comparison is
therefore single stream against single stream: ``vs_baseline_single_stream`` = our c1 rate (1 / (c1 TTFT + 255 x
c1 TPOT), from the untimed probes) / 0.2141. ``batch_vs_single_stream_baseline`` keeps the old ratio (64-way batch
throughput over the single-stream estimate) for context only.

Launch: ``python bench.py --gpus N`` spawns N ranks itself (one process per GPU, RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_ADDR=127.0.0.1 set before any GPU call) unless it already runs under torchrun.

Retrieval workload: random-init e5 embeddings of different questions are ~0.99 cosine-similar, so a
random index returns the same chunks for every query. Before each step (untimed) the bench therefore
*plants* 4 rows per query of that step (its embedding + 2% noise) at hashed row ids and restores them to
random vectors afterwards: every query retrieves 4 chunks of its own through the full 1M-row scan,
as a real corpus would (``unique_chunks_retrieved`` = 4 x queries).

After the timed steps (untimed, reported alongside): ``p50_ttft_c1_s`` - 8 queries one at a time, TTFT
from query arrival to first token; and an open-loop run (Poisson arrivals at 0.8x the measured rate,
``poisson``), both on the rank-local index shard. ``retrieval_breakdown_ms`` splits the per-step query
path into embed / scan / prompt build / tokenize / add_request.

Notes: the KV prefix cache is off (every query prefills its full prompt); score_threshold is disabled (random-init embeddings give near-zero cosine to a random
index; thresholding would drop every chunk); EOS is ignored so every query generates exactly
max_tokens (fixed work per step).
"""
from __future__ import annotations

import argparse
import json
import os
import random
import statistics
import sys
import time

import torch

METRIC = "end-to-end RAG queries/sec + p50 TTFT, Llama-3-8B gen + e5-large embed"
BASELINE_QPS = 1.0 / (0.062 + 249 * 0.0185)  # BASELINE.md row 2 (L40S, single stream)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", type=int, default=2, choices=[2, 3, 4, 5],
                    help="BASELINE.json config: 2 = headline (default), 3 = 70B TP + rerank + 10M sharded index, "
                         "4 = multimodal CLIP + Llama-3.2-Vision fp8, 5 = agentic Mixtral tool loop")
    ap.add_argument("--batch", type=int, default=None, help="concurrent queries per GPU per step (default 64)")
    ap.add_argument("--max-tokens", type=int, default=256)
    ap.add_argument("--top-k", type=int, default=4)
    ap.add_argument("--chunk-tokens", type=int, default=506)
    ap.add_argument("--index-size", type=int, default=None, help="vectors per GPU shard (default 1M)")
    ap.add_argument("--model", default="llama3-8b", choices=["llama3-8b", "tiny"])
    ap.add_argument("--embedder", default="e5-large-v2", choices=["e5-large-v2", "e5-base-v2", "tiny"])
    ap.add_argument("--max-batched-tokens", type=int, default=16384)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--decode-steps", type=int, default=8,
                    help="decode tokens per captured multi-step HIP graph run (1 = one host round trip per token)")
    ap.add_argument("--prefix-cache", action="store_true",
                    help="enable KV prefix caching (off by default: random-init embeddings retrieve the same "
                         "chunks for every query, so caching would skip most of the prefill work)")
    ap.add_argument("--kv-gb", type=float, default=None, help="KV-cache size per rank (default: 50%% of free HBM)")
    ap.add_argument("--kv-cache-dtype", default="auto", choices=["auto", "fp8"],
                    help="fp8 = OCP e4m3fn KV cache (an option, not the headline configuration: the JSON line "
                         "reports it in config.kv_cache_dtype)")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--no-plant", action="store_true", help="do not plant per-query relevant chunks")
    ap.add_argument("--no-probes", action="store_true", help="skip the untimed c1 / open-loop TTFT probes")
    ap.add_argument("--probe-c1", type=int, default=4,
                    help="queries of the concurrency-1 probe (each runs its full max_tokens: TTFT and TPOT)")
    ap.add_argument("--served-steps", type=int, default=3,
                    help="after the timed in-process steps (config 2): this many POST /generate waves through the chain "
                         "server, reported as the 'served' sub-object (0: skip)")
    ap.add_argument("--served", action="store_true",
                    help="drive the chain server instead of the engine: every query is a concurrent POST /generate "
                         "SSE stream (basic_rag example, in-process engines), TTFT measured at the client")
    from generativeaiexamples_amd.benchmarks import CONFIGS, module
    for c in CONFIGS:
        module(c).add_args(ap)
    return ap.parse_args()


def _sync():
    """Device barrier of the timed region (a no-op on the CPU rehearsal path: gloo ranks, tiny models)."""
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


def run_other_config(args):
    """Configs 3-5: generativeaiexamples_amd.benchmarks.<module>.run, same JSON contract."""
    from generativeaiexamples_amd.benchmarks import module
    from generativeaiexamples_amd.parallel.dist import init_distributed

    mod = module(args.config)
    ctx = init_distributed(tp_size=mod.tp_size(args) if hasattr(mod, "tp_size") else 1)
    torch.manual_seed(1234 + ctx.rank)
    out = mod.run(args, ctx)
    if ctx.rank == 0:
        print(json.dumps(out), flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                json.dump(out, f)
    if ctx.world_size > 1:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


def run_probes(args, embedder, index, engine, build_requests, plant, unplant, new_phase, qps_per_rank):
    """c1 TTFT / TPOT and open-loop Poisson TTFT (untimed). Every query: embed -> local 1M scan -> prompt ->
    engine; TTFT = scheduled arrival -> first token; TPOT = (finish - first token) / (tokens - 1)."""
    rank = int(os.environ.get("RANK", "0"))

    def retrieve(qids):
        qs = [synthetic_question(q) for q in qids]
        e = embedder.embed(qs, input_type="query")
        _, rows = index.search_raw(e, args.top_k)
        return build_requests(qs, rows.cpu().tolist(), new_phase())

    # concurrency 1: each query runs its full max_tokens (TTFT and per-token latency of a lone stream)
    c1, tpot, c1_ret = [], [], []
    base = 900_000 + 1000 * rank
    for i in range(args.probe_c1):
        qid = base + i
        planted = plant([qid], [synthetic_question(qid)])
        _sync()
        t0 = time.perf_counter()
        req = retrieve([qid])[0]
        c1_ret.append(time.perf_counter() - t0)  # embed + scan + prompt + add_request (host clock, not synced)
        while engine.has_work():
            engine.step()
        c1.append(req.first_token_time - t0)
        n = len(req.output_ids)
        if n > 1:
            tpot.append((req.finish_time - req.first_token_time) / (n - 1))
        unplant(planted)
    # open loop: Poisson arrivals at 0.8x the measured per-rank burst rate
    rate = 0.8 * qps_per_rank
    rng = random.Random(4242 + rank)
    n = args.batch
    arrivals, t = [], 0.0
    for _ in range(n):
        t += rng.expovariate(rate)
        arrivals.append(t)
    qids = [base + 500 + i for i in range(n)]
    planted = plant(qids, [synthetic_question(q) for q in qids])
    _sync()
    t0 = time.perf_counter()
    reqs, nxt = [], 0
    while nxt < n or engine.has_work():
        now = time.perf_counter() - t0
        due = []
        while nxt < n and arrivals[nxt] <= now:
            due.append(nxt)
            nxt += 1
        if due:
            for i, r in zip(due, retrieve([qids[i] for i in due])):
                reqs.append((arrivals[i], r))
        if engine.has_work():
            engine.step()
        elif nxt < n:
            time.sleep(max(0.0, min(0.002, arrivals[nxt] - (time.perf_counter() - t0))))
    span = time.perf_counter() - t0
    unplant(planted)
    tt = sorted(r.first_token_time - t0 - a for a, r in reqs)
    tp = statistics.median(tpot) if tpot else float("nan")
    return {"p50_ttft_c1_s": round(statistics.median(c1), 4), "ttft_c1_s": [round(x, 4) for x in c1],
            "ttft_c1_retrieve_ms": round(1000 * statistics.median(c1_ret), 2),
            "tpot_c1_ms": round(1000 * tp, 3), "decode_tok_s_c1": round(1.0 / tp, 1) if tpot else None,
            "poisson": {"rate_qps_per_gpu": round(rate, 3), "queries": n, "achieved_qps_per_gpu": round(n / span, 3),
                        "p50_ttft_s": round(tt[len(tt) // 2], 4),
                        "p90_ttft_s": round(tt[min(len(tt) - 1, int(0.9 * len(tt)))], 4)}}


def synthetic_question(q: int) -> str:
    from generativeaiexamples_amd.rag import synthetic
    return synthetic.question(q)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        from generativeaiexamples_amd.parallel.launch import spawn_ranks

        sys.exit(spawn_ranks(args.gpus))
    if (args.served or args.served_steps > 0) and args.config == 2:
        # the HTTP clients run in their own process, spawned before this one touches the GPU
        from generativeaiexamples_amd.benchmarks import served_client

        served_client.start()
    if args.config != 2:
        return run_other_config(args)
    args.batch = args.batch or 64
    args.index_size = args.index_size or 1_000_000
    from generativeaiexamples_amd.engine import EngineConfig, LLMEngine, SamplingParams
    from generativeaiexamples_amd.engine.embedder import Embedder
    from generativeaiexamples_amd.engine.tokenizer import (apply_chat_template, bert_byte_tokenizer,
                                                           llama3_byte_tokenizer, small_byte_tokenizer)
    from generativeaiexamples_amd.index.hbm_index import HBMIndex
    from generativeaiexamples_amd.index.sharded import ShardedIndex
    from generativeaiexamples_amd.models import LlamaConfig, LlamaModel
    from generativeaiexamples_amd.models.bert import BertConfig, BertModel
    from generativeaiexamples_amd.parallel.dist import init_distributed
    from generativeaiexamples_amd.rag import synthetic
    from generativeaiexamples_amd.rag.prompts import RAG_TEMPLATE, rag_user_message

    ctx = init_distributed(tp_size=1)
    dev = ctx.device
    rank, world = ctx.rank, ctx.world_size
    torch.manual_seed(1234 + rank)
    t_setup = time.perf_counter()

    # ---------------- models
    if args.model == "llama3-8b":
        lcfg = LlamaConfig.llama3_8b()
        ltok = llama3_byte_tokenizer(lcfg.vocab_size)
    else:
        lcfg = LlamaConfig.tiny(max_position=8192)
        ltok = small_byte_tokenizer(lcfg.vocab_size)
    llm = LlamaModel(lcfg, device=dev).random_init(seed=1)
    if args.embedder == "e5-large-v2":
        bcfg = BertConfig.e5_large_v2()
    elif args.embedder == "e5-base-v2":
        bcfg = BertConfig.e5_base_v2()
    else:
        bcfg = BertConfig.tiny()
    enc = BertModel(bcfg, device=dev).random_init(seed=2)
    embedder = Embedder(enc, bert_byte_tokenizer(bcfg.vocab_size))
    embedder.capture_graphs()  # every query-encoder bucket before any timed or served work
    log(f"models ready: {lcfg.name} {llm.num_params() / 1e9:.2f}B params, {bcfg.name}")

    # ---------------- index shard (1M x dim per GPU, synthetic documents on demand)
    index = HBMIndex(bcfg.hidden_size, "cosine", device=dev, capacity=args.index_size)
    ct = args.chunk_tokens
    index.add_random(args.index_size, seed=100 + rank, doc_fn=lambda r: synthetic.chunk_document(r, ct))
    sharded = ShardedIndex(index, max_queries=args.batch)  # every rank embeds args.batch queries per step: sync-free
    log(f"index ready: {args.index_size} x {bcfg.hidden_size} per shard, {world} shard(s)")

    # ---------------- engine
    # size max_model_len from a real prompt of this pipeline (+25% slack for longer questions) so no
    # request is ever cut short: every query must generate exactly max_tokens
    sample_ctx = "\n\n".join(synthetic.chunk_document(r, args.chunk_tokens).page_content for r in range(args.top_k))
    sample = apply_chat_template([{"role": "system", "content": RAG_TEMPLATE},
                                  {"role": "user", "content": rag_user_message(sample_ctx, synthetic.question(0))}], ltok)
    prompt_est = int(len(sample) * 1.25) + 64
    ecfg = EngineConfig(max_num_seqs=max(args.batch, 1), max_batched_tokens=args.max_batched_tokens,
                        max_model_len=min(lcfg.max_position, prompt_est + args.max_tokens),
                        prefill_chunk=args.max_batched_tokens, use_graphs=not args.no_graphs,
                        decode_steps=args.decode_steps,
                        prefix_cache=args.prefix_cache,
                        kv_memory_fraction=0.5,
                        kv_memory_bytes=int(args.kv_gb * (1 << 30)) if args.kv_gb else None,
                        kv_cache_dtype=args.kv_cache_dtype)
    engine = LLMEngine(llm, ltok, ecfg)
    if not args.no_graphs:
        engine.capture_graphs(max_bs=args.batch)
    log(f"engine ready: {engine.kv.num_blocks} KV blocks ({engine.kv.nbytes / 2**30:.1f} GiB), "
        f"graphs={sorted(engine.graphs)} setup {time.perf_counter() - t_setup:.1f}s")

    params = SamplingParams(temperature=0.2, top_p=0.7, max_tokens=args.max_tokens, ignore_eos=True)
    doc_of = lambda g: index.document(ShardedIndex.split_row(g)[1]) if world > 1 else index.document(g)  # noqa

    # ---------------- per-query relevant chunks (see module docstring)
    N = args.index_size
    gen = torch.Generator(device=dev)
    gen.manual_seed(77 + rank)

    def plant_rows(qid: int):
        return [(qid * 2654435761 + j * 40503 + 12345) % N for j in range(args.top_k)]

    def plant(qids, questions):
        if args.no_plant:
            return []
        e = embedder.embed(questions, input_type="query").float()
        e = torch.nn.functional.normalize(e, dim=-1)
        rows = [r for q in qids for r in plant_rows(q)]
        v = e.repeat_interleave(args.top_k, 0)
        v = v + 0.02 * torch.randn(v.shape, device=v.device, generator=gen) / (v.shape[1] ** 0.5)
        index.set_vectors(rows, v)
        return rows

    def unplant(rows):
        if rows:
            r = torch.randn(len(rows), index.dim, device=dev, generator=gen)
            index.set_vectors(rows, r)

    def build_requests(questions, rows, phase):
        """rows: retrieved global row ids per query -> engine requests (timed by phase)."""
        t = time.perf_counter()
        texts = []
        for qi, q in enumerate(questions):
            docs = [doc_of(g) for g in rows[qi] if g >= 0]
            texts.append(rag_user_message("\n\n".join(d.page_content for d in docs), q))
        t1 = time.perf_counter()
        prompts = [apply_chat_template([{"role": "system", "content": RAG_TEMPLATE},
                                        {"role": "user", "content": u}], ltok) for u in texts]
        t2 = time.perf_counter()
        reqs = [engine.add_request(pr, params) for pr in prompts]
        t3 = time.perf_counter()
        phase["prompt_build"] += t1 - t
        phase["tokenize"] += t2 - t1
        phase["add_request"] += t3 - t2
        return reqs

    def run_step(step_idx: int, phase: dict):
        qids = [(step_idx * world + rank) * args.batch + i for i in range(args.batch)]
        questions = [synthetic.question(q) for q in qids]
        planted = plant(qids, questions)
        ctx.barrier()
        _sync()
        t0 = time.perf_counter()
        emb = embedder.embed(questions, input_type="query")
        _sync()
        t_e = time.perf_counter()
        rel, rows = sharded.search_raw(emb, args.top_k)
        rows = rows.cpu().tolist()
        t_s = time.perf_counter()
        phase["embed"] += t_e - t0
        phase["scan"] += t_s - t_e
        uniq.update(g for r in rows for g in r)
        reqs = build_requests(questions, rows, phase)
        t_retrieved = time.perf_counter()
        while engine.has_work():
            engine.step()
        _sync()
        ctx.barrier()
        t1 = time.perf_counter()
        t_first = max(r.first_token_time for r in reqs)  # every prompt prefilled (its first token sampled)
        phase["prefill_wall"] += t_first - t_retrieved
        phase["decode_wall"] += t1 - t_first
        unplant(planted)
        ttft = [r.first_token_time - t0 for r in reqs]
        ntok = sum(len(r.output_ids) for r in reqs)
        short = [len(r.output_ids) for r in reqs if len(r.output_ids) != args.max_tokens]
        assert not short, f"{len(short)} queries generated != max_tokens ({short[:4]}): work would be skipped"
        plen = statistics.mean(len(r.prompt_ids) for r in reqs)
        return t1 - t0, ttft, ntok, plen, t_retrieved - t0

    def new_phase():
        return dict(embed=0.0, scan=0.0, prompt_build=0.0, tokenize=0.0, add_request=0.0, prefill_wall=0.0,
                    decode_wall=0.0)

    if args.served:
        from generativeaiexamples_amd.benchmarks.served import run_served

        out = run_served(args, ctx, dict(lcfg=lcfg, bcfg=bcfg, embedder=embedder, index=index, engine=engine,
                                         plant=plant, unplant=unplant, metric=METRIC, baseline_qps=BASELINE_QPS))
        if rank == 0:
            print(json.dumps(out), flush=True)
            if args.json_out:
                with open(args.json_out, "w") as f:
                    json.dump(out, f)
        if world > 1:
            torch.distributed.barrier()
            torch.distributed.destroy_process_group()
        return

    uniq = set()
    for w in range(args.warmup):
        dt, *_ = run_step(10_000 + w, new_phase())
        log(f"warmup {w}: {dt:.2f}s")
    uniq = set()
    phase = new_phase()
    engine.phase_ms.clear()  # GAI_STEP_TIMING=1: synchronised per-phase engine wall time of the timed steps
    stats0 = dict(engine.stats)
    times, ttfts, toks, plens, rtimes = [], [], 0, [], []
    for s in range(args.steps):
        dt, ttft, ntok, plen, rt = run_step(s, phase)
        times.append(dt)
        ttfts += ttft
        toks += ntok
        plens.append(plen)
        rtimes.append(rt)
        log(f"step {s}: {dt:.3f}s  p50 TTFT {statistics.median(ttft):.3f}s  retrieval {rt * 1000:.1f} ms")

    stats1, phase1 = dict(engine.stats), dict(engine.phase_ms)  # the timed steps only (before the probes)
    if engine.host_timeline:  # GAI_HOST_TIMELINE=1: host gaps of the pipelined decode, last timed step
        tl = engine.host_timeline
        ch = sorted(e - s for n, s, e in tl if n == "chain")
        co = sorted(e - s for n, s, e in tl if n == "complete")
        gaps = sorted(tl[i + 1][1] - tl[i][2] for i in range(len(tl) - 1))
        log(f"host timeline: {len(ch)} chained launches median {1e3 * ch[len(ch) // 2]:.2f} ms max "
            f"{1e3 * ch[-1]:.2f}; complete median {1e3 * co[len(co) // 2]:.2f} ms; between calls median "
            f"{1e3 * gaps[len(gaps) // 2]:.3f} ms max {1e3 * gaps[-1]:.3f}; nochain {sum(n == 'nochain' for n, _, _ in tl)}")
    # ---------------- untimed TTFT probes on the rank-local shard (no collectives: ranks run them freely)
    probes = {}
    if not args.no_probes:
        probes = run_probes(args, embedder, index, engine, build_requests, plant, unplant, new_phase,
                            args.batch * args.steps * world / max(1e-9, max(ctx.all_gather_obj(sum(times)))) / world)
        log(f"probes: {probes}")

    total = sum(times)
    # max over ranks
    if world > 1:
        total = max(ctx.all_gather_obj(total))  # slowest rank defines the step time
        allt = ctx.all_gather_obj(ttfts)
        ttfts = [x for part in allt for x in part]
        toks = int(sum(ctx.all_gather_obj(toks)))
    nq = args.batch * args.steps * world
    qps = nq / total
    ttfts.sort()
    p50 = ttfts[len(ttfts) // 2]
    p90 = ttfts[min(len(ttfts) - 1, int(0.9 * len(ttfts)))]
    out = {
        "metric": METRIC,
        "value": round(qps, 4),
        "unit": "queries/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000 * total / args.steps, 2),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,  # no published RAG queries/s; see vs_baseline_single_stream
        "dtype": "bf16",
        "data": "synthetic (random-init weights of the named architectures; synthetic 506-token chunk corpus "
                "and questions; score_threshold off, EOS ignored)",
        "config": {
            "model": f"{lcfg.name} + {bcfg.name} + {args.index_size}-vector exact HBM index per GPU",
            "global_batch": args.batch * world,
            "seq_len": int(statistics.mean(plens)) + args.max_tokens,
            "parallelism": f"dp{world}",
            "prompt_tokens": int(statistics.mean(plens)),
            "max_tokens": args.max_tokens,
            "top_k": args.top_k,
            "kv_cache_dtype": "bf16" if args.kv_cache_dtype == "auto" else "fp8_e4m3",
            # decode projections stored once, fragment-ordered (EngineConfig.weight_layout; GAI_WEIGHT_LAYOUT overrides)
            "weight_layout": os.environ.get("GAI_WEIGHT_LAYOUT", "fragment"),
        },
        "p50_ttft_s": round(p50, 4),
        "p90_ttft_s": round(p90, 4),
        "output_tokens_per_s": round(toks / total, 1),
        "tokens_per_query": args.max_tokens,
        "retrieval_ms": round(1000 * statistics.mean(rtimes), 2),
        "unique_chunks_retrieved": len(uniq),
        "prefix_cache": bool(args.prefix_cache),
        "baseline_qps_single_stream_l40s": round(BASELINE_QPS, 4),
        "batch_vs_single_stream_baseline": round(qps / BASELINE_QPS, 3),
        "retrieval_breakdown_ms": {k: round(1000 * v / max(1, args.steps), 2) for k, v in phase.items()
                                   if not k.endswith("_wall")},
        # wall time per step from retrieval done to the last prompt's first token, then to the last token
        "phase_ms": {k[:-5]: round(1000 * v / max(1, args.steps), 1) for k, v in phase.items() if k.endswith("_wall")},
        "planted_chunks": not args.no_plant,
        "engine_steps_per_step": {k: round((stats1[k] - stats0.get(k, 0)) / max(1, args.steps), 1)
                                  for k in ("steps", "multi_step_runs", "chained_runs", "graph_steps")
                                  if k in stats1},
        **probes,
    }
    if probes.get("p50_ttft_c1_s") and probes.get("tpot_c1_ms"):
        c1_s = probes["p50_ttft_c1_s"] + (args.max_tokens - 1) * probes["tpot_c1_ms"] / 1000.0
        out["single_stream_qps"] = round(1.0 / c1_s, 4)
        out["vs_baseline_single_stream"] = round(out["single_stream_qps"] / BASELINE_QPS, 3)
    if phase1:
        out["engine_phase_ms_per_step"] = {k: round(v / max(1, args.steps), 1) for k, v in phase1.items()}
    if args.served_steps > 0:
        # after the timed in-process steps (untimed for the headline): the same workload through the product path,
        # POST /generate SSE from a separate client process, TTFT at the client (BASELINE.md protocol)
        import copy

        from generativeaiexamples_amd.benchmarks.served import run_served

        sargs = copy.copy(args)
        sargs.steps, sargs.warmup = args.served_steps, 1
        srv = run_served(sargs, ctx, dict(lcfg=lcfg, bcfg=bcfg, embedder=embedder, index=index, engine=engine,
                                          plant=plant, unplant=unplant, metric=METRIC, baseline_qps=BASELINE_QPS))
        out["served"] = {k: srv[k] for k in ("value", "p50_ttft_s", "p90_ttft_s", "ms_per_step", "steps", "warmup",
                                             "ttft_split_p50_ms", "p50_ttft_c1_s", "tpot_c1_ms", "poisson")
                         if k in srv}
        out["served"]["path"] = "POST /generate SSE (chain server, basic_rag), client process, TTFT at the client"
        out["served"]["vs_in_process"] = round(srv["value"] / qps, 4)
        log(f"served: {out['served']}")
    if rank == 0:
        print(json.dumps(out), flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                json.dump(out, f)
    if world > 1:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
