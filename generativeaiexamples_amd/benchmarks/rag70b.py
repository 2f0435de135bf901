"""BASELINE config 3: Llama-3-70B generator tensor-parallel over the ranks (RCCL all-reduce over xGMI)
+ cross-encoder reranking of the top-40 + a 10M-vector index sharded over the ranks (reference
analogue: multi_turn_rag retrieves 40 and reranks to 4, multi_turn_rag/chains.py:147,177-191; the
70B NIM uses all GPUs, docker-compose-nim-ms.yaml:20).

All ranks form ONE serving instance (strong scaling of a fixed global batch):
  * queries are split over the ranks for the e5-large-v2 embedding (embedder DP);
  * every rank scans its 10M/N shard for all queries (fused similarity top-k kernel), candidates
    are all-gathered and merged (index DP);
  * each rank reranks the 40 candidates of its own queries (reranker DP) and the top-4 ids are
    all-gathered, so every rank builds the same prompts;
  * the 70B generator runs TP=N as ONE engine: rank 0 owns the scheduler and the requests and publishes
    every step plan; ranks 1..N-1 execute the plans (LLMEngine.follow, parallel/step_channel.py).
On one MI355X (TP=1) the whole 141 GB bf16 model plus a 20 GB index shard fits in its 288 GB.
"""
from __future__ import annotations

import os
import time

import torch

from .common import gather_list, log, median, percentile, timed_steps

METRIC = "end-to-end RAG queries/sec + p50 TTFT, Llama-3-70B TP + rerank top-40 + 10M sharded index"


def add_args(ap):
    ap.add_argument("--rag70b-model", default="llama3-70b", choices=["llama3-70b", "tiny"])
    ap.add_argument("--reranker", default="nv-rerankqa-mistral-4b",
                    help="reranker preset (models.registry.RERANKER_PRESETS)")
    ap.add_argument("--retrieve-k", type=int, default=40)
    ap.add_argument("--total-index", type=int, default=10_000_000, help="vectors over all shards")


def tp_size(args) -> int:
    return int(os.environ.get("WORLD_SIZE", "1"))


def run(args, ctx) -> dict:
    from ..engine import EngineConfig, LLMEngine, SamplingParams
    from ..engine.embedder import Embedder
    from ..engine.tokenizer import apply_chat_template, bert_byte_tokenizer, llama3_byte_tokenizer, small_byte_tokenizer
    from ..index.hbm_index import HBMIndex
    from ..index.sharded import ShardedIndex
    from ..models.bert import BertConfig, BertModel
    from ..models.llama import LlamaConfig, LlamaModel
    from ..models.registry import build_reranker_service
    from ..rag import synthetic
    from ..rag.prompts import RAG_TEMPLATE, rag_user_message

    dev, rank, world = ctx.device, ctx.rank, ctx.world_size
    tiny = args.rag70b_model == "tiny"
    gbatch = args.batch or 32
    shard = (args.index_size or args.total_index) // (1 if args.index_size else world)
    t_setup = time.perf_counter()
    lcfg = LlamaConfig.tiny(max_position=8192) if tiny else LlamaConfig.llama3_70b()
    llm = LlamaModel(lcfg, device=dev, dist_ctx=ctx).random_init(seed=31)
    tok = small_byte_tokenizer(lcfg.vocab_size) if tiny else llama3_byte_tokenizer(lcfg.vocab_size)
    bcfg = BertConfig.tiny() if tiny else BertConfig.e5_large_v2()
    emb = Embedder(BertModel(bcfg, device=dev).random_init(seed=32), bert_byte_tokenizer(bcfg.vocab_size))
    rr, rr_name = build_reranker_service("tiny-reranker" if tiny else args.reranker, device=dev, seed=33)
    index = HBMIndex(bcfg.hidden_size, "cosine", device=dev, capacity=shard)
    ct = args.chunk_tokens
    index.add_random(shard, seed=700 + rank, doc_fn=lambda r: synthetic.chunk_document(r, ct))
    sharded = ShardedIndex(index, max_queries=(gbatch + world - 1) // world)  # per-rank share of the batch
    log(f"models ready: {lcfg.name} TP={world} ({llm.num_params() / 1e9:.1f}B params/rank), {rr_name}, "
        f"index {shard} x {bcfg.hidden_size} per rank ({shard * world} total)")
    sample_ctx = "\n\n".join(synthetic.chunk_document(r, ct).page_content for r in range(args.top_k))
    prompt_est = int(len(apply_chat_template([{"role": "system", "content": RAG_TEMPLATE}, {
        "role": "user", "content": rag_user_message(sample_ctx, synthetic.question(0))}], tok)) * 1.25) + 64
    ecfg = EngineConfig(max_num_seqs=gbatch, max_batched_tokens=args.max_batched_tokens,
                        max_model_len=min(lcfg.max_position, prompt_est + args.max_tokens),
                        prefill_chunk=args.max_batched_tokens, use_graphs=not args.no_graphs, prefix_cache=False,
                        kv_memory_fraction=0.6, kv_memory_bytes=int(args.kv_gb * (1 << 30)) if args.kv_gb else None)
    engine = LLMEngine(llm, tok, ecfg)
    if not args.no_graphs:
        engine.capture_graphs(max_bs=gbatch)
    log(f"engine ready: {engine.kv.num_blocks} KV blocks, setup {time.perf_counter() - t_setup:.1f}s")
    params = SamplingParams(temperature=0.2, top_p=0.7, max_tokens=args.max_tokens, ignore_eos=True)

    def doc(g):
        s, r = ShardedIndex.split_row(g) if world > 1 else (0, g)
        return synthetic.chunk_document(r, ct)  # documents are a function of (shard-local) row id

    def step(i: int) -> dict:
        t0 = time.perf_counter()
        qs = [synthetic.question(i * gbatch + j) for j in range(gbatch)]
        mine = list(range(rank, gbatch, world))
        e = emb.embed([qs[j] for j in mine], "query")
        _, rows = sharded.search_raw(e.to(index.dtype), args.retrieve_k)
        rows = rows.cpu().tolist()
        cands = [[g for g in cand if g >= 0] for cand in rows]
        all_scores = rr.score_many([(qs[j], [doc(g).page_content for g in c]) for j, c in zip(mine, cands)])
        top = {}
        for j, cand, scores in zip(mine, cands, all_scores):
            order = sorted(range(len(cand)), key=lambda k: -scores[k])[: args.top_k]
            top[j] = [cand[k] for k in order]
        if world > 1:
            merged = {}
            for part in ctx.all_gather_obj(top):
                merged.update(part)
            top = merged
        t_ret = time.perf_counter() - t0
        if not engine.leader:  # TP follower: execute rank 0's step plans until it yields
            assert engine.follow() == "yield"
            return dict(ttft=[], tokens=0, retrieval_s=t_ret, prompt=0.0)
        reqs = []
        for j, q in enumerate(qs):
            context = "\n\n".join(doc(g).page_content for g in top[j])
            msgs = [{"role": "system", "content": RAG_TEMPLATE}, {"role": "user", "content": rag_user_message(context, q)}]
            reqs.append(engine.add_request(apply_chat_template(msgs, tok), params, request_id=f"s{i}-q{j}"))
        while engine.has_work():
            engine.step()
        engine.release_followers()
        assert all(len(r.output_ids) == args.max_tokens for r in reqs), "a query was cut short"
        return dict(ttft=[r.first_token_time - t0 for r in reqs], tokens=sum(len(r.output_ids) for r in reqs),
                    retrieval_s=t_ret, prompt=sum(len(r.prompt_ids) for r in reqs) / len(reqs))

    total, stats = timed_steps(ctx, step, args.steps, args.warmup)
    ttft = [x for s in stats for x in s["ttft"]]  # rank 0 (the TP leader) owns the requests
    toks = sum(s["tokens"] for s in stats)
    nq = gbatch * args.steps
    return {
        "metric": METRIC, "value": round(nq / total, 4), "unit": "queries/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(1000 * total / args.steps, 2), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic (random-init weights of the named architectures; synthetic 506-token chunk corpus and "
                "questions; EOS ignored)",
        "config": {"model": f"{lcfg.name} + {bcfg.name} + {rr_name} + {shard * world}-vector index",
                   "global_batch": gbatch, "seq_len": int(median([s["prompt"] for s in stats])) + args.max_tokens,
                   "parallelism": f"tp{world} (generator) / dp{world} (embed, index, rerank)",
                   "retrieve_k": args.retrieve_k, "top_k": args.top_k, "max_tokens": args.max_tokens},
        "p50_ttft_s": round(percentile(ttft, 0.5), 4), "p90_ttft_s": round(percentile(ttft, 0.9), 4),
        "output_tokens_per_s": round(toks / total, 1),
        "retrieval_rerank_ms": round(1000 * median([s["retrieval_s"] for s in stats]), 2),
    }
