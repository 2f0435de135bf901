"""BASELINE config 5: agentic multi-turn RAG on Mixtral-8x7B (MoE grouped GEMM) with a tool-calling loop
(reference analogues: query_decomposition_rag agent loop; W11 tool-call loop).

Per GPU (data parallel replicas; Mixtral-8x7B is 94 GB bf16 and fits one 288 GB MI355X):
  one timed step = ``--batch`` conversations, each running the loop
    turn 1 (plan): system prompt with the ``search_knowledge_base`` tool schema + the user question ->
      generate up to ``--plan-tokens`` tokens (a tool call);
    tool: the call is parsed (random-init weights never emit valid JSON, so the question itself is
      used as the tool query - fixed work per step) -> e5-large-v2 query embedding -> exact top-4
      search of a 1M-vector HBM index;
    turn 2 (answer): the whole history (system, user, assistant tool call, tool result with the four
      506-token chunks) -> generate ``--max-tokens`` tokens.
  Turns of all conversations are batched by the continuous-batching engine; EOS is ignored.
value = total conversations/s over all ranks; TTFT = step start -> first token of the final answer.
"""
from __future__ import annotations

import json
import time

import torch

from .common import gather_list, log, median, percentile, timed_steps

METRIC = "agentic multi-turn RAG conversations/sec, Mixtral-8x7B tool-calling loop + e5-large retrieval"

TOOL = {"type": "function", "function": {
    "name": "search_knowledge_base", "description": "Search the document store for passages relevant to a query.",
    "parameters": {"type": "object", "properties": {"query": {"type": "string"}}, "required": ["query"]}}}


def add_args(ap):
    ap.add_argument("--agent-model", default="mixtral-8x7b", choices=["mixtral-8x7b", "tiny-moe"])
    ap.add_argument("--plan-tokens", type=int, default=64)
    ap.add_argument("--ep", action="store_true",
                    help="expert parallelism over the ranks: data-parallel attention + experts sharded with all-to-all "
                         "token exchange and lockstep steps (default: one full Mixtral replica per GPU - it fits "
                         "one 288 GB MI355X, so replicas need no collective at all)")


def run(args, ctx) -> dict:
    from ..engine import EngineConfig, LLMEngine, SamplingParams
    from ..engine.embedder import Embedder
    from ..engine.tokenizer import apply_chat_template, bert_byte_tokenizer, small_byte_tokenizer
    from ..index.hbm_index import HBMIndex
    from ..models.bert import BertConfig, BertModel
    from ..models.mixtral import MixtralConfig, MixtralModel
    from ..models.registry import _generic_tok
    from ..rag import synthetic
    from ..serving.openai_api import _tool_system_prompt, parse_tool_calls

    dev, rank, world = ctx.device, ctx.rank, ctx.world_size
    batch = args.batch or 32
    index_size = args.index_size or 1_000_000
    t_setup = time.perf_counter()
    mcfg = MixtralConfig.mixtral_8x7b() if args.agent_model == "mixtral-8x7b" else MixtralConfig.tiny_moe()
    ep_group = None
    if getattr(args, "ep", False) and world > 1:
        import torch.distributed as dist
        ep_group = dist.group.WORLD
    llm = MixtralModel(mcfg, device=dev, ep_group=ep_group).random_init(seed=21)
    tok = _generic_tok(mcfg) if mcfg.vocab_size > 4096 else small_byte_tokenizer(mcfg.vocab_size)
    bcfg = BertConfig.e5_large_v2() if args.agent_model == "mixtral-8x7b" else BertConfig.tiny()
    emb = Embedder(BertModel(bcfg, device=dev).random_init(seed=22), bert_byte_tokenizer(bcfg.vocab_size))
    index = HBMIndex(bcfg.hidden_size, "cosine", device=dev, capacity=index_size)
    index.add_random(index_size, seed=500 + rank, doc_fn=lambda r: synthetic.chunk_document(r, args.chunk_tokens))
    log(f"models ready: {mcfg.name} {llm.num_params() / 1e9:.1f}B, {bcfg.name}, index {index_size}")
    ecfg = EngineConfig(max_num_seqs=batch, max_batched_tokens=args.max_batched_tokens,
                        max_model_len=min(mcfg.max_position, int(1.25 * (4 * (args.chunk_tokens + 8) + 900 + args.plan_tokens))
                                          + args.max_tokens),
                        prefill_chunk=args.max_batched_tokens, use_graphs=not args.no_graphs, prefix_cache=False,
                        kv_memory_fraction=0.5, kv_memory_bytes=int(args.kv_gb * (1 << 30)) if args.kv_gb else None)
    engine = LLMEngine(llm, tok, ecfg)
    if not args.no_graphs:
        engine.capture_graphs(max_bs=batch)
    log(f"engine ready, setup {time.perf_counter() - t_setup:.1f}s")
    sys_prompt = _tool_system_prompt([TOOL], "auto")
    plan_p = SamplingParams(temperature=0.2, top_p=0.7, max_tokens=args.plan_tokens, ignore_eos=True)
    ans_p = SamplingParams(temperature=0.2, top_p=0.7, max_tokens=args.max_tokens, ignore_eos=True)

    def run_all(reqs):
        while engine.has_work():
            engine.step()
        return reqs

    def step(i: int) -> dict:
        t0 = time.perf_counter()
        qs = [synthetic.question((i * world + rank) * batch + j) for j in range(batch)]
        convs = [[{"role": "system", "content": sys_prompt}, {"role": "user", "content": q}] for q in qs]
        plans = run_all([engine.add_request(apply_chat_template(c, tok), plan_p) for c in convs])
        queries = []
        for q, r in zip(qs, plans):
            calls = parse_tool_calls(r.text, [TOOL])
            try:
                queries.append(json.loads(calls[0]["function"]["arguments"])["query"] if calls else q)
            except Exception:
                queries.append(q)
        t_tool = time.perf_counter()
        e = emb.embed(queries, "query")
        _, rows = index.search_raw(e.to(index.dtype), 4)
        rows = rows.cpu().tolist()
        t_tool = time.perf_counter() - t_tool
        t_ans = time.perf_counter()
        answers = []
        for c, r, rr in zip(convs, plans, rows):
            call = {"name": "search_knowledge_base", "parameters": {"query": "..."}}
            ctx_txt = "\n\n".join(index.document(g).page_content for g in rr if g >= 0)
            hist = c + [{"role": "assistant", "content": json.dumps([call])}, {"role": "ipython", "content": ctx_txt}]
            answers.append(engine.add_request(apply_chat_template(hist, tok), ans_p))
        run_all(answers)
        assert all(len(r.output_ids) == args.max_tokens for r in answers), "an answer was cut short"
        assert all(len(r.output_ids) == args.plan_tokens for r in plans), "a plan was cut short"
        return dict(ttft=[a.first_token_time - t0 for a in answers], answer_ttft=[a.first_token_time - t_ans for a in answers],
                    tokens=sum(len(r.output_ids) for r in plans + answers), tool_s=t_tool,
                    prompt=sum(len(a.prompt_ids) for a in answers) / len(answers))

    total, stats = timed_steps(ctx, step, args.steps, args.warmup)
    ttft = gather_list(ctx, [x for s in stats for x in s["ttft"]])
    attft = gather_list(ctx, [x for s in stats for x in s["answer_ttft"]])
    toks = sum(gather_list(ctx, [s["tokens"] for s in stats]))
    nq = batch * args.steps * world
    return {
        "metric": METRIC, "value": round(nq / total, 4), "unit": "conversations/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1000 * total / args.steps, 2),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic (random-init weights of the named architectures; synthetic corpus/questions; "
                "EOS ignored; unparseable tool calls fall back to the question as the tool query)",
        "config": {"model": f"{mcfg.name} + {bcfg.name} + {index_size}-vector HBM index per GPU",
                   "global_batch": batch * world, "seq_len": int(median([s["prompt"] for s in stats])) + args.max_tokens,
                   "parallelism": f"dp{world}-attention+ep{world}-experts" if ep_group is not None else f"dp{world}", "turns": 2, "plan_tokens": args.plan_tokens,
                   "max_tokens": args.max_tokens},
        "p50_ttft_s": round(percentile(ttft, 0.5), 4), "p50_answer_ttft_s": round(percentile(attft, 0.5), 4),
        "output_tokens_per_s": round(toks / total, 1),
        "tool_ms": round(1000 * median([s["tool_s"] for s in stats]), 2),
    }
