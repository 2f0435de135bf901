"""BASELINE config 4: multimodal RAG - NV-CLIP ViT-L/14 retrieval + Llama-3.2-11B-Vision generation on
the fp8 MFMA GEMMs (reference analogue: RAG/examples/advanced_rag/multimodal_rag).

Per GPU (data parallel, weak scaling):
  setup (untimed): CLIP ViT-L/14 + Llama-3.2-11B-Vision (random-init weights of the real geometry,
    linear weights quantised to e4m3fn per channel), an exact HBM index of ``--index-size`` 768-d
    CLIP page embeddings: ``--ingest-images`` synthetic slide images embedded for real by the CLIP
    vision tower, the rest random unit vectors standing for already-ingested pages.
  one timed step = ``--batch`` queries:
    question -> CLIP text embedding -> exact top-1 page -> the page image's tiles through the Mllama
    vision encoder (batched across the step's queries) -> cross-attention K/V -> continuous-batching
    generation (temperature 0.2 / top_p 0.7, ``--max-tokens``, EOS ignored) attending to the page.
value = total queries/s over all ranks; TTFT = step start -> first token per query.
"""
from __future__ import annotations

import time

import torch

from .common import gather_list, log, median, percentile, timed_steps

METRIC = "multimodal RAG queries/sec + p50 TTFT, NV-CLIP ViT-L/14 + Llama-3.2-11B-Vision (fp8)"


def add_args(ap):
    ap.add_argument("--mm-model", default="llama3.2-11b-vision", choices=["llama3.2-11b-vision", "tiny"])
    ap.add_argument("--mm-clip", default="vit_l_14", choices=["vit_l_14", "tiny"])
    ap.add_argument("--ingest-images", type=int, default=256)
    ap.add_argument("--no-fp8", action="store_true")


def run(args, ctx) -> dict:
    from ..engine import EngineConfig, LLMEngine, SamplingParams
    from ..engine.tokenizer import apply_chat_template, llama3_byte_tokenizer, small_byte_tokenizer
    from ..index.hbm_index import HBMIndex
    from ..models.clip import ClipConfig, ClipModel
    from ..models.mllama import MllamaConfig, MllamaModel
    from ..rag import synthetic

    dev, rank, world = ctx.device, ctx.rank, ctx.world_size
    batch = args.batch if args.batch else 32
    index_size = args.index_size if args.index_size else 1_000_000
    t_setup = time.perf_counter()
    clip = ClipModel(getattr(ClipConfig, args.mm_clip)(), device=dev).random_init(seed=11)
    mcfg = MllamaConfig.llama32_11b_vision() if args.mm_model != "tiny" else MllamaConfig.tiny()
    llm = MllamaModel(mcfg, device=dev, max_images_in_flight=max(batch, 8)).random_init(seed=12)
    fp8 = not args.no_fp8
    if fp8:
        clip.quantize_fp8("vt")
        llm.quantize_fp8()
    tok = llama3_byte_tokenizer(mcfg.text.vocab_size) if mcfg.text.vocab_size >= 128256 else \
        small_byte_tokenizer(mcfg.text.vocab_size)
    ctok = small_byte_tokenizer(clip.cfg.vocab_size) if clip.cfg.vocab_size <= 4096 else \
        __import__("generativeaiexamples_amd.models.registry", fromlist=["_clip_tok"])._clip_tok(clip.cfg.vocab_size)
    log(f"models ready ({'fp8' if fp8 else 'bf16'}): {mcfg.name}, {clip.cfg.name}")

    # ---- page index: real CLIP embeddings of synthetic slides + random stand-ins for the rest
    index = HBMIndex(clip.cfg.projection_dim, "cosine", device=dev, capacity=index_size)
    n_real = min(args.ingest_images, index_size)
    for s in range(0, n_real, 64):
        rows = list(range(s, min(n_real, s + 64)))
        px = clip.preprocess([synthetic.page_image(rank * index_size + r) for r in rows])
        index.add(clip.encode_image(px).to(index.dtype))
    if index_size > n_real:
        index.add_random(index_size - n_real, seed=300 + rank)
    log(f"page index ready: {index_size} x {clip.cfg.projection_dim} ({n_real} real CLIP page embeddings)")

    S = mcfg.vision.image_size
    ecfg = EngineConfig(max_num_seqs=batch, max_batched_tokens=args.max_batched_tokens,
                        max_model_len=min(mcfg.text.max_position, 512 + args.max_tokens), prefill_chunk=args.max_batched_tokens,
                        use_graphs=not args.no_graphs, prefix_cache=False, kv_memory_fraction=0.3,
                        kv_memory_bytes=int(args.kv_gb * (1 << 30)) if args.kv_gb else None)
    engine = LLMEngine(llm, tok, ecfg)
    if not args.no_graphs:
        engine.capture_graphs(max_bs=batch)
    log(f"engine ready, setup {time.perf_counter() - t_setup:.1f}s")
    params = SamplingParams(temperature=0.2, top_p=0.7, max_tokens=args.max_tokens, ignore_eos=True)
    system = "You are a helpful assistant that answers questions about the slide image you are shown."

    def step(i: int) -> dict:
        t0 = time.perf_counter()
        qs = [synthetic.image_question((i * world + rank) * batch + j) for j in range(batch)]
        qe = clip.encode_text([ctok.encode(q)[:75] for q in qs])
        _, rows = index.search_raw(qe.to(index.dtype), 1)
        rows = rows[:, 0].cpu().tolist()
        ims = [llm.preprocess(synthetic.page_image(rank * index_size + max(r, 0))) for r in rows]
        states = llm.encode_images(ims)
        t_ret = time.perf_counter() - t0
        reqs = []
        for q, st in zip(qs, states):
            ids = apply_chat_template([{"role": "system", "content": system},
                                       {"role": "user", "content": [{"type": "image"}, {"type": "text", "text": q}]}],
                                      tok, image_token_id=llm.mcfg.image_token_id)
            reqs.append(engine.add_request(ids, params, images=[st]))
        while engine.has_work():
            engine.step()
        assert all(len(r.output_ids) == args.max_tokens for r in reqs), "a query was cut short"
        return dict(ttft=[r.first_token_time - t0 for r in reqs], tokens=sum(len(r.output_ids) for r in reqs),
                    retrieval_s=t_ret, tiles=sum(im.num_tiles for im in ims) / len(ims),
                    prompt=sum(len(r.prompt_ids) for r in reqs) / len(reqs))

    total, stats = timed_steps(ctx, step, args.steps, args.warmup)
    ttft = gather_list(ctx, [x for s in stats for x in s["ttft"]])
    toks = sum(gather_list(ctx, [s["tokens"] for s in stats]))
    nq = batch * args.steps * world
    qps = nq / total
    return {
        "metric": METRIC, "value": round(qps, 4), "unit": "queries/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(1000 * total / args.steps, 2), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "fp8" if fp8 else "bf16",
        "data": "synthetic (random-init weights of the named architectures; synthetic slide images and questions)",
        "config": {"model": f"{clip.cfg.name} + {mcfg.name}" + (" (fp8 e4m3 weights+activations)" if fp8 else ""),
                   "global_batch": batch * world, "seq_len": int(median([s["prompt"] for s in stats])) + args.max_tokens,
                   "parallelism": f"dp{world}", "index_size_per_gpu": index_size,
                   "image_tiles_per_query": round(median([s["tiles"] for s in stats]), 2),
                   "max_tokens": args.max_tokens},
        "p50_ttft_s": round(percentile(ttft, 0.5), 4), "p90_ttft_s": round(percentile(ttft, 0.9), 4),
        "output_tokens_per_s": round(toks / total, 1),
        "retrieval_and_vision_ms": round(1000 * median([s["retrieval_s"] for s in stats]), 2),
    }
