"""Ingest-path and query-embedding throughput on one GPU (VERDICT r5 missing #2 / next #6).

The reference's ingest is POST /documents -> embedding NIM (nv-embedqa-e5-v5) -> Milvus
(/root/reference/RAG/examples/local_deploy/docker-compose-nim-ms.yaml:30-56); its streaming ingest batches up to 256
chunks per Triton call (community/streaming_ingest_rag/docker/extras/all-MiniLM-L6-v2_config.pbtxt:3-29). Here the
same path runs in-process through the framework's real components:

  synthetic 506-token chunks -> IngestPipeline (rag/ingest_pipeline.py: load/split stage, embed stage, write stage on
  threads with bounded queues) -> LocalEmbeddings -> Embedder.embed_coalesced (DynamicBatcher, <= 256 chunks per
  encoder call, e5-large-v2 "passage: " encoding, varlen-packed micro-batches) -> VectorStore.add_embedded ->
  HBMIndex.add

and reports chunks/s per GPU plus each stage's rate. ``--query`` times the 64-query burst embed of bench.py (tokenise +
graph-replayed encoder + pooling) with a host / device split.

Random-init e5-large-v2 weights (no checkpoints offline); byte-level tokenisation (chunk_text's 506 bytes -> 506
tokens, + "passage: " and [CLS]/[SEP], truncated to the 512-token encoder window).

  python tools/ingest_bench.py --chunks 1000000 --json-out gpurun_out/ingest.json
  python tools/ingest_bench.py --query --iters 50
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def build_embedder(name: str, device):
    from generativeaiexamples_amd.engine.embedder import Embedder
    from generativeaiexamples_amd.engine.tokenizer import bert_byte_tokenizer
    from generativeaiexamples_amd.models.bert import BertConfig, BertModel

    cfg = {"e5-large-v2": BertConfig.e5_large_v2, "e5-base-v2": BertConfig.e5_base_v2,
           "minilm": BertConfig.minilm_l6_v2, "tiny": BertConfig.tiny}[name]()
    enc = BertModel(cfg, device=device).random_init(7)
    return Embedder(enc, bert_byte_tokenizer(cfg.vocab_size))


class _PassThrough:
    """The synthetic chunks are already chunk-sized: the load stage hands them on unchanged."""

    def split_documents(self, docs):
        return docs


def run_ingest(args, emb, device) -> dict:
    from generativeaiexamples_amd.chain_server.connectors import LocalEmbeddings
    from generativeaiexamples_amd.chain_server.vectorstore import VectorStore
    from generativeaiexamples_amd.rag import synthetic
    from generativeaiexamples_amd.rag.ingest_pipeline import IngestPipeline

    store = VectorStore("ingest_bench", LocalEmbeddings(emb), device=device)
    store.index._grow(args.chunks)  # one allocation up front (the index grows by doubling otherwise)
    docs_per_item = 64

    def source(n, start=0):
        for b in range(start, start + n, docs_per_item):
            yield [synthetic.chunk_document(r) for r in range(b, min(b + docs_per_item, start + n))]

    # warm-up: the encoder's first micro-batches (allocator, kernel attributes), not timed
    IngestPipeline(store, _PassThrough(), embed_batch=args.embed_batch).run(source(2 * args.embed_batch, 1 << 30))
    store.index = type(store.index)(store.index.dim, store.index.metric, device=device, name="ingest_bench")
    store.index._grow(args.chunks)
    pipe = IngestPipeline(store, _PassThrough(), embed_batch=args.embed_batch, write_batch=args.write_batch)
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    last = [t0]

    def progress_source():
        for i, item in enumerate(source(args.chunks)):
            if time.perf_counter() - last[0] > 30:
                last[0] = time.perf_counter()
                print(f"[ingest] submitted {i * docs_per_item} chunks, embedded {pipe.stats.embed.items}, "
                      f"{pipe.stats.embed.items / (last[0] - t0):.0f} chunks/s", flush=True)
            yield item

    st = pipe.run(progress_source())
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    wall = time.perf_counter() - t0
    assert len(store.index) == args.chunks, (len(store.index), args.chunks)
    assert not st.errors, st.errors[:3]
    tokens = args.chunks * min(emb.max_len, len(emb.tokenize(synthetic.chunk_text(0), "passage")))
    return {"chunks": args.chunks, "wall_s": round(wall, 2), "chunks_per_s": round(args.chunks / wall, 1),
            "tokens_per_s": round(tokens / wall), "embed_batch": args.embed_batch, "stage_rates": pipe.rates(),
            "embed_stage_busy_s": round(st.embed.seconds, 2), "write_stage_busy_s": round(st.write.seconds, 2),
            "index_rows": len(store.index)}


def run_query(args, emb, device) -> dict:
    from generativeaiexamples_amd.rag import synthetic

    emb.capture_graphs()
    qs = [[synthetic.question(s * 64 + i) for i in range(64)] for s in range(args.iters + 3)]
    walls, toks, gpu = [], [], []
    for s, batch in enumerate(qs):
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        ids = [emb.tokenize(q, "query") for q in batch]
        t1 = time.perf_counter()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        out = emb.embed_ids(ids)
        ev1.record()
        torch.cuda.synchronize(device)
        t2 = time.perf_counter()
        if s >= 3:
            walls.append(1e3 * (t2 - t0))
            toks.append(1e3 * (t1 - t0))
            gpu.append(ev0.elapsed_time(ev1))
    assert out.shape == (64, emb.dim)
    L = [len(x) for x in ids]
    return {"queries": 64, "tokens_per_query": [min(L), max(L)], "embed_ms_p50": round(statistics.median(walls), 3),
            "tokenize_ms_p50": round(statistics.median(toks), 3), "encoder_ms_p50": round(statistics.median(gpu), 3),
            "iters": args.iters}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--embedder", default="e5-large-v2")
    ap.add_argument("--chunks", type=int, default=100_000)
    ap.add_argument("--embed-batch", type=int, default=256)
    ap.add_argument("--write-batch", type=int, default=4096)
    ap.add_argument("--query", action="store_true", help="time the 64-query burst embed instead of ingest")
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--json-out", default="")
    args = ap.parse_args()
    device = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    emb = build_embedder(args.embedder, device)
    res = {"embedder": args.embedder, "device": str(device), "data": "synthetic 506-token chunks, random-init weights"}
    res.update(run_query(args, emb, device) if args.query else run_ingest(args, emb, device))
    print(json.dumps(res), flush=True)
    if args.json_out:
        with open(args.json_out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
