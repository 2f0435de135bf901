"""Stage-pipelined streaming ingest (the reference's Morpheus pipeline
source -> tokenize -> Triton MiniLM inference -> vector-DB write, with MonitorStage rates).

Stages run concurrently on threads connected by bounded queues, so document loading / chunking /
tokenisation on the host overlaps the GPU embedding of the previous batch and the index write of
the one before (the CPU side never starves the GPU, back-pressure bounds memory):

  source (files | directory watch | JSONL stream | python iterable)
    -> load + split  (loaders + text splitter, CPU)
    -> embed         (batches of ``embed_batch`` chunks -> embedding service, GPU)
    -> write         (HBM vector store add, ``write_batch`` rows per insert)

Every stage counts items and seconds; ``rates()`` reports docs/s, chunks/s, embeddings/s, rows/s like
the reference's MonitorStage lines. ``run()`` drains a finite source; ``start()`` + ``submit()`` +
``close()`` serve a long-lived stream (the Kafka-consumer role).
"""
from __future__ import annotations

import json
import logging
import os
import queue
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Iterable, List, Optional

from ..index.hbm_index import Document
from .loaders import load
from .text_splitter import RecursiveCharacterTextSplitter

log = logging.getLogger(__name__)
_END = object()


@dataclass
class StageStats:
    items: int = 0
    seconds: float = 0.0
    first: Optional[float] = None
    last: Optional[float] = None

    def tick(self, n: int, dt: float):
        now = time.perf_counter()
        self.first = self.first or now - dt
        self.last = now
        self.items += n
        self.seconds += dt

    def rate(self) -> float:
        span = (self.last - self.first) if self.first and self.last else 0.0
        return self.items / span if span > 0 else 0.0


@dataclass
class IngestStats:
    load: StageStats = field(default_factory=StageStats)
    embed: StageStats = field(default_factory=StageStats)
    write: StageStats = field(default_factory=StageStats)
    docs: int = 0
    errors: List[str] = field(default_factory=list)


class IngestPipeline:
    def __init__(self, store, splitter=None, embed_batch: int = 256, write_batch: int = 1024, queue_depth: int = 8,
                 load_fn: Optional[Callable[[str], List[Document]]] = None):
        self.store = store
        self.splitter = splitter or RecursiveCharacterTextSplitter(chunk_size=2000, chunk_overlap=200)
        self.embed_batch, self.write_batch = embed_batch, write_batch
        self.load_fn = load_fn or (lambda p: load(p, os.path.basename(p)))
        self.q_in: queue.Queue = queue.Queue(queue_depth * 4)
        self.q_chunks: queue.Queue = queue.Queue(queue_depth)
        self.q_vecs: queue.Queue = queue.Queue(queue_depth)
        self.stats = IngestStats()
        self.threads: List[threading.Thread] = []

    # ------------------------------------------------------------------ stages
    def _load_stage(self):
        buf: List[Document] = []
        while True:
            item = self.q_in.get()
            if item is _END:
                break
            t0 = time.perf_counter()
            try:
                docs = item if isinstance(item, list) else self.load_fn(item) if isinstance(item, str) else [item]
                chunks = self.splitter.split_documents(docs)
            except Exception as e:  # a bad document must not stop the stream
                self.stats.errors.append(f"{item}: {e}")
                continue
            self.stats.docs += 1
            self.stats.load.tick(len(chunks), time.perf_counter() - t0)
            buf += chunks
            while len(buf) >= self.embed_batch:
                self.q_chunks.put(buf[: self.embed_batch])
                buf = buf[self.embed_batch:]
        if buf:
            self.q_chunks.put(buf)
        self.q_chunks.put(_END)

    def _embed_stage(self):
        emb = self.store.emb
        while True:
            batch = self.q_chunks.get()
            if batch is _END:
                break
            t0 = time.perf_counter()
            vecs = emb.embed_tensor([d.page_content for d in batch], "passage")
            self.stats.embed.tick(len(batch), time.perf_counter() - t0)
            self.q_vecs.put((vecs, batch))
        self.q_vecs.put(_END)

    def _write_stage(self):
        pend_v, pend_d = [], []

        def flush():
            if not pend_d:
                return
            import torch
            t0 = time.perf_counter()
            v = torch.cat(pend_v) if len(pend_v) > 1 else pend_v[0]
            self.store.add_embedded(v, list(pend_d))
            self.stats.write.tick(len(pend_d), time.perf_counter() - t0)
            pend_v.clear()
            pend_d.clear()

        while True:
            item = self.q_vecs.get()
            if item is _END:
                break
            vecs, docs = item
            pend_v.append(vecs)
            pend_d.extend(docs)
            if len(pend_d) >= self.write_batch:
                flush()
        flush()
        if getattr(self.store, "persist", None):
            self.store.index.save(self.store.persist)

    # ------------------------------------------------------------------ control
    def start(self):
        for fn in (self._load_stage, self._embed_stage, self._write_stage):
            t = threading.Thread(target=fn, daemon=True, name=f"ingest-{fn.__name__}")
            t.start()
            self.threads.append(t)
        return self

    def submit(self, item):
        """A file path, a Document, or a list of Documents."""
        self.q_in.put(item)

    def close(self, timeout: float = 3600) -> IngestStats:
        self.q_in.put(_END)
        for t in self.threads:
            t.join(timeout)
        return self.stats

    def run(self, source: Iterable) -> IngestStats:
        self.start()
        for item in source:
            self.submit(item)
        return self.close()

    def rates(self) -> dict:
        s = self.stats
        return {"docs": s.docs, "chunks_per_s": round(s.load.rate(), 1), "embeddings_per_s": round(s.embed.rate(), 1),
                "rows_written_per_s": round(s.write.rate(), 1), "errors": len(s.errors)}


def directory_source(path: str, exts=(".txt", ".md", ".pdf", ".html", ".csv", ".json", ".docx", ".pptx")):
    for root, _, files in os.walk(path):
        for f in sorted(files):
            if f.lower().endswith(exts):
                yield os.path.join(root, f)


def jsonl_source(path: str, text_key: str = "text"):
    """One document per JSONL line (``{"text": ..., any metadata}``), like a Kafka topic dump."""
    with open(path, encoding="utf-8") as f:
        for line in f:
            if line.strip():
                row = json.loads(line)
                text = row.pop(text_key, "")
                yield Document(text, row)
