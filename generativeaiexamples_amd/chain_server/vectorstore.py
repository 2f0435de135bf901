"""Vector-store facade over the HBM index (the LangChain VectorStore / LlamaIndex VectorStoreIndex
roles of the reference: ``add_documents``, ``similarity_search_with_relevance_scores``,
``as_retriever(search_type="similarity_score_threshold")``, delete and list by filename).
Collections are named (``COLLECTION_NAME`` env, ``conv_store`` for multi-turn memory) and each is
one :class:`HBMIndex`, optionally persisted (snapshot + WAL) under ``APP_VECTORSTORE_PERSISTDIR``."""
from __future__ import annotations

import logging
import os
import threading
from typing import Dict, List, Optional, Tuple

from ..index.bm25 import BM25Index, rrf
from ..index.hbm_index import Document, HBMIndex
from ..utils.metrics import METRICS
from . import tracing
from .connectors import Embeddings

log = logging.getLogger(__name__)


class Retriever:
    def __init__(self, store: "VectorStore", k: int = 4, score_threshold: Optional[float] = None):
        self.store, self.k, self.threshold = store, k, score_threshold

    def get_relevant_documents(self, query: str) -> List[Document]:
        return [d for d, _ in self.store.similarity_search_with_relevance_scores(query, self.k, self.threshold)]

    invoke = get_relevant_documents


class VectorStore:
    def __init__(self, name: str, embeddings: Embeddings, metric: str = "cosine", device=None,
                 persist_dir: Optional[str] = None, batch: int = 256, hybrid: bool = False):
        self.name, self.emb, self.batch = name, embeddings, batch
        self.bm25: Optional[BM25Index] = BM25Index() if hybrid else None
        self.persist = os.path.join(persist_dir, name) if persist_dir else None
        self.lock = threading.Lock()
        if self.persist and os.path.exists(os.path.join(self.persist, "index.json")):
            self.index = HBMIndex.load(self.persist, device=device)
            log.info("loaded collection %s (%d vectors) from %s", name, len(self.index), self.persist)
        else:
            self.index = HBMIndex(embeddings.dim or 1024, metric, device=device, name=name)
        if self.persist:
            self.index.attach_wal(self.persist)
        if self.bm25 is not None and len(self.index):  # rebuild the sparse side from the restored documents
            live = self.index.live_rows()
            self.bm25.add(live, [self.index.document(r).page_content for r in live])

    def add_embedded(self, vecs, docs: List[Document]) -> List[int]:
        """Insert already-embedded chunks (the streaming-ingest write stage)."""
        with self.lock:
            if self.index.dim != vecs.shape[1] and len(self.index) == 0:
                self.index = HBMIndex(vecs.shape[1], self.index.metric, device=self.index.device, name=self.name)
                if self.persist:
                    self.index.attach_wal(self.persist)
            rows = self.index.add(vecs, docs)
            if self.index.device.type == "cuda":  # queries scan on the retrieval stream: writes land first
                import torch

                torch.cuda.current_stream(self.index.device).synchronize()
            if self.bm25 is not None:
                self.bm25.add(rows, [d.page_content for d in docs])
            return rows

    def add_documents(self, docs: List[Document]) -> List[int]:
        rows: List[int] = []
        for i in range(0, len(docs), self.batch):
            part = docs[i:i + self.batch]
            vecs = self.emb.embed_tensor([d.page_content for d in part], "passage")
            rows += self.add_embedded(vecs, part)
        if self.persist:
            self.index.save(self.persist)
        return rows

    add_texts = lambda self, texts, metadatas=None: self.add_documents(  # noqa: E731
        [Document(t, (metadatas or [{}] * len(texts))[i]) for i, t in enumerate(texts)])

    # ---- query path: concurrent queries of this collection coalesce into ONE embed + ONE scan
    @property
    def batcher(self):
        if getattr(self, "_batcher", None) is None:
            from ..engine.embedder import DynamicBatcher

            from ..utils.streams import RETRIEVAL_GATE

            with self.lock:
                if getattr(self, "_batcher", None) is None:
                    self._batcher = DynamicBatcher(self._search_batch, max_batch=256, name=f"search-{self.name}",
                                                   gate=RETRIEVAL_GATE)
        return self._batcher

    def _search_batch(self, items: List[Tuple[str, int, Optional[float]]]) -> List[List[Tuple[Document, float]]]:
        """[(query, k, threshold)] -> hits per query: one query-embedding micro-batch and one exact scan of
        the index for all of them (the scan streams the whole index once per batch, not once per query),
        on the high-priority retrieval stream."""
        from ..utils.streams import on_retrieval_stream

        with on_retrieval_stream(self.index.device):
            q = self.emb.embed_tensor([it[0] for it in items], "query")
            kmax = max(it[1] for it in items)
            hits = self.index.search(q.to(self.index.device), kmax, None)
        return [[(h.document, h.score) for h in hs[:k] if thr is None or h.score >= thr]
                for hs, (_, k, thr) in zip(hits, items)]

    @tracing.traced("retriever")
    def similarity_search_with_relevance_scores(self, query: str, k: int = 4, score_threshold: Optional[float] = None,
                                                filter: Optional[dict] = None) -> List[Tuple[Document, float]]:  # noqa: A002
        """Top-k (document, relevance) for a query. ``filter`` (LangChain's metadata-equality dict) searches only
        the matching rows inside the index - a partition scan for partition keys such as ``conversation`` - so a
        filtered top-k is exact however large the rest of the collection is."""
        import time

        t0 = time.perf_counter()
        if filter:
            from ..utils.streams import on_retrieval_stream
            with on_retrieval_stream(self.index.device):
                q = self.emb.embed_tensor([query], "query")
                hits = self.index.search(q.to(self.index.device), k, score_threshold, filter=filter)[0]
            hits = [(h.document, h.score) for h in hits]
        else:
            hits = self.batcher.submit((query, k, score_threshold)).result()
        METRICS.search.observe(time.perf_counter() - t0)
        return hits

    @tracing.traced("retriever")
    def hybrid_search(self, query: str, k: int = 4, candidates: int = 40) -> List[Tuple[Document, float]]:
        """Dense (HBM cosine top-``candidates``) + sparse (BM25 top-``candidates``) fused by reciprocal rank."""
        import time

        if self.bm25 is None:
            return self.similarity_search_with_relevance_scores(query, k)
        t0 = time.perf_counter()
        q = self.emb.embed_tensor([query], "query")
        dense = [h.row for h in self.index.search(q, candidates)[0]]
        sparse = [r for r, _ in self.bm25.search(query, candidates)]
        fused = rrf([dense, sparse], k)
        METRICS.search.observe(time.perf_counter() - t0)
        return [(self.index.document(r), s) for r, s in fused]

    def similarity_search(self, query: str, k: int = 4) -> List[Document]:
        return [d for d, _ in self.similarity_search_with_relevance_scores(query, k)]

    def as_retriever(self, search_type: str = "similarity", k: int = 4, score_threshold: Optional[float] = None):
        return Retriever(self, k, score_threshold if search_type == "similarity_score_threshold" else None)

    def delete_filename(self, filename: str) -> bool:
        n = self.index.delete_filename(filename)
        if self.bm25 is not None and n:  # deletes may compact (renumber) the dense rows: rebuild the sparse side
            self.bm25 = BM25Index()
            live = self.index.live_rows()
            self.bm25.add(live, [self.index.document(r).page_content for r in live])
        if self.persist and n:
            self.index.save(self.persist)
        return n > 0

    def filenames(self) -> List[str]:
        return self.index.filenames()

    def __len__(self):
        return len(self.index)


_STORES: Dict[str, VectorStore] = {}
_LOCK = threading.Lock()


def get_store(name: str, embeddings: Embeddings, metric: str = "cosine", persist_dir: Optional[str] = None,
              device=None, hybrid: bool = False) -> VectorStore:
    with _LOCK:
        if name not in _STORES:
            _STORES[name] = VectorStore(name, embeddings, metric, device, persist_dir, hybrid=hybrid)
        return _STORES[name]


def reset_stores():
    with _LOCK:
        _STORES.clear()
