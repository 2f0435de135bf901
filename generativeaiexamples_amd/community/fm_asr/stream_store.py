"""Streaming-transcript store of the FM-radio RAG app (reference: /root/reference/community/fm-asr-streaming-rag/
chain-server/accumulator.py:29-63, database.py:38-94, retriever.py:41-211).

* ``TimestampDatabase``: every finalized chunk with its arrival time and source (sqlite3), queried by recency
  (``recent``: since a time) or by a window around a past time (``past``).
* ``StreamRetriever``: the same chunks embedded into the HBM vector index (one collection per app, passages with the
  embedder's ``passage`` prefix), searched by similarity, reranked when a reranker is available, and thinned by the
  reference's outlier rule (drop chunks whose relevance falls more than max(stdev, 0.1 |mean|) below the best).
* ``TextAccumulator``: per-source text buffer. New text is appended and re-split (recursive character splitter,
  ``chunk_size`` / ``chunk_overlap``); every chunk but the last is final - stored in both stores - and the last stays
  in the buffer to grow.
"""
from __future__ import annotations

import datetime as _dt
import sqlite3
import statistics
import threading
from typing import Callable, Dict, List, Optional

from ...chain_server.connectors import rerank
from ...index.hbm_index import Document
from ...rag.text_splitter import RecursiveCharacterTextSplitter

_FMT = "%Y-%m-%d %H:%M:%S.%f"


class TimestampDatabase:
    def __init__(self, path: str = ":memory:", clock: Callable[[], _dt.datetime] = _dt.datetime.now):
        self.conn = sqlite3.connect(path, check_same_thread=False)
        self.clock = clock
        self.lock = threading.Lock()
        with self.lock:
            self.conn.execute("CREATE TABLE IF NOT EXISTS messages (id INTEGER PRIMARY KEY, text TEXT, "
                              "timestamp TEXT, source_id TEXT)")
            self.conn.commit()

    def insert_docs(self, docs: List[str], source_id: str) -> None:
        now = self.clock().strftime(_FMT)
        with self.lock:
            self.conn.executemany("INSERT INTO messages (text, timestamp, source_id) VALUES (?, ?, ?)",
                                  [(d, now, source_id) for d in docs])
            self.conn.commit()

    @staticmethod
    def _doc(row) -> Document:
        return Document(row[1], {"tstamp": _dt.datetime.strptime(row[2], _FMT), "source_id": row[3]})

    def recent(self, since: _dt.datetime) -> List[Document]:
        """Every chunk stored at or after ``since``, oldest first."""
        with self.lock:
            rows = self.conn.execute("SELECT * FROM messages WHERE timestamp >= ? ORDER BY id",
                                     (since.strftime(_FMT),)).fetchall()
        return [self._doc(r) for r in rows]

    def past(self, when: _dt.datetime, window: float = 90.0) -> List[Document]:
        """Chunks stored within ``window`` seconds of ``when``."""
        lo = (when - _dt.timedelta(seconds=window)).strftime(_FMT)
        hi = (when + _dt.timedelta(seconds=window)).strftime(_FMT)
        with self.lock:
            rows = self.conn.execute("SELECT * FROM messages WHERE timestamp BETWEEN ? AND ? ORDER BY id",
                                     (lo, hi)).fetchall()
        return [self._doc(r) for r in rows]

    def __len__(self) -> int:
        with self.lock:
            return self.conn.execute("SELECT COUNT(*) FROM messages").fetchone()[0]


def drop_outliers(docs: List[Document], min_cv: float = 0.1) -> List[Document]:
    """Keep the chunks whose relevance lies within max(stdev, min_cv |mean|) of the best one (docs sorted best first)."""
    scores = [float(d.metadata.get("relevance_score", 0.0)) for d in docs]
    if len(scores) < 2:
        return docs
    floor = scores[0] - max(statistics.stdev(scores), min_cv * abs(statistics.mean(scores)))
    return [d for d, s in zip(docs, scores) if s >= floor]


class StreamRetriever:
    """Vector side of the stream store. ``store``: a chain-server VectorStore; ``ranker``: optional Ranker."""

    def __init__(self, store, ranker=None, outlier_min_docs: int = 5):
        self.store, self.ranker, self.outlier_min_docs = store, ranker, outlier_min_docs

    def add_docs(self, docs: List[str], source_id: str) -> int:
        if not docs:
            return 0
        self.store.add_documents([Document(d, {"source_id": source_id, "filename": source_id}) for d in docs])
        return len(docs)

    def search(self, query: str, max_entries: int = 8) -> List[Document]:
        if len(self.store) == 0:
            return []
        hits = self.store.similarity_search_with_relevance_scores(query, max_entries)
        docs = []
        for d, s in hits:
            md = dict(d.metadata)
            md.setdefault("relevance_score", float(s))
            docs.append(Document(d.page_content, md))
        if self.ranker is not None and docs:
            docs = rerank(self.ranker, docs, query, len(docs))
        docs.sort(key=lambda d: -float(d.metadata.get("relevance_score", 0.0)))
        if len(docs) > self.outlier_min_docs:
            docs = drop_outliers(docs)
        return docs


class TextAccumulator:
    def __init__(self, retriever: Optional[StreamRetriever], chunk_size: int = 1024, chunk_overlap: int = 200,
                 timestamp_db: Optional[TimestampDatabase] = None,
                 on_final: Optional[Callable[[str, str], None]] = None):
        self.splitter = RecursiveCharacterTextSplitter(chunk_size, chunk_overlap)
        self.chunk_size, self.chunk_overlap = chunk_size, chunk_overlap
        self.buffers: Dict[str, str] = {}
        self.timestamp_db = timestamp_db if timestamp_db is not None else TimestampDatabase()
        self.retriever = retriever
        self.on_final = on_final  # e.g. the reference's push of each finalized chunk to its frontend
        self.lock = threading.Lock()

    def update(self, source_id: str, text: str) -> Dict[str, str]:
        with self.lock:
            cur = self.buffers.get(source_id, "")
            docs = self.splitter.split_text(f"{cur} {text}".strip()) or [""]
            self.buffers[source_id], final = docs[-1], docs[:-1]
        if final:
            self.timestamp_db.insert_docs(final, source_id)
            if self.retriever is not None:
                self.retriever.add_docs(final, source_id)
            if self.on_final is not None:
                for d in final:
                    self.on_final(source_id, d)
        return {"status": f"Added {len(final)} entries"}

    def pending(self, source_id: str) -> str:
        return self.buffers.get(source_id, "")
