"""BM25 sparse index + hybrid fusion (the reference's NeMo-Retriever profile runs
Elasticsearch BM25 next to the dense index, ``RetrieverConfig.nr_pipeline = 'ranked_hybrid'``).

The sparse side lives next to the HBM dense index and shares its row ids: an inverted index of
per-term posting arrays (numpy), Okapi BM25 scoring (k1 = 1.2, b = 0.75) by scatter-adding the
postings of the query terms, deletes by tombstone. ``rrf`` fuses ranked lists with reciprocal-rank
fusion (score = sum 1 / (60 + rank)), the standard score-free way to merge BM25 and cosine lists.
"""
from __future__ import annotations

import math
import re
import threading
from collections import Counter, defaultdict
from typing import Dict, List, Sequence, Tuple

import numpy as np

_TOK = re.compile(r"[a-z0-9]+")
_STOP = frozenset("a an and are as at be by for from has have in is it its of on or that the this to was were "
                  "will with what which who how".split())


def terms(text: str) -> List[str]:
    return [t for t in _TOK.findall(text.lower()) if t not in _STOP]


class BM25Index:
    def __init__(self, k1: float = 1.2, b: float = 0.75):
        self.k1, self.b = k1, b
        self.post: Dict[str, Tuple[List[int], List[int]]] = defaultdict(lambda: ([], []))
        self.doclen: Dict[int, int] = {}
        self.total_len = 0
        self.dead: set = set()
        self.lock = threading.Lock()

    def __len__(self):
        return len(self.doclen)

    def add(self, rows: Sequence[int], texts: Sequence[str]):
        with self.lock:
            for r, t in zip(rows, texts):
                tf = Counter(terms(t))
                for term, c in tf.items():
                    p = self.post[term]
                    p[0].append(int(r))
                    p[1].append(c)
                n = sum(tf.values())
                self.doclen[int(r)] = n
                self.total_len += n
                self.dead.discard(int(r))

    def delete(self, rows: Sequence[int]):
        with self.lock:
            for r in rows:
                n = self.doclen.pop(int(r), None)
                if n is not None:
                    self.total_len -= n
                    self.dead.add(int(r))

    def search(self, query: str, k: int) -> List[Tuple[int, float]]:
        with self.lock:
            N = len(self.doclen)
            if N == 0:
                return []
            avgdl = self.total_len / N
            scores: Dict[int, float] = defaultdict(float)
            for term in set(terms(query)):
                if term not in self.post:
                    continue
                rows, tfs = self.post[term]
                r = np.asarray(rows, np.int64)
                tf = np.asarray(tfs, np.float64)
                alive = np.fromiter((x not in self.dead for x in rows), bool, len(rows)) if self.dead else None
                if alive is not None:
                    r, tf = r[alive], tf[alive]
                if not len(r):
                    continue
                df = len(r)
                idf = math.log(1.0 + (N - df + 0.5) / (df + 0.5))
                dl = np.fromiter((self.doclen[int(x)] for x in r), np.float64, len(r))
                s = idf * tf * (self.k1 + 1) / (tf + self.k1 * (1 - self.b + self.b * dl / avgdl))
                for x, v in zip(r.tolist(), s.tolist()):
                    scores[x] += v
            top = sorted(scores.items(), key=lambda kv: -kv[1])[:k]
            return top


def rrf(ranked_lists: Sequence[Sequence[int]], k: int, c: int = 60) -> List[Tuple[int, float]]:
    """Reciprocal-rank fusion of several ranked id lists -> top-k (id, fused score)."""
    acc: Dict[int, float] = defaultdict(float)
    for lst in ranked_lists:
        for rank, rid in enumerate(lst):
            acc[rid] += 1.0 / (c + rank + 1)
    return sorted(acc.items(), key=lambda kv: -kv[1])[:k]
