"""Exact, HBM-resident vector index (replaces Milvus GPU_IVF_FLAT / pgvector / FAISS IndexFlatL2,
SURVEY S4-S6; ``create_vectorstore_langchain`` utils.py:288-332).

* vectors live in one bf16 ``[capacity, dim]`` HBM tensor (grown by doubling); a 1M x 1024 index
  is 2 GiB, a 10M one 20 GiB - trivially resident in 288 GB;
* search is the fused similarity-GEMM + top-k HIP kernel (never materialises [nq, N] scores):
  exact, so recall >= the reference's IVF (nlist 64, nprobe 16);
* metrics: ``cosine`` (normalised inner product, relevance = cosine), ``ip`` and ``l2``
  (relevance = 1 - d/sqrt(2) like LangChain's euclidean relevance fn), all through one per-row
  fp32 bias (0, 0 or -|x|^2/2, and -inf for deleted rows - tombstones);
* documents (text + metadata) are kept in a host-side store keyed by row; delete-by-filename
  tombstones rows and compacts when a quarter of the index is dead;
* persistence: ``save(dir)`` / ``load(dir)`` write vectors (raw bf16), bias and a JSONL doc store
  plus an append-only write-ahead log of inserts/deletes, so the HBM index survives restarts
  (the reference's in-process FAISS store is lost on restart).
"""
from __future__ import annotations

import json
import math
import os
import threading
from dataclasses import dataclass, field
from typing import Any, Dict, Iterable, List, Optional, Sequence

import numpy as np
import torch

from .. import ops


def _hashable(v):
    return v if isinstance(v, (str, int, float, bool, type(None))) else json.dumps(v, sort_keys=True, default=str)


@dataclass
class Document:
    page_content: str
    metadata: Dict[str, Any] = field(default_factory=dict)


@dataclass
class SearchHit:
    row: int
    score: float          # relevance score (higher is better)
    document: Document


PARTITION_KEYS = ("conversation",)


class HBMIndex:
    def __init__(self, dim: int, metric: str = "cosine", device=None, capacity: int = 1 << 14,
                 dtype=torch.bfloat16, name: str = "default"):
        assert metric in ("cosine", "ip", "l2")
        self.dim, self.metric, self.dtype, self.name = dim, metric, dtype, name
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        capacity = max(capacity, 16)
        self.vectors = torch.zeros(capacity, dim, dtype=dtype, device=self.device)
        self.bias = torch.full((capacity,), float("-inf"), dtype=torch.float32, device=self.device)
        self.n = 0
        self.docs: List[Optional[Document]] = []
        self.dead = 0
        self.lock = threading.RLock()
        self.wal = None
        # metadata keys whose values partition the rows (a conversation's memory, a tenant): a filtered search on
        # one of them scans only that partition's rows, so a small partition is never crowded out of a global
        # top-k by the rest of the collection
        self.partition_keys = set(PARTITION_KEYS)
        self.parts: Dict[tuple, List[int]] = {}

    # ------------------------------------------------------------------ sizing
    def __len__(self) -> int:
        return self.n - self.dead

    @property
    def capacity(self) -> int:
        return self.vectors.shape[0]

    def _grow(self, need: int):
        if need <= self.capacity:
            return
        cap = self.capacity
        while cap < need:
            cap *= 2
        v = torch.zeros(cap, self.dim, dtype=self.dtype, device=self.device)
        b = torch.full((cap,), float("-inf"), dtype=torch.float32, device=self.device)
        v[: self.n] = self.vectors[: self.n]
        b[: self.n] = self.bias[: self.n]
        self.vectors, self.bias = v, b

    # ------------------------------------------------------------------ mutation
    def _prep(self, vecs: torch.Tensor) -> torch.Tensor:
        vecs = vecs.to(self.device, torch.float32)
        if self.metric == "cosine":
            vecs = torch.nn.functional.normalize(vecs, dim=-1)
        return vecs

    def add(self, vectors: torch.Tensor, documents: Sequence[Document] | None = None) -> List[int]:
        if vectors.ndim == 1:
            vectors = vectors[None]
        assert vectors.shape[1] == self.dim, f"dim {vectors.shape[1]} != index dim {self.dim}"
        v = self._prep(vectors)
        k = v.shape[0]
        documents = list(documents) if documents is not None else [None] * k
        with self.lock:
            self._grow(self.n + k)
            rows = list(range(self.n, self.n + k))
            self.vectors[self.n:self.n + k] = v.to(self.dtype)
            if self.metric == "l2":
                self.bias[self.n:self.n + k] = -0.5 * v.to(self.dtype).float().pow(2).sum(-1)
            else:
                self.bias[self.n:self.n + k] = 0.0
            self.docs.extend(documents)
            self.n += k
            self._index_parts(rows, documents)
            if self.wal:
                for r, d in zip(rows, documents):
                    self.wal.write(json.dumps({"op": "add", "row": r, "doc": _doc_json(d)}) + "\n")
                self.wal.flush()
        return rows

    def _index_parts(self, rows: Sequence[int], documents: Sequence[Optional[Document]]):
        for r, d in zip(rows, documents):
            if d is None:
                continue
            for key in self.partition_keys & d.metadata.keys():
                self.parts.setdefault((key, _hashable(d.metadata[key])), []).append(r)

    def _unindex_parts(self, rows: Sequence[int]):
        """Drop deleted rows from their partitions (only the partitions those rows' documents name; the full
        rebuild is for compact() and load(), which renumber rows)."""
        gone: Dict[tuple, set] = {}
        for r in rows:
            d = self.docs[r]
            if d is None:
                continue
            for key in self.partition_keys & d.metadata.keys():
                gone.setdefault((key, _hashable(d.metadata[key])), set()).add(r)
        for pk, rs in gone.items():
            left = [r for r in self.parts.get(pk, []) if r not in rs]
            if left:
                self.parts[pk] = left
            else:
                self.parts.pop(pk, None)

    def _rebuild_parts(self):
        self.parts = {}
        self._index_parts(range(self.n), self.docs[: self.n])

    def add_random(self, n: int, seed: int = 0, doc_fn=None, chunk: int = 1 << 20):
        """Bulk-insert n random unit vectors (synthetic corpora for benchmarks); docs lazily from doc_fn(row)."""
        g = torch.Generator(device=self.device)
        g.manual_seed(seed)
        with self.lock:
            self._grow(self.n + n)
            done = 0
            while done < n:
                k = min(chunk, n - done)
                v = torch.randn(k, self.dim, device=self.device, generator=g)
                v = torch.nn.functional.normalize(v, dim=-1)
                self.vectors[self.n:self.n + k] = v.to(self.dtype)
                self.bias[self.n:self.n + k] = 0.0 if self.metric != "l2" else -0.5
                self.n += k
                done += k
            self.docs.extend([None] * n)
            self.doc_fn = doc_fn

    def set_vectors(self, rows: Sequence[int], vectors: torch.Tensor) -> None:
        """Overwrite the vectors of existing rows (same preparation as ``add``). Synthetic benchmarks plant
        a question's relevant chunks this way so that every query retrieves its own rows."""
        v = self._prep(vectors if vectors.ndim == 2 else vectors[None])
        idx = torch.as_tensor(list(rows), dtype=torch.long, device=self.device)
        assert idx.numel() == v.shape[0] and (idx.numel() == 0 or int(idx.max()) < self.n)
        with self.lock:
            self.vectors[idx] = v.to(self.dtype)
            if self.metric == "l2":
                self.bias[idx] = -0.5 * v.to(self.dtype).float().pow(2).sum(-1)

    def delete(self, predicate) -> int:
        """Tombstone every row whose document satisfies predicate(doc). Returns #deleted."""
        with self.lock:
            rows = [i for i, d in enumerate(self.docs) if d is not None and predicate(d)]
            if rows:
                idx = torch.tensor(rows, device=self.device)
                self.bias[idx] = float("-inf")
                self._unindex_parts(rows)
                for r in rows:
                    self.docs[r] = None
                self.dead += len(rows)
                if self.wal:
                    self.wal.write(json.dumps({"op": "del", "rows": rows}) + "\n")
                    self.wal.flush()
                if self.dead * 4 > self.n and self.n > 1024:
                    self.compact()
            return len(rows)

    def delete_filename(self, filename: str) -> int:
        return self.delete(lambda d: d.metadata.get("filename") == filename or
                           os.path.basename(str(d.metadata.get("source", ""))) == filename)

    def live_rows(self) -> List[int]:
        """Rows holding a stored document (not deleted)."""
        return [i for i, d in enumerate(self.docs[: self.n]) if d is not None]

    def compact(self):
        with self.lock:
            keep = torch.nonzero(torch.isfinite(self.bias[: self.n])).flatten().tolist()
            idx = torch.tensor(keep, dtype=torch.long, device=self.device)
            v, b = self.vectors[idx].clone(), self.bias[idx].clone()
            docs = [self.docs[i] for i in keep]
            self.n = len(keep)
            self.vectors[: self.n] = v
            self.bias[: self.n] = b
            self.bias[self.n:] = float("-inf")
            self.docs = docs
            self.dead = 0
            self._rebuild_parts()

    # ------------------------------------------------------------------ query
    def _relevance(self, raw: torch.Tensor, q: torch.Tensor) -> torch.Tensor:
        if self.metric == "l2":
            # raw = q.x - |x|^2/2  ->  d^2 = |q|^2 - 2 raw
            d2 = (q.float().pow(2).sum(-1, keepdim=True) - 2 * raw).clamp_min(0)
            return 1.0 - d2.sqrt() / math.sqrt(2.0)
        return raw

    def search_raw(self, queries: torch.Tensor, k: int):
        """-> (relevance [nq, k'], rows [nq, k']) on device."""
        from ..utils.profiling import roctx_range
        with roctx_range("index_search"):
            return self._search_raw(queries, k)

    def _search_raw(self, queries: torch.Tensor, k: int):
        q = self._prep(queries if queries.ndim == 2 else queries[None])
        with self.lock:
            if self.n == 0:
                z = torch.empty(q.shape[0], 0, device=self.device)
                return z, z.long()
            k = min(k, 64)
            raw, rows = ops.sim_topk(q.to(self.dtype), self.vectors, self.bias, self.n, k)
        rel = self._relevance(raw, q)
        return rel, rows

    def rows_where(self, filt: Dict[str, Any]) -> List[int]:
        """Live rows whose document metadata equals every (key, value) of ``filt``: a partition lookup when one
        key is a partition key, else a scan of the stored documents."""
        with self.lock:
            cand = None
            for key, val in filt.items():
                if key in self.partition_keys:
                    cand = list(self.parts.get((key, _hashable(val)), []))
                    break
            if cand is None:
                cand = range(self.n)
            return [r for r in cand if r < len(self.docs) and self.docs[r] is not None
                    and all(self.docs[r].metadata.get(k2) == v2 for k2, v2 in filt.items())]

    def _search_rows(self, q: torch.Tensor, k: int, rows: List[int]):
        """Exact top-k over a row subset (gathered to a contiguous slab, same scan kernel and bias)."""
        if not rows:
            z = torch.empty(q.shape[0], 0, device=self.device)
            return z, z.long()
        idx = torch.tensor(rows, dtype=torch.long, device=self.device)
        with self.lock:
            sub, bias = self.vectors.index_select(0, idx).contiguous(), self.bias.index_select(0, idx).contiguous()
        raw, loc = ops.sim_topk(q.to(self.dtype), sub, bias, len(rows), min(k, 64, len(rows)))
        out = torch.where(loc >= 0, idx[loc.clamp_min(0)], torch.full_like(loc, -1))
        return self._relevance(raw, q), out

    def search(self, queries: torch.Tensor, k: int = 4, score_threshold: Optional[float] = None,
               filter: Optional[Dict[str, Any]] = None) -> List[List[SearchHit]]:  # noqa: A002 - LangChain's name
        if filter:
            q = self._prep(queries if queries.ndim == 2 else queries[None])
            rel, rows = self._search_rows(q, k, self.rows_where(filter))
        else:
            rel, rows = self.search_raw(queries, k)
        rel, rows = rel.cpu().tolist(), rows.cpu().tolist()
        out = []
        for rs, ids in zip(rel, rows):
            hits = []
            for s, r in zip(rs, ids):
                if r < 0 or not math.isfinite(s):
                    continue
                if score_threshold is not None and s < score_threshold:
                    continue
                hits.append(SearchHit(r, s, self.document(r)))
            out.append(hits)
        return out

    def document(self, row: int) -> Document:
        d = self.docs[row] if row < len(self.docs) else None
        if d is None and getattr(self, "doc_fn", None) is not None:
            return self.doc_fn(row)
        return d if d is not None else Document("", {})

    def filenames(self) -> List[str]:
        seen, out = set(), []
        for d in self.docs:
            if d is None:
                continue
            f = d.metadata.get("filename") or os.path.basename(str(d.metadata.get("source", "")))
            if f and f not in seen:
                seen.add(f)
                out.append(f)
        return out

    # ------------------------------------------------------------------ persistence
    def save(self, path: str):
        os.makedirs(path, exist_ok=True)
        with self.lock:
            v = self.vectors[: self.n].view(torch.int16).cpu().numpy()
            v.tofile(os.path.join(path, "vectors.bf16"))
            self.bias[: self.n].cpu().numpy().tofile(os.path.join(path, "bias.f32"))
            with open(os.path.join(path, "meta.jsonl"), "w") as f:
                for d in self.docs:
                    f.write(json.dumps(_doc_json(d)) + "\n")
            with open(os.path.join(path, "index.json"), "w") as f:
                json.dump({"dim": self.dim, "metric": self.metric, "n": self.n, "dead": self.dead,
                           "name": self.name, "format": 1}, f)
            # a checkpoint supersedes the WAL
            open(os.path.join(path, "wal.jsonl"), "w").close()

    @classmethod
    def load(cls, path: str, device=None) -> "HBMIndex":
        with open(os.path.join(path, "index.json")) as f:
            meta = json.load(f)
        idx = cls(meta["dim"], meta["metric"], device=device, capacity=max(meta["n"], 16), name=meta.get("name", ""))
        n = meta["n"]
        if n:
            v = np.fromfile(os.path.join(path, "vectors.bf16"), dtype=np.int16).reshape(n, meta["dim"])
            idx.vectors[:n] = torch.from_numpy(v).view(torch.bfloat16).to(idx.device)
            idx.bias[:n] = torch.from_numpy(np.fromfile(os.path.join(path, "bias.f32"), dtype=np.float32)).to(idx.device)
        with open(os.path.join(path, "meta.jsonl")) as f:
            idx.docs = [_doc_from_json(json.loads(line)) for line in f]
        idx.n, idx.dead = n, meta.get("dead", 0)
        idx._replay_wal(path)
        idx._rebuild_parts()
        return idx

    def _replay_wal(self, path: str):
        p = os.path.join(path, "wal.jsonl")
        if not os.path.exists(p):
            return
        with open(p) as f:
            for line in f:
                if not line.strip():
                    continue
                e = json.loads(line)
                if e["op"] == "del":
                    for r in e["rows"]:
                        if r < self.n and self.docs[r] is not None:
                            self.docs[r] = None
                            self.bias[r] = float("-inf")
                            self.dead += 1
                # "add" entries carry documents only; vectors are recovered by re-embedding on ingest replay

    def attach_wal(self, path: str):
        os.makedirs(path, exist_ok=True)
        self.wal = open(os.path.join(path, "wal.jsonl"), "a")


def _doc_json(d: Optional[Document]):
    return None if d is None else {"page_content": d.page_content, "metadata": d.metadata}


def _doc_from_json(o) -> Optional[Document]:
    return None if o is None else Document(o["page_content"], o.get("metadata", {}))
