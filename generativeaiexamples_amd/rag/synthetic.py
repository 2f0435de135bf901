"""Deterministic synthetic corpus and query set (no datasets offline).

Chunk ``i`` is a reproducible pseudo-random word sequence of ~``chunk_tokens`` tokens (the
reference splits documents into 510-token chunks, compose uses 506; configuration.py:86-90,
basic_rag/langchain/docker-compose.yaml:40-41). Text is generated on demand from the row id, so
a 10M-row index needs no host storage for its documents.
"""
from __future__ import annotations

import numpy as np

from ..index.hbm_index import Document

_WORDS = (
    "accelerator bandwidth cache kernel wavefront matrix tensor memory latency throughput cluster "
    "pipeline retrieval embedding vector index query document passage context answer model layer "
    "attention softmax gradient batch token sequence prefix decode prefill schedule router replica "
    "shard collective reduce gather scatter stream graph launch compiler register buffer queue "
    "policy service request response latency budget quality recall precision benchmark report "
    "network storage compute energy thermal clock frequency voltage power board rack node fabric"
).split()


_TABLE_N = 1 << 18
_TABLE: list = []


def _table() -> list:
    """A fixed pseudo-random word stream (built once, 256K words): chunk ``row`` reads a row-dependent window
    of it, so a chunk costs a list slice + a join (~5 us) instead of a per-chunk generator (~50 us)."""
    if not _TABLE:
        idx = np.random.default_rng(20240601).integers(len(_WORDS), size=_TABLE_N)
        _TABLE.extend(_WORDS[i] for i in idx.tolist())
    return _TABLE


def chunk_text(row: int, chunk_tokens: int = 506, bytes_per_token: float = 1.0) -> str:
    target = int(chunk_tokens * bytes_per_token)
    t = _table()
    off = (row * 2654435761) % (_TABLE_N - target)
    parts, n = [], 0
    for w in t[off:off + target // 2]:  # words are >= 3 bytes: the window always reaches target
        parts.append(w)
        n += len(w) + 1
        if n > target:
            break
    return " ".join(parts)[:target]


def chunk_document(row: int, chunk_tokens: int = 506) -> Document:
    return Document(chunk_text(row, chunk_tokens), {"filename": f"synthetic_{row // 64:07d}.txt", "row": row})


def question(i: int) -> str:
    rng = np.random.default_rng(i + 12345)
    a, b = (_WORDS[int(x)] for x in rng.integers(len(_WORDS), size=2))
    return f"What does the report say about the {a} of the {b} in section {i % 97}?"


def page_image(row: int, h: int = 720, w: int = 960) -> np.ndarray:
    """Deterministic synthetic 'slide / chart page' (HWC uint8): light background, a title band and
    a bar chart whose bar heights/colours derive from the row id (multimodal RAG corpus)."""
    rng = np.random.default_rng(row * 40503 % (1 << 32))
    img = np.full((h, w, 3), 245, dtype=np.uint8)
    img[: h // 10] = rng.integers(20, 120, size=3, dtype=np.uint8)
    nb = int(rng.integers(3, 9))
    bw = w // (2 * nb + 1)
    base = h - h // 12
    for i in range(nb):
        bh = int(rng.integers(h // 8, h // 2))
        x0 = (2 * i + 1) * bw
        img[base - bh:base, x0:x0 + bw] = rng.integers(0, 255, size=3, dtype=np.uint8)
    img[base:base + 2, bw // 2: w - bw // 2] = 30
    return img


def image_question(i: int) -> str:
    rng = np.random.default_rng(i + 777)
    a = _WORDS[int(rng.integers(len(_WORDS)))]
    return f"Which bar in the {a} chart is the tallest, and what trend does slide {i % 53} show?"
