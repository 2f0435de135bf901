"""Text splitters used by the ingest pipelines.

* :class:`TokenTextSplitter` - windows of ``tokens_per_chunk`` tokens with ``overlap`` tokens of
  overlap, counted with the embedding model's tokenizer (the reference uses a sentence-transformers
  token splitter with ``tokens_per_chunk = chunk_size - 2`` to leave room for [CLS]/[SEP],
  RAG/src/chain_server/utils.py:474-489).
* :class:`RecursiveCharacterTextSplitter` - paragraph / line / sentence / word fallback by
  characters (multimodal example: 1000 / 100; synthetic data generator: 3000 / 100).
* :class:`CharacterTextSplitter` - single separator (query-decomposition example).
"""
from __future__ import annotations

import re
from typing import Callable, Iterable, List, Optional, Sequence

from ..index.hbm_index import Document


class TextSplitter:
    def split_text(self, text: str) -> List[str]:
        raise NotImplementedError

    def split_documents(self, docs: Iterable[Document]) -> List[Document]:
        out = []
        for d in docs:
            for i, chunk in enumerate(self.split_text(d.page_content)):
                md = dict(d.metadata)
                md["chunk"] = i
                out.append(Document(chunk, md))
        return out


class TokenTextSplitter(TextSplitter):
    def __init__(self, tokenizer, tokens_per_chunk: int = 508, overlap: int = 200):
        if overlap >= tokens_per_chunk:
            raise ValueError("overlap must be smaller than tokens_per_chunk")
        self.tok, self.n, self.overlap = tokenizer, tokens_per_chunk, overlap

    def split_text(self, text: str) -> List[str]:
        ids = self.tok.encode(text)
        if not ids:
            return []
        out, step = [], self.n - self.overlap
        for s in range(0, len(ids), step):
            piece = ids[s:s + self.n]
            t = self.tok.decode(piece).strip()
            if t:
                out.append(t)
            if s + self.n >= len(ids):
                break
        return out


class RecursiveCharacterTextSplitter(TextSplitter):
    def __init__(self, chunk_size: int = 1000, chunk_overlap: int = 100,
                 separators: Optional[Sequence[str]] = None, length_function: Callable[[str], int] = len):
        self.size, self.overlap = chunk_size, chunk_overlap
        self.seps = list(separators or ["\n\n", "\n", ". ", " ", ""])
        self.length = length_function

    def _merge(self, pieces: List[str], sep: str) -> List[str]:
        out, cur, cur_len = [], [], 0
        for p in pieces:
            pl = self.length(p)
            if cur and cur_len + pl + (len(sep) if cur else 0) > self.size:
                out.append(sep.join(cur))
                # keep a tail of the previous chunk as overlap
                while cur and cur_len > self.overlap:
                    cur_len -= self.length(cur[0]) + len(sep)
                    cur.pop(0)
            cur.append(p)
            cur_len += pl + (len(sep) if len(cur) > 1 else 0)
        if cur:
            out.append(sep.join(cur))
        return [o for o in out if o.strip()]

    def _split(self, text: str, seps: List[str]) -> List[str]:
        sep = seps[-1]
        rest: List[str] = []
        for i, s in enumerate(seps):
            if s == "" or s in text:
                sep, rest = s, seps[i + 1:]
                break
        parts = list(text) if sep == "" else text.split(sep)
        good, out = [], []
        for p in parts:
            if self.length(p) <= self.size:
                good.append(p)
            else:
                if good:
                    out.extend(self._merge(good, sep))
                    good = []
                out.extend(self._split(p, rest) if rest else [p])
        if good:
            out.extend(self._merge(good, sep))
        return out

    def split_text(self, text: str) -> List[str]:
        return self._split(text, self.seps)


class CharacterTextSplitter(RecursiveCharacterTextSplitter):
    def __init__(self, separator: str = "\n\n", chunk_size: int = 1000, chunk_overlap: int = 200):
        super().__init__(chunk_size, chunk_overlap, [separator])


def sentences(text: str) -> List[str]:
    return [s for s in re.split(r"(?<=[.!?])\s+", text) if s]
