"""FAISS-API facade over the HBM index (the reference's chain-server builds
``FAISS(IndexFlatL2)`` in process, utils.py:305-306, and the notebooks use ``FAISS.from_texts`` /
``save_local`` / ``load_local``, langchain_basic_RAG.ipynb cells 20-22).

``FAISS`` keeps those method names and signatures so notebook code runs unchanged against the exact
HBM index (GPU when available). ``embedding`` may be this framework's :class:`Embeddings` or any
LangChain-style object with ``embed_documents`` / ``embed_query``. Persistence uses the index's own
snapshot format (raw vectors + JSONL documents, no pickle), so ``allow_dangerous_deserialization`` is
accepted and ignored.
"""
from __future__ import annotations

from typing import Iterable, List, Optional, Sequence, Tuple

import torch

from ..chain_server.connectors import Embeddings
from ..chain_server.vectorstore import VectorStore
from ..index.hbm_index import Document, HBMIndex


class _LangChainEmbeddings(Embeddings):
    def __init__(self, lc):
        self.lc = lc
        self.dim = None

    def embed_tensor(self, texts, input_type):
        vecs = self.lc.embed_query(texts[0]) if (input_type == "query" and len(texts) == 1) else None
        rows = [vecs] if vecs is not None else self.lc.embed_documents(list(texts))
        return torch.tensor(rows, dtype=torch.float32)


def _wrap(embedding) -> Embeddings:
    return embedding if hasattr(embedding, "embed_tensor") else _LangChainEmbeddings(embedding)


class FAISS:
    def __init__(self, store: VectorStore):
        self.store = store

    # ---------------------------------------------------------------- construction
    @classmethod
    def from_texts(cls, texts: Sequence[str], embedding, metadatas: Optional[List[dict]] = None, metric: str = "l2",
                   device=None, **kw) -> "FAISS":
        vs = VectorStore(kw.get("index_name", "faiss"), _wrap(embedding), metric=metric, device=device)
        vs.add_texts(list(texts), metadatas)
        return cls(vs)

    @classmethod
    def from_documents(cls, documents: Sequence[Document], embedding, **kw) -> "FAISS":
        return cls.from_texts([d.page_content for d in documents], embedding, [d.metadata for d in documents], **kw)

    def add_texts(self, texts: Iterable[str], metadatas: Optional[List[dict]] = None) -> List[int]:
        return self.store.add_texts(list(texts), metadatas)

    def add_documents(self, documents: Sequence[Document]) -> List[int]:
        return self.store.add_documents(list(documents))

    # ---------------------------------------------------------------- query
    def similarity_search_with_score(self, query: str, k: int = 4) -> List[Tuple[Document, float]]:
        return self.store.similarity_search_with_relevance_scores(query, k)

    similarity_search_with_relevance_scores = similarity_search_with_score

    def similarity_search(self, query: str, k: int = 4) -> List[Document]:
        return [d for d, _ in self.similarity_search_with_score(query, k)]

    def as_retriever(self, search_type: str = "similarity", search_kwargs: Optional[dict] = None, **kw):
        sk = search_kwargs or {}
        return self.store.as_retriever(search_type, sk.get("k", 4), sk.get("score_threshold"))

    # ---------------------------------------------------------------- persistence
    def save_local(self, folder_path: str, index_name: str = "index"):
        self.store.index.save(folder_path)

    @classmethod
    def load_local(cls, folder_path: str, embeddings, index_name: str = "index",
                   allow_dangerous_deserialization: bool = False, device=None) -> "FAISS":
        vs = VectorStore("faiss", _wrap(embeddings), device=device)
        vs.index = HBMIndex.load(folder_path, device=device or vs.index.device)
        return cls(vs)

    @property
    def index(self):
        return self.store.index
