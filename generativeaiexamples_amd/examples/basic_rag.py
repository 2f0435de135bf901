"""basic_rag (E1 of SURVEY §2.2; reference RAG/examples/basic_rag/langchain/chains.py:52-256).

ingest: load (txt/md/pdf/html/docx/pptx/csv) -> token splitter (chunk_size-2 / overlap) -> embed
"passage:" -> HBM index. rag_chain: embed "query:" -> exact top-k with the relevance threshold ->
``rag_template`` system prompt + "Context: ...\\n\\nQuestion: ..." -> streamed generation.
llm_chain: ``chat_template`` + history + question. Also the LlamaIndex flavour (E2) with its
1 500-token context cap (LimitRetrievedNodesLength, utils.py:103-134).
"""
from __future__ import annotations

import logging
import os
from typing import Any, Dict, Generator, List

from ..chain_server.base import BaseExample
from ..chain_server.utils import (del_docs_vectorstore, get_config, get_docs_vectorstore, get_llm, get_prompts,
                                  get_text_splitter, get_vectorstore)
from ..rag import loaders
from ..rag.prompts import rag_user_message

log = logging.getLogger(__name__)
NO_CONTEXT = ("No response generated from the knowledge base. Make sure the question is relevant to the "
              "ingested documents.")


def _history_messages(chat_history: List[Dict[str, str]]) -> List[Dict[str, str]]:
    return [{"role": m["role"], "content": m["content"]} for m in chat_history
            if m.get("role") in ("user", "assistant") and m.get("content")]


class BasicRAG(BaseExample):
    """Retrieval-augmented chat over the HBM index with the in-process (or remote) generator."""

    def __init__(self):
        self.cfg = get_config()
        self.prompts = get_prompts()
        self._store = None
        self._splitter = None

    @property
    def store(self):
        if self._store is None:
            self._store = get_vectorstore()
        return self._store

    @property
    def splitter(self):
        if self._splitter is None:
            self._splitter = get_text_splitter()
        return self._splitter

    # --------------------------------------------------------------------------- ingest
    def ingest_docs(self, filepath: str, filename: str) -> None:
        ext = os.path.splitext(filename)[1].lower()
        if ext not in loaders.SUPPORTED:
            raise ValueError(f"{filename} is not a supported file type ({', '.join(sorted(loaders.SUPPORTED))})")
        docs = loaders.load(filepath, filename)
        chunks = self.splitter.split_documents(docs)
        if not chunks:
            raise ValueError(f"no text could be extracted from {filename}")
        self.store.add_documents(chunks)
        log.info("ingested %s: %d chunks", filename, len(chunks))

    # --------------------------------------------------------------------------- chains
    def llm_chain(self, query: str, chat_history: List[Dict[str, str]], **kwargs) -> Generator[str, None, None]:
        msgs = [{"role": "system", "content": self.prompts["chat_template"]}]
        msgs += _history_messages(chat_history)
        msgs.append({"role": "user", "content": query})
        return get_llm(**kwargs).stream(msgs)

    def retrieve(self, query: str):
        """Dense top-k with the score threshold; with a hybrid store (APP_VECTORSTORE_HYBRID=true) the
        retriever's nrPipeline selects BM25+dense reciprocal-rank fusion ('hybrid') or fusion of 40
        candidates reranked to top-k ('ranked_hybrid', the reference NeMo-Retriever default)."""
        r = self.cfg.retriever
        if self.store.bm25 is not None and r.nr_pipeline in ("hybrid", "ranked_hybrid"):
            from ..chain_server.utils import get_ranking_model
            ranker = get_ranking_model() if r.nr_pipeline == "ranked_hybrid" else None
            hits = self.store.hybrid_search(query, 40 if ranker else r.top_k)
            if ranker and hits:
                docs = ranker.compress_documents([d for d, _ in hits], query)
                return [(d, d.metadata.get("relevance_score", 0.0)) for d in docs]
            return hits
        return self.store.similarity_search_with_relevance_scores(query, r.top_k, r.score_threshold)

    def rag_chain(self, query: str, chat_history: List[Dict[str, str]], **kwargs) -> Generator[str, None, None]:
        hits = self.retrieve(query)
        if not hits:
            return iter([NO_CONTEXT])
        context = "\n\n".join(d.page_content for d, _ in hits)
        msgs = [{"role": "system", "content": self.prompts["rag_template"]}]
        msgs += _history_messages(chat_history)
        msgs.append({"role": "user", "content": rag_user_message(context, query)})
        return get_llm(**kwargs).stream(msgs)

    # --------------------------------------------------------------------------- documents
    def document_search(self, content: str, num_docs: int) -> List[Dict[str, Any]]:
        hits = self.store.similarity_search_with_relevance_scores(content, num_docs)
        return [{"content": d.page_content, "filename": d.metadata.get("filename", ""), "score": s} for d, s in hits]

    def get_documents(self) -> List[str]:
        return get_docs_vectorstore(self.store)

    def delete_documents(self, filenames: List[str]) -> bool:
        return del_docs_vectorstore(self.store, filenames)


class LlamaIndexRAG(BasicRAG):
    """basic_rag/llamaindex flavour (E2): top-k retrieval, retrieved nodes capped at 1 500 tokens in
    total, and the per-node filename reported correctly by /search (reference defect §7.7 item 4)."""

    MAX_CONTEXT_TOKENS = 1500

    def rag_chain(self, query: str, chat_history: List[Dict[str, str]], **kwargs) -> Generator[str, None, None]:
        r = self.cfg.retriever
        hits = self.store.similarity_search_with_relevance_scores(query, r.top_k)
        if not hits:
            return iter([NO_CONTEXT])
        tok = self.splitter.tok
        kept, used = [], 0
        for d, _ in hits:
            n = len(tok.encode(d.page_content))
            if used + n > self.MAX_CONTEXT_TOKENS:
                break
            kept.append(d.page_content)
            used += n
        context = "\n\n".join(kept) if kept else hits[0][0].page_content
        msgs = [{"role": "system", "content": self.prompts["rag_template"]},
                {"role": "user", "content": rag_user_message(context, query)}]
        return get_llm(**kwargs).stream(msgs)
