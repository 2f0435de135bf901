"""advanced_rag/multi_turn_rag (E3; reference RAG/examples/advanced_rag/multi_turn_rag/chains.py:62-367).

Two stores: the document store and a conversation-memory store. With a reranker, 40 candidates
are retrieved from each and reranked down to top_k (chains.py:147,173-195); the answer is streamed
and the (question, answer) turn is written back to memory.

Fixed relative to the reference: memory is partitioned per session instead of one
global collection shared by all users (the reference's single ``conv_store``, chains.py:138). The session is the
``X-Session-Id`` header of POST /generate (passed in as ``session_id``); a client that sends none falls back to a key
derived from the conversation's first user message. The fallback messages are actually delivered (the reference's
generator swallowed them).
"""
from __future__ import annotations

import hashlib
import logging
from typing import Dict, Generator, List, Optional

from ..chain_server.utils import get_llm, get_ranking_model, get_vectorstore
from ..index.hbm_index import Document
from .basic_rag import NO_CONTEXT, BasicRAG

log = logging.getLogger(__name__)
CANDIDATES_WITH_RANKER = 40


def conversation_key(chat_history: List[Dict[str, str]], query: str, session_id: Optional[str] = None) -> str:
    """Memory partition of a conversation: the explicit session id when the client sends one (two users who both
    open with "Hi" then never share memory), else a hash of the first user message."""
    if session_id:
        return "s-" + hashlib.sha1(session_id.encode()).hexdigest()[:16]
    first = next((m["content"] for m in chat_history if m.get("role") == "user"), query)
    return hashlib.sha1(first.encode()).hexdigest()[:16]


class MultiTurnRAG(BasicRAG):
    def __init__(self):
        super().__init__()
        self._conv = None
        self._ranker_checked = False
        self._ranker = None

    @property
    def conv_store(self):
        if self._conv is None:
            self._conv = get_vectorstore(collection="conv_store")
        return self._conv

    @property
    def ranker(self):
        if not self._ranker_checked:
            self._ranker = get_ranking_model()
            self._ranker_checked = True
        return self._ranker

    def _fetch(self, store, query, conv_id=None):
        """k = 40 candidates when a ranker exists (else top_k), kept above ``retriever.score_threshold`` like the
        reference's ``similarity_score_threshold`` retrievers (chains.py:147-167); memory is searched inside the
        conversation's own partition of the index (exact top-k of that conversation, never crowded out)."""
        r = self.cfg.retriever
        k = CANDIDATES_WITH_RANKER if self.ranker else r.top_k
        hits = store.similarity_search_with_relevance_scores(
            query, k, r.score_threshold, filter={"conversation": conv_id} if conv_id else None)
        docs = [d for d, _ in hits][:k]
        if self.ranker and docs:
            docs = self.ranker.compress_documents(docs, query)
        else:
            docs = docs[: r.top_k]
        return docs

    def rag_chain(self, query: str, chat_history: List[Dict[str, str]], session_id: Optional[str] = None,
                  **kwargs) -> Generator[str, None, None]:
        conv_id = conversation_key(chat_history, query, session_id)
        docs = self._fetch(self.store, query)
        memory = self._fetch(self.conv_store, query, conv_id) if len(self.conv_store) else []
        if not docs and not memory:
            yield NO_CONTEXT
            return
        sys_prompt = self.prompts["multi_turn_rag_template"].format(
            history="\n".join(d.page_content for d in memory), context="\n\n".join(d.page_content for d in docs))
        msgs = [{"role": "system", "content": sys_prompt}, {"role": "user", "content": query}]
        answer = []
        for chunk in get_llm(**kwargs).stream(msgs):
            answer.append(chunk)
            yield chunk
        turn = f"User: {query}\nAssistant: {''.join(answer)}"
        self.conv_store.add_documents([Document(turn, {"conversation": conv_id, "filename": f"conversation-{conv_id}"})])
