"""Retrieval strategies and the answer fact-check of the multimodal / O-RAN assistants (reference:
/root/reference/community/oran-chatbot-multimodal/Multimodal_Assistant.py:92-165 and 396-616 - ``rag_type`` 0 plain
retrieval, 1 multi-query (five LLM-suggested related questions, every query retrieved, duplicates dropped, cross-encoder
top 10), 2 HyDE (the query extended with a hypothetical answer), 3 multi-query retriever (rephrasings of the question); history-aware query rewriting;
guardrails/fact_check.py - a second model call that checks the answer against the context and starts with TRUE / FALSE).

MI355X-first detail: the augmented queries of one request are submitted to the vector store's dynamic batcher together,
so all of them share ONE query-embedding batch and ONE scan of the HBM index (``VectorStore._search_batch``) instead of
one embed + scan per query; the reranker scores all unique candidates in one cross-encoder batch.
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import Callable, Dict, Iterator, List, Optional, Sequence, Tuple

from ..chain_server.connectors import rerank
from ..index.hbm_index import Document

RELATED_QUESTIONS = (
    "Suggest five further questions closely related to the user's question that would help retrieve the documentation "
    "needed to answer it. Each must be short, self-contained and about a different aspect. One question per line, no "
    "numbering, nothing else.")
REPHRASINGS = (
    "Write three different phrasings of the user's question that ask for exactly the same information, to widen a "
    "similarity search. One per line, nothing else.")
HYPOTHETICAL_ANSWER = (
    "Write a detailed, plausible answer to the question in the style of technical documentation on the subject. It is "
    "used only to search for the real documentation, so favour the vocabulary such documents would use.")
REWRITE_WITH_HISTORY = (
    "Rewrite the user's follow-up question so that it is clear and self-contained given the conversation history: "
    "resolve every reference to earlier turns and keep its full intent. Reply with the rewritten question only.")
FACT_CHECK = (
    "Fact-check a model's answer against the context documents only - no outside knowledge. Check every claim in the "
    "RESPONSE against the CONTEXT and whether it answers the QUESTION. Begin your reply with TRUE if the response is "
    "fully supported and answers the question, otherwise with FALSE, then explain briefly and suggest follow-up "
    "questions the documents could answer.")

STRATEGIES = ("plain", "multi_query", "hyde", "multi_query_retriever")


def _ask(llm, system: str, user: str, **kw) -> str:
    r = llm.invoke([{"role": "system", "content": system}, {"role": "user", "content": user}], **kw)
    return getattr(r, "content", r) or ""


def related_questions(llm, query: str, n: int = 5, prompt: str = RELATED_QUESTIONS) -> List[str]:
    lines = [re.sub(r"^\s*(?:\d+[.)]|[-*•])\s*", "", ln).strip() for ln in
             _ask(llm, prompt, f"Question: {query}", temperature=0.0, max_tokens=400).splitlines()]
    return [ln for ln in lines if len(ln) > 3 and ln.lower() != query.lower()][:n]


def hypothetical_answer(llm, query: str) -> str:
    return _ask(llm, HYPOTHETICAL_ANSWER, f"Question: {query}", temperature=0.0, max_tokens=400).strip()


def rewrite_with_history(llm, query: str, history: Sequence[Tuple[str, str]]) -> str:
    if not history:
        return query
    hist = "\n".join(f"User: {u}\nAssistant: {a}" for u, a in history)
    out = _ask(llm, REWRITE_WITH_HISTORY, f"History:\n{hist}\n\nFollow-up question: {query}", temperature=0.0,
               max_tokens=200).strip()
    return out or query


def batched_search(store, queries: Sequence[str], k: int) -> List[List[Tuple[Document, float]]]:
    """All queries through the store's batcher at once (one embed + one index scan); stores without a batcher are
    searched one query at a time."""
    b = getattr(store, "batcher", None)
    if b is None or len(store) == 0:
        return [store.similarity_search_with_relevance_scores(q, k) if len(store) else [] for q in queries]
    futs = b.submit_many([(q, k, None) for q in queries])
    return [f.result() for f in futs]


def dedupe(hit_lists: Sequence[Sequence[Tuple[Document, float]]]) -> List[Document]:
    """Unique passages across queries (first occurrence keeps its metadata; best score kept)."""
    best: Dict[str, Document] = {}
    for hits in hit_lists:
        for d, s in hits:
            cur = best.get(d.page_content)
            if cur is None or float(s) > cur.metadata.get("relevance_score", float("-inf")):
                best[d.page_content] = Document(d.page_content, dict(d.metadata, relevance_score=float(s)))
    return sorted(best.values(), key=lambda d: -d.metadata["relevance_score"])


@dataclass
class Retrieval:
    query: str
    queries: List[str]
    documents: List[Document] = field(default_factory=list)

    @property
    def context(self) -> str:
        return "\n\n".join(d.page_content for d in self.documents)

    def sources(self) -> Dict[str, str]:
        """source -> concatenated passages (the reference's per-source citation panel)."""
        out: Dict[str, str] = {}
        for d in self.documents:
            src = d.metadata.get("source", d.metadata.get("filename", ""))
            out[src] = f"{out[src]}\n\n{d.page_content}" if src in out else d.page_content
        return out


def retrieve(strategy: str, llm, store, query: str, k: int = 4, top_n: int = 10, ranker=None) -> Retrieval:
    if strategy not in STRATEGIES:
        raise ValueError(f"unknown strategy {strategy!r}; one of {STRATEGIES}")
    if strategy == "plain":
        queries = [query]
    elif strategy == "hyde":
        queries = [f"{query} {hypothetical_answer(llm, query)}".strip()]
    elif strategy == "multi_query":  # the question plus five related questions, retrieved together
        queries = [query] + related_questions(llm, query)
    else:  # LangChain MultiQueryRetriever's form: three rephrasings of the same question
        queries = [query] + related_questions(llm, query, 3, REPHRASINGS)
    docs = dedupe(batched_search(store, queries, k))
    if ranker is not None and docs and strategy != "plain":
        docs = rerank(ranker, docs, query, top_n)  # scored against the ORIGINAL question
    return Retrieval(query, queries, docs[:top_n] if strategy != "plain" else docs[:k])


@dataclass
class FactCheck:
    verdict: Optional[bool]
    text: str


def parse_fact_check(text: str) -> FactCheck:
    m = re.search(r"\b(TRUE|FALSE)\b", text or "")
    return FactCheck(None if m is None else m.group(1) == "TRUE", (text or "").strip())


def fact_check_stream(llm, context: str, query: str, response: str) -> Iterator[str]:
    msgs = [{"role": "system", "content": FACT_CHECK},
            {"role": "user", "content": f"CONTEXT:\n{context}\n\nQUESTION:\n{query}\n\nRESPONSE:\n{response}"}]
    yield from llm.stream(msgs, temperature=0.0, max_tokens=512)


def fact_check(llm, context: str, query: str, response: str) -> FactCheck:
    return parse_fact_check("".join(fact_check_stream(llm, context, query, response)))


class AssistantChain:
    """The assistants' turn: optional image description folded into the question, history-aware rewrite, one of the
    retrieval strategies, a streamed answer, then the streamed fact-check."""

    def __init__(self, llm, store, ranker=None, strategy: str = "multi_query", k: int = 4, top_n: int = 10,
                 system: str = "You are a helpful assistant for technical documentation. Answer from the relevant "
                               "documents; say so when they do not cover the question.",
                 describe_image: Optional[Callable[[bytes], str]] = None, check_facts: bool = True):
        self.llm, self.store, self.ranker, self.strategy = llm, store, ranker, strategy
        self.k, self.top_n, self.system, self.describe_image = k, top_n, system, describe_image
        self.check_facts = check_facts
        self.history: List[Tuple[str, str]] = []
        self.last: Optional[Retrieval] = None

    def turn(self, question: str, image: Optional[bytes] = None) -> Iterator[str]:
        if image is not None and self.describe_image is not None:
            question = (f"I have uploaded an image with the following description: {self.describe_image(image)} "
                        f"Here is the question: {question}")
        q = rewrite_with_history(self.llm, question, self.history)
        r = self.last = retrieve(self.strategy, self.llm, self.store, q, self.k, self.top_n, self.ranker)
        msgs = [{"role": "system", "content": self.system},
                {"role": "user", "content": f"Relevant documents:\n{r.context}\n\nQUESTION:\n{q}"}]
        answer = ""
        for piece in self.llm.stream(msgs, temperature=0.2, max_tokens=1024):
            answer += piece
            yield piece
        self.history.append((q, answer))
        if self.check_facts:
            yield "\n\nFact check: "
            yield from fact_check_stream(self.llm, r.context, q, answer)
