"""Routed multi-source RAG (reference: /root/reference/community/routing-multisource-rag/workflow.py:128-391 and
prompts.py:16-125 - a routing model decides whether a message needs retrieval at all; if so the query is rewritten
into search terms with the previous user turn, sent to every source concurrently (the vector database and a web-search
LLM with a timeout), the results collected, and the answer synthesised from as many chunks as fit the context window
after the system prompt, the history and the generation budget).

Sources are callables ``(query) -> list[Document]``; ``vector_source`` wraps a chain-server VectorStore and
``llm_source`` wraps any chat model used as an answer engine (the reference's Perplexity role). A source that fails or
exceeds ``source_timeout_s`` contributes nothing. ``count_tokens`` defaults to the served model's tokenizer.
"""
from __future__ import annotations

import re
import time
from concurrent.futures import ThreadPoolExecutor
from concurrent.futures import TimeoutError as FutureTimeout
from dataclasses import dataclass, field
from typing import Callable, Dict, Iterator, List, Optional

from ...index.hbm_index import Document

ROUTE = ("Decide whether answering the user's message needs the document database / search sources (product "
         "documentation, general knowledge on the web). Small talk, requests about the conversation itself, and tasks "
         "on text the user supplied (proof-reading, debugging given code, counting) do not. Reply with exactly "
         "'use_search: true' or 'use_search: false'.")
REWRITE = ("Turn the user's text into the most informative keyword search query: drop formatting instructions "
           "(tables, emails, summaries), expand acronyms, add important keywords, and use the previous question when "
           "the text refers to it. Reply with the query only.")
SYSTEM = ("You are a helpful agent. Be brief and to the point; say you don't know rather than invent facts not in the "
          "documents; prefer newer information when documents carry dates; only make a table when asked.\n\n"
          "Relevant documents:\n{context}\n\nConversation so far:\n{history}")


@dataclass
class RoutedAnswer:
    use_search: bool
    query: str
    documents: List[Document] = field(default_factory=list)
    timings: Dict[str, float] = field(default_factory=dict)
    stream: Optional[Iterator[str]] = None

    def text(self) -> str:
        return "".join(self.stream or [])


def vector_source(store, k: int = 5) -> Callable[[str], List[Document]]:
    def search(q: str) -> List[Document]:
        if len(store) == 0:
            return []
        return [Document(d.page_content, dict(d.metadata, relevance_score=float(s), source_name="vectorstore"))
                for d, s in store.similarity_search_with_relevance_scores(q, k)]
    return search


def llm_source(llm, name: str = "web") -> Callable[[str], List[Document]]:
    def ask(q: str) -> List[Document]:
        r = llm.invoke([{"role": "system", "content": "Be precise and concise."}, {"role": "user", "content": q}],
                       temperature=0.0, max_tokens=512)
        text = (getattr(r, "content", r) or "").strip()
        return [Document(text, {"source_name": name, "relevance_score": 0.5})] if text else []
    return ask


def parse_route(text: str) -> bool:
    m = re.search(r"use_search\s*[:=]\s*(true|false)", (text or "").lower()) or \
        re.search(r"\b(true|false|yes|no)\b", (text or "").lower())
    return True if m is None else m.group(1) in ("true", "yes")  # unparseable: search (safer than guessing)


class RoutedRag:
    def __init__(self, llm, sources: Dict[str, Callable[[str], List[Document]]], routing_llm=None,
                 context_window: int = 8192, max_tokens: int = 1024, n_history: int = 6,
                 source_timeout_s: float = 20.0, count_tokens: Optional[Callable[[str], int]] = None):
        self.llm, self.router, self.sources = llm, routing_llm or llm, dict(sources)
        self.context_window, self.max_tokens, self.n_history = context_window, max_tokens, n_history
        self.timeout = source_timeout_s
        tok = getattr(getattr(llm, "engine", None), "tokenizer", None)
        self.count = count_tokens or ((lambda s: len(tok.encode(s))) if tok is not None
                                      else (lambda s: max(1, len(s) // 4)))
        # several workers per source: concurrent requests (and a source call still running past its timeout) must not
        # queue the next request's calls behind them, or every later gather would time out too
        self.pool = ThreadPoolExecutor(max_workers=max(16, 8 * len(self.sources)))

    def _ask(self, llm, system: str, user: str, max_tokens: int) -> str:
        r = llm.invoke([{"role": "system", "content": system}, {"role": "user", "content": user}], temperature=0.0,
                       max_tokens=max_tokens)
        return getattr(r, "content", r) or ""

    def route(self, query: str) -> bool:
        return parse_route(self._ask(self.router, ROUTE, query, 16))

    def rewrite(self, query: str, messages: List[dict]) -> str:
        prev = [m["content"] for m in messages[:-1] if m.get("role") == "user"][-1:]
        user = (f"Previous question: {prev[0]}\n" if prev else "") + f"Text: {query}"
        out = self._ask(self.llm, REWRITE, user, 96).strip().strip('"').splitlines()
        return out[0].strip() if out and out[0].strip() else query

    def gather(self, query: str) -> Dict[str, List[Document]]:
        futs = {name: self.pool.submit(fn, query) for name, fn in self.sources.items()}
        out, t_end = {}, time.monotonic() + self.timeout
        for name, f in futs.items():
            try:
                out[name] = f.result(timeout=max(0.0, t_end - time.monotonic()))
            except FutureTimeout:
                out[name] = []
            except Exception:  # noqa: BLE001 - a failing source contributes nothing
                out[name] = []
        return out

    def pack(self, docs: List[Document], history: str, query: str) -> List[Document]:
        """Chunks in order until the window (prompt + history + query + generation budget) is full."""
        used = self.count(SYSTEM.format(context="", history=history)) + self.count(query) + self.max_tokens
        kept = []
        for d in docs:
            n = self.count(f"Source text: {d.page_content}\n")
            if used + n > self.context_window:
                break
            kept.append(d)
            used += n
        return kept

    def answer(self, messages: List[dict]) -> RoutedAnswer:
        query = messages[-1]["content"]
        t0 = time.perf_counter()
        use = self.route(query)
        res = RoutedAnswer(use, query, timings={"route_s": time.perf_counter() - t0})
        hist_msgs = messages[-self.n_history - 1:-1]
        history = "".join(f"{m['role']}: {m['content']}\n" for m in hist_msgs)
        if use:
            t1 = time.perf_counter()
            res.query = self.rewrite(query, messages)
            res.timings["rewrite_s"] = time.perf_counter() - t1
            t2 = time.perf_counter()
            got = self.gather(res.query)
            res.timings["retrieve_s"] = time.perf_counter() - t2
            docs = [d for name in self.sources for d in got.get(name, [])]
            res.documents = self.pack(docs, history, query)
        ctx = "".join(f"Source text: {d.page_content}\n" for d in res.documents)
        msgs = [{"role": "system", "content": SYSTEM.format(context=ctx or "(none)", history=history or "(none)")},
                {"role": "user", "content": query}]
        res.stream = iter(self.llm.stream(msgs, temperature=0.2, max_tokens=self.max_tokens))
        return res
