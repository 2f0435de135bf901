"""Agentic RAG community flows (SURVEY §2.9 log_analysis_multi_agent_rag, routing-multisource-rag): the bounded state
graph, the self-corrective log RAG (grading, rewriting, regeneration, loop bounds) and routed multi-source RAG
(routing, concurrent sources with timeout, token-budgeted packing) - scripted LLMs, crc32 hashing embedder, CPU."""
import threading
import time
import zlib

import pytest
import torch

from generativeaiexamples_amd.chain_server.connectors import Embeddings
from generativeaiexamples_amd.community.agentic_rag import (END, START, CorrectiveRag, GraphRecursionError,
                                                            HybridLogRetriever, RoutedRag, StateGraph, llm_source,
                                                            parse_route)
from generativeaiexamples_amd.community.agentic_rag import corrective as cr
from generativeaiexamples_amd.community.agentic_rag import routing as rt
from generativeaiexamples_amd.index.hbm_index import Document

LOG = "\n".join([
    "2024-05-01 10:00:01 INFO service started on port 8080",
    "2024-05-01 10:00:05 INFO connected to database replica-2",
    "2024-05-01 10:03:17 ERROR OutOfMemoryError in worker-7 while allocating tensor buffer of 4 GB",
    "2024-05-01 10:03:18 WARN worker-7 restarting after OutOfMemoryError",
    "2024-05-01 10:07:42 ERROR connection refused by database replica-2 timeout after 30s",
] * 3)


class _Emb(Embeddings):
    dim = 64

    def embed_tensor(self, texts, input_type):
        out = torch.zeros(len(texts), self.dim)
        for i, t in enumerate(texts):
            for w in t.lower().split():
                out[i, zlib.crc32(w.strip(".,?:").encode()) % self.dim] += 1.0
        return torch.nn.functional.normalize(out + 1e-3, dim=-1)


def test_state_graph_basics():
    g = StateGraph()
    g.add_node("a", lambda s: {"n": s["n"] + 1}).add_node("b", lambda s: {"n": s["n"] * 10})
    g.add_edge(START, "a").add_conditional_edges("a", lambda s: "again" if s["n"] < 3 else "done",
                                                 {"again": "a", "done": "b"})
    g.add_edge("b", END)
    out = g.compile().invoke({"n": 0})
    assert out["n"] == 30 and out["trace"] == ["a", "a", "a", "b"]
    with pytest.raises(GraphRecursionError):
        g.compile(max_steps=2).invoke({"n": 0})
    with pytest.raises(ValueError):
        StateGraph().add_node("x", lambda s: None).add_edge("x", "missing").add_edge(START, "x").compile()
    bad = StateGraph().add_node("x", lambda s: None)
    bad.add_edge(START, "x").add_conditional_edges("x", lambda s: "?", {"ok": END})
    with pytest.raises(KeyError):
        bad.compile().invoke({})


class _LogLLM:
    """Grades documents by keyword; scripted rewrite / grounding / usefulness answers."""

    def __init__(self, relevant_word="outofmemoryerror", grounded=("yes",), useful=("yes",)):
        self.word, self.grounded, self.useful = relevant_word, list(grounded), list(useful)
        self.lock, self.inflight, self.peak, self.calls = threading.Lock(), 0, 0, []

    def invoke(self, messages, **kw):
        with self.lock:
            self.inflight += 1
            self.peak = max(self.peak, self.inflight)
        try:
            sys_, user = messages[0]["content"], messages[-1]["content"]
            self.calls.append(sys_[:12])
            if sys_ == cr.GRADE_DOC:
                time.sleep(0.02)
                excerpt = user.split("Question:")[0].lower()
                return "yes" if self.word and self.word in excerpt else "no"
            if sys_ == cr.REWRITE:
                self.word = "outofmemoryerror"  # the rewritten query finds the OOM lines
                return "OutOfMemoryError worker restart"
            if sys_ == cr.GRADE_GROUNDED:
                return self.grounded.pop(0) if self.grounded else "yes"
            if sys_ == cr.GRADE_ANSWER:
                return self.useful.pop(0) if self.useful else "yes"
            return "worker-7 ran out of memory allocating a 4 GB tensor buffer; raise its memory limit."
        finally:
            with self.lock:
                self.inflight -= 1


def _retriever():
    return HybridLogRetriever(_Emb(), text=LOG, chunk_size=160, chunk_overlap=0, device="cpu")


def test_corrective_rag_direct_path():
    llm = _LogLLM()
    out = CorrectiveRag(llm, _retriever(), k=4).run("Why did worker-7 crash with OutOfMemoryError?")
    assert out["trace"] == ["retrieve", "rerank", "grade_documents", "generate"]
    assert out["documents"] and all("outofmemoryerror" in d.page_content.lower() for d in out["documents"])
    assert "4 GB" in out["generation"] and llm.peak >= 2  # grades issued concurrently


def test_corrective_rag_rewrites_then_regenerates():
    llm = _LogLLM(relevant_word=None, grounded=("no", "yes"))
    out = CorrectiveRag(llm, _retriever(), k=3).run("what went wrong?")
    assert out["trace"] == ["retrieve", "rerank", "grade_documents", "transform_query", "retrieve", "rerank",
                            "grade_documents", "generate", "generate"]
    assert out["question"] == "OutOfMemoryError worker restart" and out["transform_count"] == 1
    assert out["generations"] == 2


def test_corrective_rag_bounded_when_nothing_relevant():
    class Never(_LogLLM):
        def invoke(self, messages, **kw):
            if messages[0]["content"] == cr.REWRITE:
                return "still nothing"
            if messages[0]["content"] == cr.GRADE_ANSWER:
                return "no"
            return super().invoke(messages, **kw)

    out = CorrectiveRag(Never(relevant_word=None), _retriever(), k=2, max_transforms=2).run("q")
    assert out["transform_count"] == 2 and out["trace"][-1] == "generate" and out["documents"] == []


def test_routed_rag_search_and_shortcut():
    class LLM:
        def __init__(self):
            self.seen = []

        def invoke(self, messages, **kw):
            sys_ = messages[0]["content"]
            if sys_ == rt.ROUTE:
                return "use_search: false" if "hello" in messages[-1]["content"].lower() else "use_search: true"
            if sys_ == rt.REWRITE:
                self.seen.append(messages[-1]["content"])
                return '"MI355X HBM3E memory capacity"'
            return "web says 288 GB"

        def stream(self, messages, **kw):
            self.seen.append(messages[0]["content"])
            yield "ok"

    class Store:
        def __len__(self):
            return 2

        def similarity_search_with_relevance_scores(self, q, k):
            return [(Document("A" * 400, {}), 0.9), (Document("B" * 400, {}), 0.8)]

    def slow(q):
        time.sleep(2.0)
        return [Document("late", {})]

    llm = LLM()
    rag = RoutedRag(llm, {"vectorstore": rt.vector_source(Store()), "web": llm_source(llm), "slow": slow},
                    context_window=300, max_tokens=100, source_timeout_s=0.5, count_tokens=lambda s: len(s) // 4)
    msgs = [{"role": "user", "content": "how much memory?"}, {"role": "assistant", "content": "which GPU?"},
            {"role": "user", "content": "the MI355X"}]
    t0 = time.perf_counter()
    res = rag.answer(msgs)
    assert time.perf_counter() - t0 < 1.8  # the slow source timed out instead of blocking
    assert res.use_search and res.query == "MI355X HBM3E memory capacity"
    assert "Previous question: how much memory?" in llm.seen[0]
    # window 300 - generation 100 - prompt/history: only the first 400-char chunk (~100 tokens) fits
    assert [d.page_content[:1] for d in res.documents] == ["A"]
    assert res.text() == "ok" and "Source text: AAAA" in llm.seen[-1]
    res = rag.answer([{"role": "user", "content": "Hello!"}])
    assert not res.use_search and res.documents == [] and res.text() == "ok" and "(none)" in llm.seen[-1]


def test_parse_route():
    assert parse_route("use_search: true") and not parse_route("use_search: False")
    assert not parse_route("No.") and parse_route("I am not sure")
