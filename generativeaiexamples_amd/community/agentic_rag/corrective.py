"""Self-corrective RAG over log files (reference: /root/reference/community/log_analysis_multi_agent_rag -
multiagent.py:11-42 hybrid BM25 + dense ensemble retriever over the split log, graphnodes.py:11-70 retrieve / rerank /
grade documents / generate / transform query, graphedges.py:3-59 the two routing decisions, bat_ai.py:29-61 the graph,
utils.py:21-60 the grader chains with yes/no structured outputs).

Flow: retrieve -> rerank -> grade_documents -(none relevant)-> transform_query -> retrieve ...
                                          -(some relevant)-> generate -> grade_generation -> END | transform_query |
                                                                                               generate (ungrounded)
Every document grade of one pass is issued concurrently (one decode batch on the in-process engine). Loops are bounded:
after ``max_transforms`` rewrites the flow generates with what it has and accepts the answer, and an answer judged
ungrounded is regenerated at most ``max_regenerations`` times.
"""
from __future__ import annotations

import re
from concurrent.futures import ThreadPoolExecutor
from typing import List, Optional

from ...chain_server.connectors import rerank
from ...index.hbm_index import Document
from ...rag.text_splitter import RecursiveCharacterTextSplitter
from .graph import END, START, StateGraph

QA_SYSTEM = ("You are an expert in analysing system and application logs. Answer the question from the log excerpts "
             "given as context: name the errors, their likely root causes and concrete fixes. If the excerpts do not "
             "contain the answer, say so.")
GRADE_DOC = ("You judge whether a retrieved log excerpt is relevant to a question. It is relevant if it contains "
             "keywords, errors or events related to the question. Reply with one word: yes or no.")
GRADE_GROUNDED = ("You judge whether an answer is grounded in, and supported by, the given log excerpts. Reply with one "
                  "word: yes or no.")
GRADE_ANSWER = "You judge whether an answer resolves the question. Reply with one word: yes or no."
REWRITE = ("Rewrite the question into a better search query for retrieving relevant log lines: keep error names, "
           "component names and identifiers, add likely log keywords. Reply with the query only.")


def _yes(text: str) -> Optional[bool]:
    m = re.search(r"\b(yes|no)\b", (getattr(text, "content", text) or "").lower())
    return None if m is None else m.group(1) == "yes"


class HybridLogRetriever:
    """A log file split into overlapping chunks in a hybrid (BM25 + HBM-cosine, RRF-fused) collection."""

    def __init__(self, embeddings, text: str = "", path: Optional[str] = None, chunk_size: int = 2000,
                 chunk_overlap: int = 500, device=None, name: str = "logs"):
        from ...chain_server.vectorstore import VectorStore

        if path is not None:
            with open(path, errors="replace") as f:
                text = f.read()
        self.store = VectorStore(name, embeddings, device=device, hybrid=True)
        chunks = RecursiveCharacterTextSplitter(chunk_size, chunk_overlap).split_text(text)
        if chunks:
            self.store.add_documents([Document(c, {"source": path or name, "chunk": i}) for i, c in enumerate(chunks)])

    def __call__(self, query: str, k: int = 4) -> List[Document]:
        if len(self.store) == 0:
            return []
        return [Document(d.page_content, dict(d.metadata, relevance_score=float(s)))
                for d, s in self.store.hybrid_search(query, k)]


class CorrectiveRag:
    def __init__(self, llm, retriever, ranker=None, k: int = 4, max_transforms: int = 2, max_regenerations: int = 1,
                 check_grounding: bool = True):
        self.llm, self.retriever, self.ranker, self.k = llm, retriever, ranker, k
        self.max_transforms, self.max_regen, self.check_grounding = max_transforms, max_regenerations, check_grounding
        g = StateGraph()
        g.add_node("retrieve", self.retrieve).add_node("rerank", self.rerank)
        g.add_node("grade_documents", self.grade_documents).add_node("generate", self.generate)
        g.add_node("transform_query", self.transform_query)
        g.add_edge(START, "retrieve").add_edge("retrieve", "rerank").add_edge("rerank", "grade_documents")
        g.add_conditional_edges("grade_documents", self.decide_to_generate,
                                {"transform_query": "transform_query", "generate": "generate"})
        g.add_edge("transform_query", "retrieve")
        g.add_conditional_edges("generate", self.grade_generation,
                                {"not supported": "generate", "useful": END, "not useful": "transform_query"})
        self.graph = g.compile(max_steps=6 * (max_transforms + max_regenerations + 2))

    def _ask(self, system: str, user: str, max_tokens: int = 8) -> str:
        r = self.llm.invoke([{"role": "system", "content": system}, {"role": "user", "content": user}],
                            temperature=0.0, max_tokens=max_tokens)
        return getattr(r, "content", r) or ""

    # ---- nodes
    def retrieve(self, s: dict) -> dict:
        return {"documents": self.retriever(s["question"], self.k)}

    def rerank(self, s: dict) -> dict:
        docs = s["documents"]
        if self.ranker is None or not docs:
            return {}
        return {"documents": rerank(self.ranker, docs, s["question"], len(docs))}

    def grade_documents(self, s: dict) -> dict:
        docs = s["documents"]
        if not docs:
            return {"documents": []}
        with ThreadPoolExecutor(max_workers=min(32, len(docs))) as ex:
            grades = list(ex.map(lambda d: _yes(self._ask(
                GRADE_DOC, f"Log excerpt:\n{d.page_content}\n\nQuestion: {s['question']}")), docs))
        return {"documents": [d for d, ok in zip(docs, grades) if ok]}

    def transform_query(self, s: dict) -> dict:
        q = self._ask(REWRITE, s["question"], max_tokens=96).strip().splitlines()
        return {"question": (q[0].strip() if q and q[0].strip() else s["question"]),
                "transform_count": s.get("transform_count", 0) + 1}

    def generate(self, s: dict) -> dict:
        ctx = "\n\n".join(d.page_content for d in s["documents"])
        ans = self._ask(QA_SYSTEM, f"Context:\n{ctx}\n\nQuestion: {s['original_question']}", max_tokens=768)
        return {"generation": ans.strip(), "generations": s.get("generations", 0) + 1}

    # ---- edges
    def decide_to_generate(self, s: dict) -> str:
        if s.get("transform_count", 0) >= self.max_transforms:
            return "generate"
        return "generate" if s["documents"] else "transform_query"

    def grade_generation(self, s: dict) -> str:
        ctx = "\n\n".join(d.page_content for d in s["documents"])
        if self.check_grounding and s["documents"] and s.get("generations", 0) <= self.max_regen:
            grounded = _yes(self._ask(GRADE_GROUNDED, f"Log excerpts:\n{ctx}\n\nAnswer: {s['generation']}"))
            if grounded is False:
                return "not supported"
        useful = _yes(self._ask(GRADE_ANSWER, f"Question: {s['original_question']}\n\nAnswer: {s['generation']}"))
        if useful is False and s.get("transform_count", 0) < self.max_transforms:
            return "not useful"
        return "useful"  # unparseable grades are accepted, as the reference does, so the flow always ends

    def run(self, question: str) -> dict:
        return self.graph.invoke({"question": question, "original_question": question, "documents": [],
                                  "transform_count": 0, "generations": 0})
