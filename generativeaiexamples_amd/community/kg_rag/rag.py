"""Text / graph / combined RAG answers over a knowledge graph and a hybrid vector collection (reference:
/root/reference/community/knowledge_graph_rag/backend/routers/chat.py:44-95 and routers/evaluation.py:101-194 - the
model names the question's entities, each entity's 2-hop graph facts become context, optionally together with the
top-5 hybrid (dense + sparse, RRF-fused) passages after reranking; evaluation runs all three variants per question).

``store`` is a chain-server ``VectorStore`` (``hybrid=True`` gives the BM25 + HBM-cosine fusion the reference gets
from Milvus' sparse + dense search); ``ranker`` an optional chain-server reranker. When the model's entity list does
not parse, or names nothing in the graph, entities are found by matching graph node names inside the question, so a
weak model still gets graph context (the reference falls back to a "no graph triples" disclaimer).
"""
from __future__ import annotations

import ast
import json
import re
from concurrent.futures import ThreadPoolExecutor
from typing import Dict, List, Optional, Tuple

from ...chain_server.connectors import rerank
from ...index.hbm_index import Document
from .graph import KnowledgeGraph

SYSTEM = ("You are a helpful assistant. Answer only from the context you are given; if the context does not cover the "
          "question, say so politely instead of answering.")
ENTITY_PROMPT = ("List the named entities that appear in the user's question. Reply with JSON only, of the form "
                 '{"entities": ["...", "..."]}; every entity must be text taken from the question. '
                 'Example: "How does Contoso compare with Fabrikam?" -> {"entities": ["Contoso", "Fabrikam"]}')
NO_GRAPH = ("No knowledge-graph relationships were found for this question. If you answer from general knowledge, say "
            "that the answer is not grounded in the provided graph.")


def parse_entities(reply: str) -> Optional[List[str]]:
    """{"entities": [...]} or a bare list, possibly wrapped in prose or a fenced block; None if nothing parses."""
    text = getattr(reply, "content", reply) or ""
    for m in re.finditer(r"\{.*?\}|\[.*?\]", text, re.S):
        for parse in (json.loads, ast.literal_eval):
            try:
                obj = parse(m.group(0))
            except (ValueError, SyntaxError, TypeError):
                continue
            ents = obj.get("entities") if isinstance(obj, dict) else obj
            if isinstance(ents, list):
                return [str(e).strip() for e in ents if str(e).strip()]
    return None


class KGRag:
    def __init__(self, llm, graph: KnowledgeGraph, store=None, ranker=None, k: int = 5, depth: int = 2,
                 both_directions: bool = False):
        self.llm, self.graph, self.store, self.ranker = llm, graph, store, ranker
        self.k, self.depth, self.both = k, depth, both_directions

    def _ask(self, user: str, system: str = SYSTEM, **kw) -> str:
        r = self.llm.invoke([{"role": "system", "content": system}, {"role": "user", "content": user}], **kw)
        return getattr(r, "content", r)

    # ---- context builders
    def entities(self, question: str) -> List[str]:
        ents = parse_entities(self._ask(question, ENTITY_PROMPT, temperature=0.0, max_tokens=128)) or []
        known = [e for e in ents if e in self.graph]
        return known or self.graph.find_entities(question) or ents

    def graph_facts(self, question: str) -> List[str]:
        facts, seen = [], set()
        for e in self.entities(question):
            for f in self.graph.entity_knowledge(e, depth=self.depth, both_directions=self.both):
                if f not in seen:
                    seen.add(f)
                    facts.append(f)
        return facts

    def passages(self, question: str) -> List[str]:
        if self.store is None or len(self.store) == 0:
            return []
        search = getattr(self.store, "hybrid_search", None) or self.store.similarity_search_with_relevance_scores
        hits = search(question, max(self.k * 4, self.k) if self.ranker is not None else self.k)
        docs = [Document(d.page_content, dict(d.metadata, relevance_score=float(s))) for d, s in hits]
        if self.ranker is not None and docs:
            docs = rerank(self.ranker, docs, question, self.k)
        return [d.page_content for d in docs[: self.k]]

    # ---- answers: (answer, contexts)
    def _answer(self, question: str, context: str) -> str:
        return self._ask(f"Context: {context}\n\nUser query: {question}", temperature=0.2, max_tokens=512)

    def text_rag(self, question: str) -> Tuple[str, List[str]]:
        ps = self.passages(question)
        ctx = "Relevant passages from the knowledge base:\n\n" + "\n".join(ps)
        return self._answer(question, ctx), ps

    def graph_rag(self, question: str) -> Tuple[str, List[str]]:
        facts = self.graph_facts(question)
        ctx = ("Relationships from the knowledge graph:\n" + "\n".join(facts)) if facts else NO_GRAPH
        return self._answer(question, ctx), facts or ["no relationship found"]

    def combined_rag(self, question: str) -> Tuple[str, List[str]]:
        ps, facts = self.passages(question), self.graph_facts(question)
        ctx = "Relevant passages from the knowledge base:\n\n" + "\n".join(ps)
        ctx += ("\n\nRelationships from the knowledge graph:\n" + "\n".join(facts)) if facts else f"\n\n{NO_GRAPH}"
        return self._answer(question, ctx), ps + facts

    def chat(self, question: str, use_kg: bool = True) -> Dict[str, object]:
        """The reference's POST /chat/ body: graph + passages when ``use_kg``, the bare question otherwise."""
        if not use_kg:
            return {"user_input": question, "use_kg": False, "context": "",
                    "assistant_response": self._ask(question, temperature=0.2, max_tokens=512)}
        answer, ctx = self.combined_rag(question)
        return {"user_input": question, "use_kg": True, "context": "\n".join(ctx), "assistant_response": answer}

    def evaluate_question(self, question: str, gt_answer: str) -> Dict[str, object]:
        """All three variants side by side (evaluation.py process_question), run concurrently."""
        with ThreadPoolExecutor(max_workers=3) as ex:
            ft, fg, fc = (ex.submit(f, question) for f in (self.text_rag, self.graph_rag, self.combined_rag))
            (ta, tc), (ga, gc), (ca, cc) = ft.result(), fg.result(), fc.result()
        return {"question": question, "gt_answer": gt_answer, "textRAG_answer": ta, "graphRAG_answer": ga,
                "combined_answer": ca, "text_RAG_context_response": tc, "graph_RAG_context_response": gc,
                "combined_RAG_context_response": cc}
