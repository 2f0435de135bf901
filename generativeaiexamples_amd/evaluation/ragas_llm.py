"""LLM-judged RAGAS metrics (the algorithms of ragas 0.1.x, which the reference runs in
RAG/tools/evaluation/rag_evaluator/evaluator.py:97-162 with an API-catalog LLM + embeddings).

ragas itself is not installable offline, so its six metrics are re-implemented on this framework's own
served models. Every judge call asks for JSON under a ``response_format: json_schema`` - the model server
enforces it with constrained decoding (engine/guided.py), so the judge output always parses, where
ragas retries on "Invalid JSON response" (the reference README's known warning):

  faithfulness       the answer is split into atomic statements (LLM), each statement gets an NLI verdict
                     against the retrieved contexts (LLM); score = supported / statements
  answer_relevancy   the LLM writes ``n`` questions the answer would answer (+ a noncommittal flag);
                     score = mean cos(emb(question), emb(generated)), 0 if the answer is noncommittal
  context_precision  per retrieved context (in rank order) a verdict "useful for the ground-truth answer";
                     score = average precision sum_k(P@k * v_k) / sum_k v_k
  context_recall     each ground-truth-answer sentence is classified as attributable to the contexts;
                     score = attributed / sentences
  context_relevancy  the LLM extracts the context sentences needed to answer the question;
                     score = extracted / context sentences
  answer_similarity  cos(emb(answer), emb(ground truth))
  ragas_score        harmonic mean of faithfulness, context_relevancy, answer_relevancy, context_recall
                     (evaluator.py:92-94)

Numeric parity with ragas' own prompts is unpinned (different judge model, prompts re-written here); the
algorithmic definitions are the same.
"""
from __future__ import annotations

import json
import math
import re
import statistics
from typing import Callable, Dict, List, Optional, Sequence

JudgeFn = Callable[..., str]  # (messages, schema=None) -> str

_SENT = re.compile(r"(?<=[.!?])\s+|\n+")

S_STATEMENTS = {"type": "object", "properties": {"statements": {"type": "array", "items": {"type": "string"}}},
                "required": ["statements"]}
S_VERDICTS = {"type": "object", "properties": {"verdicts": {"type": "array", "items": {
    "type": "object", "properties": {"statement": {"type": "string"}, "verdict": {"type": "integer", "enum": [0, 1]}},
    "required": ["statement", "verdict"]}}}, "required": ["verdicts"]}
S_QUESTION = {"type": "object", "properties": {"question": {"type": "string"},
                                               "noncommittal": {"type": "integer", "enum": [0, 1]}},
              "required": ["question", "noncommittal"]}
S_VERDICT = {"type": "object", "properties": {"reason": {"type": "string"}, "verdict": {"type": "integer", "enum": [0, 1]}},
             "required": ["reason", "verdict"]}
S_ATTRIB = {"type": "object", "properties": {"classifications": {"type": "array", "items": {
    "type": "object", "properties": {"statement": {"type": "string"}, "attributed": {"type": "integer", "enum": [0, 1]}},
    "required": ["statement", "attributed"]}}}, "required": ["classifications"]}
S_SENTENCES = {"type": "object", "properties": {"sentences": {"type": "array", "items": {"type": "string"}}},
               "required": ["sentences"]}


def sentences(text: str) -> List[str]:
    return [s.strip() for s in _SENT.split(text or "") if s.strip()]


def _cos(a, b) -> float:
    na = math.sqrt(sum(x * x for x in a)) or 1.0
    nb = math.sqrt(sum(x * x for x in b)) or 1.0
    return sum(x * y for x, y in zip(a, b)) / (na * nb)


def _json(text: str):
    """The constrained server returns bare JSON; tolerate a prose wrapper from unconstrained judges."""
    try:
        return json.loads(text)
    except (json.JSONDecodeError, TypeError):
        m = re.search(r"\{.*\}", text or "", re.S)
        if m:
            try:
                return json.loads(m.group(0))
            except json.JSONDecodeError:
                return None
    return None


def _ask(llm: JudgeFn, system: str, user: str, schema: dict):
    try:
        return _json(llm([{"role": "system", "content": system}, {"role": "user", "content": user}], schema=schema))
    except TypeError:  # a judge callable without structured output
        return _json(llm([{"role": "system", "content": system + " Reply with JSON only."},
                          {"role": "user", "content": user}]))


class RagasJudge:
    def __init__(self, llm: JudgeFn, embed: Optional[Callable[[List[str]], List[List[float]]]] = None,
                 n_questions: int = 3):
        self.llm, self.embed, self.n = llm, embed, n_questions

    # ------------------------------------------------------------------ metrics
    def faithfulness(self, q: str, a: str, ctxs: Sequence[str]) -> float:
        st = _ask(self.llm, "Break the answer into short, self-contained factual statements.",
                  f"Question: {q}\nAnswer: {a}\nReturn {{\"statements\": [...]}}.", S_STATEMENTS)
        stmts = [s for s in (st or {}).get("statements", []) if isinstance(s, str) and s.strip()]
        if not stmts:
            stmts = sentences(a)
        if not stmts:
            return 0.0
        ctx = "\n".join(ctxs)
        v = _ask(self.llm, "You judge natural-language inference. For each statement decide whether it can be "
                           "directly inferred from the context (verdict 1) or not (verdict 0).",
                 f"Context:\n{ctx}\n\nStatements:\n" + "\n".join(f"- {s}" for s in stmts), S_VERDICTS)
        verdicts = [int(x.get("verdict", 0)) for x in (v or {}).get("verdicts", []) if isinstance(x, dict)]
        verdicts = (verdicts + [0] * len(stmts))[:len(stmts)]
        return sum(verdicts) / len(stmts)

    def answer_relevancy(self, q: str, a: str) -> float:
        if self.embed is None:
            raise ValueError("answer_relevancy needs an embedding model")
        gens, noncommittal = [], False
        for i in range(self.n):
            r = _ask(self.llm, "Write the question that the given answer answers. Mark noncommittal = 1 if the "
                               "answer is evasive or vague (e.g. 'I don't know').",
                     f"Answer: {a}\n(variant {i + 1})", S_QUESTION) or {}
            if isinstance(r.get("question"), str) and r["question"].strip():
                gens.append(r["question"])
            noncommittal |= bool(r.get("noncommittal", 0))
        if not gens:
            return 0.0
        e = self.embed([q] + gens)
        return 0.0 if noncommittal else max(0.0, statistics.fmean(_cos(e[0], x) for x in e[1:]))

    def context_precision(self, q: str, gt: str, ctxs: Sequence[str]) -> float:
        v = []
        for c in ctxs:
            r = _ask(self.llm, "Decide whether the context was useful in arriving at the given answer "
                               "(verdict 1) or not (verdict 0).",
                     f"Question: {q}\nContext: {c}\nAnswer: {gt}", S_VERDICT) or {}
            v.append(int(r.get("verdict", 0)))
        if not sum(v):
            return 0.0
        hits, num = 0, 0.0
        for k, x in enumerate(v, 1):
            hits += x
            num += (hits / k) * x
        return num / sum(v)

    def context_recall(self, q: str, gt: str, ctxs: Sequence[str]) -> float:
        sents = sentences(gt)
        if not sents:
            return 0.0
        r = _ask(self.llm, "For each sentence of the answer decide whether it can be attributed to the "
                           "context (attributed 1) or not (attributed 0).",
                 f"Question: {q}\nContext:\n" + "\n".join(ctxs) + "\n\nAnswer sentences:\n"
                 + "\n".join(f"- {s}" for s in sents), S_ATTRIB) or {}
        att = [int(x.get("attributed", 0)) for x in r.get("classifications", []) if isinstance(x, dict)]
        att = (att + [0] * len(sents))[:len(sents)]
        return sum(att) / len(sents)

    def context_relevancy(self, q: str, ctxs: Sequence[str]) -> float:
        cs = [s for c in ctxs for s in sentences(c)]
        if not cs:
            return 0.0
        r = _ask(self.llm, "Extract, word for word, the sentences of the context that are needed to answer the "
                           "question. Return an empty list if none are.",
                 f"Question: {q}\nContext:\n" + "\n".join(ctxs), S_SENTENCES) or {}
        norm = {re.sub(r"\s+", " ", s).strip().lower() for s in cs}
        got = {re.sub(r"\s+", " ", s).strip().lower() for s in r.get("sentences", []) if isinstance(s, str)}
        return min(1.0, len(got & norm) / len(cs))

    def answer_similarity(self, a: str, gt: str) -> float:
        if self.embed is None:
            raise ValueError("answer_similarity needs an embedding model")
        e = self.embed([a, gt])
        return max(0.0, _cos(e[0], e[1]))

    # ------------------------------------------------------------------ rows
    def score_row(self, row: Dict) -> Dict[str, float]:
        q, a = row.get("question", ""), row.get("answer", "")
        ctxs = list(row.get("contexts") or [])
        gt = row.get("gt_answer", row.get("ground_truth_answer", ""))
        out = {"faithfulness": self.faithfulness(q, a, ctxs), "context_precision": self.context_precision(q, gt, ctxs),
               "context_recall": self.context_recall(q, gt, ctxs), "context_relevancy": self.context_relevancy(q, ctxs)}
        if self.embed is not None:
            out["answer_relevancy"] = self.answer_relevancy(q, a)
            out["answer_similarity"] = self.answer_similarity(a, gt)
        else:
            out["answer_relevancy"] = out["answer_similarity"] = 0.0
        four = [out["faithfulness"], out["context_relevancy"], out["answer_relevancy"], out["context_recall"]]
        out["ragas_score"] = statistics.harmonic_mean(four) if all(v > 0 for v in four) else 0.0
        return out
