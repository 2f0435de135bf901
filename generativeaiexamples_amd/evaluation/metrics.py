"""RAGAS-style RAG metrics computed with this framework's own models (T3; the reference calls ragas 0.1.7
with an API-catalog LLM + embeddings, rag_evaluator/evaluator.py:97-162 - ragas is not available
offline, so the six metrics are re-defined here; numeric parity with ragas is unpinned).

Per row (question, answer, contexts, gt_answer, gt_context), every score in [0, 1]:
  answer_similarity  cos(emb(answer), emb(gt_answer)) clipped at 0
  faithfulness       fraction of answer statements supported by the retrieved contexts
  context_precision  rank-weighted precision of the retrieved contexts w.r.t. the ground-truth context
  context_relevancy  fraction of context sentences relevant to the question
  answer_relevancy   cos(emb(question), emb(answer)) clipped at 0
  context_recall     fraction of ground-truth-answer statements supported by the retrieved contexts
  ragas_score        harmonic mean of faithfulness, context_relevancy, answer_relevancy, context_recall
                     (reference calculate_ragas_score, evaluator.py:92-94)
"Supported" is lexical entailment: >= ``support`` of a statement's content words occur in the
evidence. These word-overlap scores are the offline fallback (``--lexical_ragas``); with a judge LLM,
``eval_ragas`` runs the ragas algorithms themselves (evaluation/ragas_llm.py: statement extraction + NLI
verdicts, generated-question relevancy, LLM-judged precision / recall / relevancy).
"""
from __future__ import annotations

import json
import math
import re
import statistics
from typing import Callable, Dict, List, Optional, Sequence

_STOP = set("a an the of to in on for and or is are was were be been it this that with as by at from what which "
            "who whom how why when where does do did not no can could should would will shall may might".split())
_SENT = re.compile(r"(?<=[.!?])\s+|\n+")
_WORD = re.compile(r"[a-z0-9]+")


def statements(text: str) -> List[str]:
    return [s.strip() for s in _SENT.split(text or "") if len(_WORD.findall(s.lower())) >= 2]


def content_words(text: str) -> set:
    return {w for w in _WORD.findall((text or "").lower()) if w not in _STOP}


def supported(stmt: str, evidence_words: set, support: float = 0.5) -> bool:
    w = content_words(stmt)
    return bool(w) and len(w & evidence_words) / len(w) >= support


def _cos(a, b) -> float:
    na = math.sqrt(sum(x * x for x in a)) or 1.0
    nb = math.sqrt(sum(x * x for x in b)) or 1.0
    return max(0.0, sum(x * y for x, y in zip(a, b)) / (na * nb))


def _judge_yes(llm, stmt: str, evidence: str) -> bool:
    r = llm([{"role": "system", "content": "Answer only 'yes' or 'no'."},
             {"role": "user", "content": f"Context:\n{evidence}\n\nStatement: {stmt}\n"
                                         f"Can the statement be inferred from the context?"}])
    return r.strip().lower().startswith("yes")


def score_row(row: Dict, embed: Optional[Callable[[List[str]], List[List[float]]]] = None,
              llm=None, support: float = 0.5) -> Dict[str, float]:
    q, a = row.get("question", ""), row.get("answer", "")
    ctxs = list(row.get("contexts") or [])
    gt_a = row.get("gt_answer", row.get("ground_truth_answer", ""))
    gt_c = row.get("gt_context", row.get("ground_truth_context", ""))
    ev = "\n".join(ctxs)
    evw = content_words(ev)

    def frac_supported(text):
        st = statements(text)
        if not st:
            return 0.0
        ok = [(_judge_yes(llm, s, ev) if llm else supported(s, evw, support)) for s in st]
        return sum(ok) / len(st)

    out = {"faithfulness": frac_supported(a), "context_recall": frac_supported(gt_a)}
    gtw = content_words(gt_c)
    hits, prec = 0, []
    for k, c in enumerate(ctxs, 1):
        cw = content_words(c)
        rel = bool(cw) and len(cw & gtw) / len(cw) >= support
        hits += rel
        if rel:
            prec.append(hits / k)
    out["context_precision"] = sum(prec) / max(1, hits) if hits else 0.0
    qw = content_words(q)
    cs = [s for c in ctxs for s in statements(c)]
    out["context_relevancy"] = (sum(bool(content_words(s) & qw) for s in cs) / len(cs)) if cs else 0.0
    if embed is not None:
        e = embed([q, a, gt_a])
        out["answer_relevancy"], out["answer_similarity"] = _cos(e[0], e[1]), _cos(e[1], e[2])
    else:
        aw, gw = content_words(a), content_words(gt_a)
        out["answer_relevancy"] = len(aw & qw) / len(qw) if qw else 0.0
        out["answer_similarity"] = len(aw & gw) / len(aw | gw) if (aw | gw) else 0.0
    four = [out["faithfulness"], out["context_relevancy"], out["answer_relevancy"], out["context_recall"]]
    out["ragas_score"] = statistics.harmonic_mean(four) if all(v > 0 for v in four) else 0.0
    return out


METRIC_NAMES = ("answer_similarity", "faithfulness", "context_precision", "context_relevancy", "answer_relevancy",
                "context_recall", "ragas_score")


def eval_ragas(ev_file: str, ev_result: str, embed=None, llm=None) -> Dict[str, float]:
    """Score every row of the eval JSON; writes ``<ev_result>.json`` (aggregate) and
    ``<ev_result>.rows.json`` (per row; the reference writes a parquet of the same table)."""
    with open(ev_file, encoding="utf-8") as f:
        data = json.load(f)
    if llm is not None:  # the ragas algorithms with a judge LLM (evaluation/ragas_llm.py)
        from .ragas_llm import RagasJudge

        judge = RagasJudge(llm, embed)
        rows = [dict(d, **judge.score_row(d)) for d in data]
    else:
        rows = [dict(d, **score_row(d, embed)) for d in data]
    agg = {m: statistics.fmean(r[m] for r in rows) for m in METRIC_NAMES if rows}
    four = [agg.get(k, 0.0) for k in ("faithfulness", "context_relevancy", "answer_relevancy", "context_recall")]
    agg["ragas_score"] = statistics.harmonic_mean(four) if all(v > 0 for v in four) else 0.0
    with open(ev_result + ".json", "w", encoding="utf-8") as f:
        json.dump(agg, f, indent=2)
    with open(ev_result + ".rows.json", "w", encoding="utf-8") as f:
        json.dump(rows, f, indent=2)
    return agg


def aggregate(rows: Sequence[Dict]) -> Dict[str, float]:
    return {m: statistics.fmean(r[m] for r in rows) for m in METRIC_NAMES}
