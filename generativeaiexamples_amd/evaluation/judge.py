"""LLM-as-judge evaluation (T3; reference eval_llm_judge, rag_evaluator/evaluator.py:165-235): a Likert 1-5
rating + explanation per row in a JSON reply; ratings of 0 count as 1, unparseable replies are
dropped from the mean; results written as JSON."""
from __future__ import annotations

import json
import re
import statistics
from typing import Dict, List

SYS_PROMPT = (
    "You are an impartial judge that evaluates the quality of an assistant's answer to the question provided. "
    "Rate the answer on a Likert scale from 1 to 5 (1 = wrong or irrelevant, 5 = fully correct, complete and "
    "grounded). You must use both the reference context and the reference answer to guide your evaluation. "
    "Reply strictly as JSON: {\"Rating\": <1-5>, \"Explanation\": \"<one or two sentences>\"}.")

TEMPLATE = ("[The Start of Reference Context]\n{ctx}\n[The End of Reference Context]\n"
            "[Question]\n{q}\n[The Start of Reference Answer]\n{ref}\n[The End of Reference Answer]\n"
            "[The Start of Assistant's Answer]\n{ans}\n[The End of Assistant's Answer]")


def parse_rating(reply: str):
    try:
        obj = json.loads(reply[reply.index("{"): reply.rindex("}") + 1])
        r = int(obj.get("Rating", obj.get("rating")))
        return max(1, min(5, r if r != 0 else 1)), str(obj.get("Explanation", obj.get("Explanantion", "")))
    except (ValueError, TypeError, KeyError):
        m = re.search(r"[Rr]ating\D{0,5}([0-5])", reply)
        return (max(1, int(m.group(1))), reply.strip()) if m else (None, reply.strip())


def eval_llm_judge(ev_file: str, ev_result: str, llm) -> Dict:
    with open(ev_file, encoding="utf-8") as f:
        data = json.load(f)
    rows: List[Dict] = []
    for d in data:
        ref = d.get("gt_answer", d.get("ground_truth_answer", ""))
        ctx = d.get("gt_context", d.get("ground_truth_context", ""))
        reply = llm([{"role": "system", "content": SYS_PROMPT},
                     {"role": "user", "content": TEMPLATE.format(ctx=ctx, q=d["question"], ref=ref, ans=d.get("answer", ""))}])
        rating, expl = parse_rating(reply)
        rows.append({"question": d["question"], "answer": d.get("answer", ""), "gt_answer": ref, "rating": rating,
                     "explanation": expl})
    rated = [r["rating"] for r in rows if r["rating"]]
    out = {"num_judgements": len(rows), "num_ratings": len(rated),
           "mean_rating": round(statistics.fmean(rated), 1) if rated else None, "rows": rows}
    with open(ev_result + ".json", "w", encoding="utf-8") as f:
        json.dump(out, f, indent=2)
    return out
