"""advanced_rag/query_decomposition_rag (E4; reference chains.py:151-389).

A small planning agent: the LLM decomposes the question into sub-questions and picks a tool
(``Search`` over the knowledge base, ``Math`` for arithmetic, ``Nil`` when done) as JSON; each
Search sub-question retrieves context and has the LLM extract a short answer into a ledger; Math
asks the LLM for an expression that is evaluated by a restricted AST evaluator (never ``eval`` -
the reference's ``eval`` on model output is a security defect). The loop stops
on ``Nil``, a repeated sub-question or after ``max_iterations``; the final answer is streamed
from the ledger.
"""
from __future__ import annotations

import ast
import json
import logging
import operator
import re
from typing import Dict, Generator, List

from ..chain_server.utils import get_llm
from .basic_rag import BasicRAG

log = logging.getLogger(__name__)

PLANNER_PROMPT = (
    "You answer questions by breaking them into simpler sub-questions. Tools: 'Search' (look up facts in "
    "the knowledge base), 'Math' (do arithmetic on known numbers), 'Nil' (no more tools needed).\n"
    "Known so far:\n{ledger}\n\nQuestion: {question}\n"
    'Reply ONLY with JSON: {{"Tool_Request": "Search"|"Math"|"Nil", "Generated Sub Questions": [..]}}'
)
EXTRACT_PROMPT = "Using only this context, answer the question in one sentence.\nContext: {context}\nQuestion: {q}"
MATH_PROMPT = ("Write a single arithmetic expression (numbers, + - * / ** and parentheses only) that answers: "
               "{q}\nKnown facts:\n{ledger}\nReply with the expression only.")
FINAL_PROMPT = "Sub questions and answers:\n{ledger}\n\nUsing them, answer the question: {question}"

_OPS = {ast.Add: operator.add, ast.Sub: operator.sub, ast.Mult: operator.mul, ast.Div: operator.truediv,
        ast.Pow: operator.pow, ast.Mod: operator.mod, ast.FloorDiv: operator.floordiv, ast.USub: operator.neg,
        ast.UAdd: operator.pos}


def safe_math(expr: str) -> float:
    """Evaluate a pure arithmetic expression (no names, calls or attributes)."""
    expr = expr.strip().strip("`").replace("^", "**")
    tree = ast.parse(expr, mode="eval")

    def ev(n):
        if isinstance(n, ast.Expression):
            return ev(n.body)
        if isinstance(n, ast.Constant) and isinstance(n.value, (int, float)):
            return n.value
        if isinstance(n, ast.BinOp) and type(n.op) in _OPS:
            a, b = ev(n.left), ev(n.right)
            if isinstance(n.op, ast.Pow) and abs(b) > 64:
                raise ValueError("exponent too large")
            return _OPS[type(n.op)](a, b)
        if isinstance(n, ast.UnaryOp) and type(n.op) in _OPS:
            return _OPS[type(n.op)](ev(n.operand))
        raise ValueError(f"unsupported expression element: {type(n).__name__}")

    return ev(tree)


def parse_plan(text: str) -> Dict:
    m = re.search(r"\{.*\}", text, re.S)
    if not m:
        return {"Tool_Request": "Nil", "Generated Sub Questions": []}
    try:
        obj = json.loads(m.group(0))
    except json.JSONDecodeError:
        return {"Tool_Request": "Nil", "Generated Sub Questions": []}
    tool = str(obj.get("Tool_Request", "Nil")).strip().capitalize()
    subs = obj.get("Generated Sub Questions") or []
    if isinstance(subs, str):
        subs = [subs]
    return {"Tool_Request": tool if tool in ("Search", "Math", "Nil") else "Nil",
            "Generated Sub Questions": [str(s) for s in subs][:5]}


class QueryDecompositionRAG(BasicRAG):
    max_iterations = 3

    def run_agent(self, question: str, **kw) -> List[Dict[str, str]]:
        llm = get_llm(temperature=0.1, top_p=0.7, max_tokens=256)
        ledger: List[Dict[str, str]] = []
        seen = set()
        for _ in range(self.max_iterations):
            led = "\n".join(f"- {e['question']}: {e['answer']}" for e in ledger) or "(nothing yet)"
            plan = parse_plan(llm.invoke([{"role": "user", "content": PLANNER_PROMPT.format(ledger=led,
                                                                                             question=question)}]))
            subs = [s for s in plan["Generated Sub Questions"] if s not in seen]
            if plan["Tool_Request"] == "Nil" or not subs:
                break
            for q in subs:
                seen.add(q)
                if plan["Tool_Request"] == "Search":
                    hits = self.retrieve(q)
                    ctx = "\n".join(d.page_content for d, _ in hits) or "(no documents)"
                    ans = llm.invoke([{"role": "user", "content": EXTRACT_PROMPT.format(context=ctx, q=q)}])
                else:
                    expr = llm.invoke([{"role": "user", "content": MATH_PROMPT.format(q=q, ledger=led)}])
                    try:
                        ans = str(safe_math(expr.splitlines()[0] if expr.strip() else "0"))
                    except Exception as e:
                        ans = f"could not compute ({e})"
                ledger.append({"question": q, "answer": ans.strip()})
        return ledger

    def rag_chain(self, query: str, chat_history: List[Dict[str, str]], **kwargs) -> Generator[str, None, None]:
        ledger = self.run_agent(query)
        if not ledger:  # nothing decomposed: plain RAG answer
            return super().rag_chain(query, chat_history, **kwargs)
        led = "\n".join(f"{e['question']}: {e['answer']}" for e in ledger)
        return get_llm(**kwargs).stream([{"role": "user", "content": FINAL_PROMPT.format(ledger=led, question=query)}])
