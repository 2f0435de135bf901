"""Data-analysis agent over a pandas DataFrame (reference: /root/reference/community/data-analysis-agent/
data_analysis_agent.py:131-431 - query understanding (is a plot wanted?), code writing for the answer or the plot,
execution, a reasoning pass that explains the result (with the model's thinking shown separately) and a dataset
insight summary).

The reference executes the model's Python with ``exec``. Here nothing the model writes is executed as code:
computations go through the framework's AST allow-listed pandas evaluator (``examples/structured_data.py``
``safe_pandas_eval``), and a plot is a declarative spec (kind, x, y, aggregation) that this module validates against
the frame's columns and turns into plot data plus a Vega-Lite spec for the UI to render.
"""
from __future__ import annotations

import json
import re
from typing import Any, Dict, Tuple

PLOT_WORDS = ("plot", "chart", "graph", "visuali", "histogram", "scatter", "bar chart", "line chart", "trend")
UNDERSTAND = ("Does the user's request ask for a plot, chart or other visualisation? Reply with one word: yes or no.")
CODE = ("You are given a pandas DataFrame `df` with columns {columns} and dtypes:\n{dtypes}\nFirst rows:\n{head}\n\n"
        "Write ONE Python expression using `df` (and `pd`) that computes the answer to: {question}\n"
        "Reply with the expression only.")
PLOT = ("You are given a pandas DataFrame `df` with columns {columns} and dtypes:\n{dtypes}\n"
        "Describe the plot that answers the request as JSON only: {{\"kind\": \"bar|line|scatter|hist\", \"x\": "
        "<column>, \"y\": <column or null>, \"agg\": \"sum|mean|count|max|min|none\", \"title\": <string>}}.\n"
        "Request: {question}")
REASON = ("Explain to the user, in a few sentences, what the result means for their question. Think first inside "
          "<think>...</think>, then give the explanation.")
INSIGHT = ("Summarise what this dataset is about in a short paragraph and suggest four analysis questions a user could "
           "ask about it.")
_AGGS = ("sum", "mean", "count", "max", "min", "none")
_KINDS = ("bar", "line", "scatter", "hist")


def _ask(llm, system: str, user: str, max_tokens: int = 512) -> str:
    r = llm.invoke([{"role": "system", "content": system}, {"role": "user", "content": user}], temperature=0.0,
                   max_tokens=max_tokens)
    return getattr(r, "content", r) or ""


def split_thinking(text: str) -> Tuple[str, str]:
    """(thinking, answer) from a reply with an optional <think> block."""
    m = re.search(r"<think>(.*?)</think>", text or "", re.S)
    if not m:
        return "", (text or "").strip()
    return m.group(1).strip(), (text[: m.start()] + text[m.end():]).strip()


def _first_code(text: str) -> str:
    m = re.search(r"```(?:python)?\s*(.*?)```", text or "", re.S)
    lines = [ln.strip() for ln in (m.group(1) if m else text or "").splitlines() if ln.strip()]
    return lines[0] if lines else ""


def wants_plot(llm, question: str) -> bool:
    low = question.lower()
    if any(w in low for w in PLOT_WORDS):
        return True
    m = re.search(r"\b(yes|no)\b", _ask(llm, UNDERSTAND, question, 4).lower())
    return bool(m and m.group(1) == "yes")


def plot_data(df, spec: Dict[str, Any]) -> Dict[str, Any]:
    """Validate a plot spec against ``df`` and compute its data (no model code runs)."""
    kind, x, y = spec.get("kind"), spec.get("x"), spec.get("y")
    agg = spec.get("agg") or "none"
    if kind not in _KINDS:
        raise ValueError(f"unsupported plot kind {kind!r}")
    if x not in df.columns or (y is not None and y not in df.columns):
        raise ValueError(f"unknown column in plot spec: {x!r} / {y!r}")
    if agg not in _AGGS:
        raise ValueError(f"unsupported aggregation {agg!r}")
    if kind == "hist":
        counts = df[x].value_counts(bins=min(20, max(1, df[x].nunique()))).sort_index() \
            if df[x].dtype.kind in "fiu" else df[x].value_counts()
        rows = [{"x": str(k), "y": int(v)} for k, v in counts.items()]
    elif agg == "none" or y is None:
        if y is None and agg == "count":
            s = df.groupby(x).size()
            rows = [{"x": k, "y": int(v)} for k, v in s.items()]
        else:
            rows = [{"x": a, "y": b} for a, b in zip(df[x].tolist(), df[y].tolist())] if y else \
                [{"x": a} for a in df[x].tolist()]
    else:
        s = getattr(df.groupby(x)[y], agg)()
        rows = [{"x": k, "y": float(v)} for k, v in s.items()]
    mark = {"bar": "bar", "line": "line", "scatter": "point", "hist": "bar"}[kind]
    vega = {"$schema": "https://vega.github.io/schema/vega-lite/v5.json", "title": spec.get("title", ""),
            "data": {"values": rows}, "mark": mark,
            "encoding": {"x": {"field": "x", "type": "nominal" if kind in ("bar", "hist") else "quantitative",
                               "title": x},
                         "y": {"field": "y", "type": "quantitative", "title": y or "count"}}}
    return {"rows": rows, "vega_lite": vega}


class DataAnalysisAgent:
    def __init__(self, llm, df):
        self.llm, self.df = llm, df

    def _frame_info(self) -> Dict[str, str]:
        return {"columns": list(self.df.columns), "dtypes": self.df.dtypes.to_string(),
                "head": self.df.head(5).to_string()}

    def answer(self, question: str, reason: bool = True) -> Dict[str, Any]:
        from ...examples.structured_data import safe_pandas_eval

        info = self._frame_info()
        out: Dict[str, Any] = {"question": question, "plot": None, "result": None, "error": None}
        if wants_plot(self.llm, question):
            raw = _ask(self.llm, PLOT.format(question=question, **info), "Plot spec:", 200)
            from ..fm_asr.chains import first_json_object

            spec = first_json_object(raw)
            try:
                if spec is None:
                    raise ValueError("the model returned no plot spec")
                out["plot"] = dict(plot_data(self.df, spec), spec=spec)
                out["result"] = out["plot"]["rows"][:50]
            except ValueError as e:
                out["error"] = str(e)
        else:
            expr = _first_code(_ask(self.llm, CODE.format(question=question, **info), "Expression:", 200))
            out["code"] = expr
            try:
                res = safe_pandas_eval(expr, self.df)
                out["result"] = res.to_dict() if hasattr(res, "to_dict") else res
            except Exception as e:  # noqa: BLE001 - rejected or failing expression: reported, not raised
                out["error"] = f"{type(e).__name__}: {e}"
        if reason and out["error"] is None:
            thinking, text = split_thinking(_ask(self.llm, REASON, f"Question: {question}\nResult: "
                                                 f"{json.dumps(out['result'], default=str)[:4000]}", 600))
            out["thinking"], out["explanation"] = thinking, text
        return out

    def insights(self) -> str:
        desc = self.df.describe(include="all").transpose().head(40).to_string()
        return _ask(self.llm, INSIGHT, f"Columns and statistics:\n{desc}", 400).strip()
