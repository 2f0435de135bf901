"""advanced_rag/structured_data_rag (E5; reference chains.py:60-229 with PandasAI).

CSV files are ingested into one pandas DataFrame (column compatibility enforced, like the
reference's csv_utils). A question is answered by asking the LLM for a single pandas expression
over ``df`` and evaluating it in a sandbox (AST allow-list: no imports, no dunder attributes, no
builtins beyond a small set, bounded output) - the PandasAI agent of the reference executes
generated code unrestricted. The result is then phrased by the LLM (``csv_response_template``).
"""
from __future__ import annotations

import ast
import logging
import os
import threading
from typing import Any, Dict, Generator, List

import pandas as pd

from ..chain_server.base import BaseExample
from ..chain_server.utils import get_config, get_llm, get_prompts

log = logging.getLogger(__name__)

CODE_PROMPT = ("You are given a pandas DataFrame `df` with columns {columns}. First rows:\n{head}\n\n"
               "Write ONE Python expression using `df` (and `pd`) that computes the answer to: {question}\n"
               "Reply with the expression only.")
RESPONSE_PROMPT = ("Question: {question}\nComputed result:\n{result}\n\nAnswer the question in plain language "
                   "using the computed result.")

_ALLOWED_NODES = (ast.Expression, ast.Call, ast.Attribute, ast.Name, ast.Load, ast.Constant, ast.Subscript,
                  ast.Slice, ast.Tuple, ast.List, ast.Dict, ast.Compare, ast.BinOp, ast.UnaryOp, ast.BoolOp,
                  ast.keyword, ast.Eq, ast.NotEq, ast.Lt, ast.LtE, ast.Gt, ast.GtE, ast.And, ast.Or, ast.Not,
                  ast.BitAnd, ast.BitOr, ast.Invert, ast.Add, ast.Sub, ast.Mult, ast.Div, ast.Mod, ast.USub,
                  ast.In, ast.NotIn, ast.IfExp, ast.FloorDiv, ast.Pow)
_SAFE_BUILTINS = {"len": len, "round": round, "min": min, "max": max, "sum": sum, "abs": abs, "sorted": sorted,
                  "list": list, "str": str, "int": int, "float": float}
# Allow-list of attributes an expression may touch (DataFrame / Series / GroupBy / .str / .dt accessors).
# Everything else - readers (read_pickle / read_csv: arbitrary files or URLs), writers (to_json, to_hdf,
# to_markdown(buf=...)), eval/query/apply/pipe (code execution) - is rejected at parse time.
_ALLOWED_ATTRS = frozenset("""
    loc iloc at iat shape columns index dtypes size ndim empty T values
    head tail nlargest nsmallest sort_values sort_index sort groupby agg aggregate
    mean median sum count min max std var mode nunique unique value_counts describe quantile prod cumsum
    cummax cummin idxmax idxmin abs round clip corr cov rank pct_change diff
    isna isnull notna notnull fillna dropna drop_duplicates duplicated isin between where mask
    reset_index set_index rename astype copy get first last nth size filter
    str dt contains startswith endswith lower upper strip len split replace year month day
    to_list tolist to_dict item any all eq ne lt le gt ge add sub mul div truediv floordiv mod pow
    merge join concat DataFrame Series to_datetime to_numeric cut
""".split())
# a subset of ``pd`` functions, reachable only as pd.<name>
_PD_FUNCS = frozenset({"concat", "to_datetime", "to_numeric", "cut", "DataFrame", "Series", "isna", "notna"})
# keyword arguments that name a file, buffer, URL or callable
_BANNED_KWARGS = frozenset({"path", "path_or_buf", "buf", "filepath_or_buffer", "func", "engine", "storage_options",
                            "io", "con", "excel_writer"})


class _SafePd:
    """The only view of pandas an expression gets: the allow-listed functions, nothing else."""

    def __init__(self):
        for n in _PD_FUNCS:
            setattr(self, n, getattr(pd, n))


def safe_pandas_eval(expr: str, df: pd.DataFrame) -> Any:
    """Evaluate one LLM-written pandas expression over ``df`` under an AST allow-list: allowed node types,
    allow-listed attribute names only (no readers / writers / eval / apply), no keyword argument that can
    name a path, buffer, URL or callable, and no string argument that looks like a path or URL."""
    expr = expr.strip().strip("`")
    if expr.startswith("python"):
        expr = expr[6:].strip()
    tree = ast.parse(expr, mode="eval")
    for node in ast.walk(tree):
        if not isinstance(node, _ALLOWED_NODES):
            raise ValueError(f"disallowed syntax: {type(node).__name__}")
        if isinstance(node, ast.Attribute):
            if node.attr.startswith("_") or node.attr not in _ALLOWED_ATTRS:
                raise ValueError(f"attribute {node.attr!r} is not allowed")
            if isinstance(node.value, ast.Name) and node.value.id == "pd" and node.attr not in _PD_FUNCS:
                raise ValueError(f"pd.{node.attr} is not allowed")
        if isinstance(node, ast.Name) and node.id not in ("df", "pd", *_SAFE_BUILTINS):
            raise ValueError(f"unknown name {node.id}")
        if isinstance(node, ast.keyword) and (node.arg is None or node.arg in _BANNED_KWARGS):
            raise ValueError(f"keyword argument {node.arg!r} is not allowed")
        if isinstance(node, ast.Constant) and isinstance(node.value, str) and (
                node.value.startswith(("/", "~")) or ".." in node.value or "\\" in node.value
                or "://" in node.value):
            raise ValueError("path-like string arguments are not allowed")
    return eval(compile(tree, "<pandas-expr>", "eval"), {"__builtins__": _SAFE_BUILTINS}, {"df": df, "pd": _SafePd()})


class StructuredDataRAG(BaseExample):
    def __init__(self):
        self.cfg = get_config()
        self.prompts = get_prompts()
        self.df: pd.DataFrame | None = None
        self.files: List[str] = []
        self.lock = threading.Lock()

    def ingest_docs(self, filepath: str, filename: str) -> None:
        if not filename.lower().endswith(".csv"):
            raise ValueError(f"{filename} is not a CSV file")
        new = pd.read_csv(filepath)
        with self.lock:
            if self.df is not None and list(new.columns) != list(self.df.columns):
                raise ValueError("CSV columns do not match the already ingested CSV files")
            self.df = new if self.df is None else pd.concat([self.df, new], ignore_index=True)
            self.files.append(filename)

    def llm_chain(self, query: str, chat_history: List[Dict[str, str]], **kwargs) -> Generator[str, None, None]:
        return get_llm(**kwargs).stream([{"role": "system", "content": self.prompts["chat_template"]},
                                         {"role": "user", "content": query}])

    def rag_chain(self, query: str, chat_history: List[Dict[str, str]], **kwargs) -> Generator[str, None, None]:
        if self.df is None:
            return iter(["No CSV file has been ingested yet."])
        llm = get_llm(temperature=0.1, max_tokens=200)
        expr = llm.invoke([{"role": "user", "content": CODE_PROMPT.format(
            columns=list(self.df.columns), head=self.df.head(5).to_string(), question=query)}])
        result = None
        for attempt in range(2):
            try:
                result = safe_pandas_eval(expr.strip().splitlines()[0] if expr.strip() else "df.shape", self.df)
                break
            except Exception as e:
                expr = llm.invoke([{"role": "user", "content": f"The expression failed with: {e}. "
                                    + CODE_PROMPT.format(columns=list(self.df.columns),
                                                         head=self.df.head(3).to_string(), question=query)}])
        if result is None:
            return iter(["Could not compute an answer from the CSV data."])
        text = result.to_string()[:4000] if hasattr(result, "to_string") else str(result)[:4000]
        tmpl = self.prompts.get("csv_response_template", RESPONSE_PROMPT)
        try:
            content = tmpl.format(question=query, result=text, query=query, data=text)
        except (KeyError, IndexError):
            content = RESPONSE_PROMPT.format(question=query, result=text)
        return get_llm(**kwargs).stream([{"role": "user", "content": content}])

    def document_search(self, content: str, num_docs: int):
        if self.df is None:
            return []
        mask = self.df.astype(str).apply(lambda c: c.str.contains(content, case=False, regex=False)).any(axis=1)
        return [{"content": r.to_json(), "filename": self.files[0] if self.files else "", "score": 1.0}
                for _, r in self.df[mask].head(num_docs).iterrows()]

    def get_documents(self) -> List[str]:
        return list(self.files)

    def delete_documents(self, filenames: List[str]) -> bool:
        with self.lock:
            self.files = [f for f in self.files if f not in filenames]
            if not self.files:
                self.df = None
        return True
