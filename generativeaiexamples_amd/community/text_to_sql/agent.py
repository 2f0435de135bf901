"""Retrieval-augmented text-to-SQL (reference: /root/reference/community/Vanna_with_NVIDIA_AI_Endpoints/
vanna_with_NVIDIA.ipynb - Vanna with a Milvus store and an OpenAI-compatible NIM: ``connect_to_sqlite``, ``train`` on
DDL / documentation / question-SQL pairs, ``generate_sql`` from the retrieved training data, ``run_sql``; and
SQLServer_AI_with_NVIDIA_NIM, which embeds table rows for similarity search from SQL).

Training data lives in ONE HBM collection partitioned by ``kind`` (ddl / documentation / sql); a question retrieves
each kind with a filtered (partition) scan. Generated SQL runs on a read-only connection: an sqlite authorizer allows
only SELECT / READ / FUNCTION / recursive-CTE actions, so a generated ``DROP`` / ``UPDATE`` / ``ATTACH`` is refused by
the database rather than by string matching. A query that fails is sent back to the model once with the error
(self-correction); ``ask`` can also phrase the result.
"""
from __future__ import annotations

import re
import sqlite3
import threading
import time
import uuid
from typing import Dict, List, Optional, Tuple

from ...index.hbm_index import Document

SQL_SYSTEM = ("You are a {dialect} expert. Write ONE {dialect} query that answers the question, using only the tables "
              "and columns in the schema below. Reply with the SQL in a ```sql block and nothing else.\n\n"
              "Schema:\n{ddl}\n\nDocumentation:\n{docs}\n\nExamples of questions and their SQL:\n{examples}")
FIX_PROMPT = "The query failed with: {error}\nReturn a corrected query in a ```sql block."
SUMMARY_SYSTEM = "Answer the user's question in one or two sentences from the query result."

_READ_ACTIONS = {sqlite3.SQLITE_SELECT, sqlite3.SQLITE_READ, sqlite3.SQLITE_FUNCTION,
                 getattr(sqlite3, "SQLITE_RECURSIVE", 33)}


def _authorizer(action, *_):
    return sqlite3.SQLITE_OK if action in _READ_ACTIONS else sqlite3.SQLITE_DENY


def extract_sql(text: str) -> Optional[str]:
    text = getattr(text, "content", text) or ""
    m = re.search(r"```(?:sql|sqlite)?\s*(.*?)```", text, re.S | re.I)
    body = m.group(1) if m else text
    m = re.search(r"\b(WITH|SELECT)\b.*", body, re.S | re.I)
    if not m:
        return None
    sql = _first_statement(m.group(0)).strip()
    return sql or None


def _first_statement(sql: str) -> str:
    """Text up to the first ``;`` outside quoted literals / identifiers (one statement; trailing prose dropped)."""
    quote = None
    for i, ch in enumerate(sql):
        if quote:
            if ch == quote:
                quote = None
        elif ch in "'\"`[":
            quote = "]" if ch == "[" else ch
        elif ch == ";":
            return sql[:i]
    return sql


class SqlAgent:
    def __init__(self, llm, store, dialect: str = "SQLite", n_examples: int = 5, n_ddl: int = 6, n_docs: int = 4,
                 query_timeout_s: float = 30.0):
        self.llm, self.store, self.dialect = llm, store, dialect
        self.query_timeout_s = query_timeout_s
        self._deadline = float("inf")
        self.n_examples, self.n_ddl, self.n_docs = n_examples, n_ddl, n_docs
        self.conn: Optional[sqlite3.Connection] = None
        self.db_lock = threading.Lock()  # one connection shared by request threads: one statement at a time
        self.training: Dict[str, Tuple[str, Document]] = {}

    # ---- database
    def connect_to_sqlite(self, path: str, read_only: bool = True) -> None:
        self.conn = sqlite3.connect(path, check_same_thread=False)
        if read_only:
            self.conn.set_authorizer(_authorizer)
        # a runaway statement (an unbounded recursive CTE, a huge cross join) is interrupted at the deadline
        self.conn.set_progress_handler(lambda: int(time.monotonic() > self._deadline), 10_000)

    def run_sql(self, sql: str):
        import pandas as pd

        if self.conn is None:
            raise RuntimeError("connect_to_sqlite first")
        with self.db_lock:
            self._deadline = time.monotonic() + self.query_timeout_s
            try:
                cur = self.conn.execute(sql)
                cols = [c[0] for c in cur.description or []]
                rows = cur.fetchall()
            finally:
                self._deadline = float("inf")
        return pd.DataFrame(rows, columns=cols)

    def schema_ddl(self) -> List[str]:
        with self.db_lock:
            rows = self.conn.execute("SELECT sql FROM sqlite_master WHERE sql IS NOT NULL AND type IN ('table', 'view')"
                                     ).fetchall()
        return [r[0] for r in rows]

    # ---- training data
    def train(self, ddl: Optional[str] = None, documentation: Optional[str] = None, question: Optional[str] = None,
              sql: Optional[str] = None) -> str:
        if question is not None and sql is None:
            raise ValueError("a training question needs its sql")
        if ddl:
            kind, text = "ddl", ddl
        elif documentation:
            kind, text = "documentation", documentation
        elif sql:
            kind, text = "sql", f"Question: {question or ''}\nSQL: {sql}"
        else:
            raise ValueError("nothing to train on")
        tid = f"{uuid.uuid4()}-{kind}"
        doc = Document(text, {"kind": kind, "id": tid, "filename": tid})
        self.store.add_documents([doc])
        self.training[tid] = (kind, doc)
        return tid

    def train_schema(self) -> int:
        return sum(1 for d in self.schema_ddl() if self.train(ddl=d))

    def get_training_data(self) -> List[dict]:
        return [{"id": tid, "kind": k, "content": d.page_content} for tid, (k, d) in self.training.items()]

    def remove_training_data(self, tid: str) -> bool:
        if tid not in self.training:
            return False
        self.store.delete_filename(tid)
        del self.training[tid]
        return True

    def _related(self, question: str, kind: str, k: int) -> List[str]:
        if k <= 0 or not any(kd == kind for kd, _ in self.training.values()):
            return []
        hits = self.store.similarity_search_with_relevance_scores(question, k, filter={"kind": kind})
        return [d.page_content for d, _ in hits]

    # ---- generation
    def prompt(self, question: str) -> List[dict]:
        sys_ = SQL_SYSTEM.format(dialect=self.dialect,
                                 ddl="\n\n".join(self._related(question, "ddl", self.n_ddl)) or "(none)",
                                 docs="\n".join(self._related(question, "documentation", self.n_docs)) or "(none)",
                                 examples="\n\n".join(self._related(question, "sql", self.n_examples)) or "(none)")
        return [{"role": "system", "content": sys_}, {"role": "user", "content": question}]

    def generate_sql(self, question: str) -> Optional[str]:
        r = self.llm.invoke(self.prompt(question), temperature=0.0, max_tokens=512)
        return extract_sql(r)

    def ask(self, question: str, summarize: bool = False, retries: int = 1) -> dict:
        msgs = self.prompt(question)
        reply = self.llm.invoke(msgs, temperature=0.0, max_tokens=512)
        sql, err, df = extract_sql(reply), None, None
        for attempt in range(retries + 1):
            if sql is None:
                err = "the model returned no SQL query"
            else:
                try:
                    df = self.run_sql(sql)
                    err = None
                    break
                except sqlite3.Error as e:
                    err = str(e)
            if attempt == retries:
                break
            msgs = msgs + [{"role": "assistant", "content": getattr(reply, "content", reply) or ""},
                           {"role": "user", "content": FIX_PROMPT.format(error=err)}]
            reply = self.llm.invoke(msgs, temperature=0.0, max_tokens=512)
            sql = extract_sql(reply)
        out = {"question": question, "sql": sql, "error": err, "df": df}
        if summarize and df is not None:
            r = self.llm.invoke([{"role": "system", "content": SUMMARY_SYSTEM},
                                 {"role": "user", "content": f"Question: {question}\nResult:\n{df.head(20).to_string()}"}],
                                temperature=0.0, max_tokens=200)
            out["summary"] = getattr(r, "content", r)
        return out
