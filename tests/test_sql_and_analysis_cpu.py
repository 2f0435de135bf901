"""Text-to-SQL (Vanna / SQL Server AI community projects) and the data-analysis agent: retrieval of
training data by kind, read-only execution enforced by the database, one self-correction round, sandboxed pandas
answers, validated declarative plots - scripted LLMs, crc32 hashing embedder, CPU."""
import sqlite3
import zlib

import pandas as pd
import pytest
import torch

from generativeaiexamples_amd.chain_server.connectors import Embeddings
from generativeaiexamples_amd.chain_server.vectorstore import VectorStore
from generativeaiexamples_amd.community.data_analysis import DataAnalysisAgent, plot_data, split_thinking
from generativeaiexamples_amd.community.data_analysis import agent as da
from generativeaiexamples_amd.community.text_to_sql import SqlAgent, extract_sql


class _Emb(Embeddings):
    dim = 64

    def embed_tensor(self, texts, input_type):
        out = torch.zeros(len(texts), self.dim)
        for i, t in enumerate(texts):
            for w in t.lower().replace("(", " ").replace(",", " ").split():
                out[i, zlib.crc32(w.strip(".,?:;").encode()) % self.dim] += 1.0
        return torch.nn.functional.normalize(out + 1e-3, dim=-1)


@pytest.fixture()
def db(tmp_path):
    p = str(tmp_path / "steam.db")
    c = sqlite3.connect(p)
    c.execute("CREATE TABLE games (id INTEGER PRIMARY KEY, name TEXT, positive INTEGER, players INTEGER, indie INTEGER)")
    c.executemany("INSERT INTO games VALUES (?, ?, ?, ?, ?)",
                  [(1, "Alpha", 900, 50000, 1), (2, "Beta", 1500, 20000, 0), (3, "Gamma", 300, 90000, 1),
                   (4, "Delta", 1200, 10000, 0)])
    c.commit()
    c.close()
    return p


def test_extract_sql():
    assert extract_sql("Here:\n```sql\nSELECT name FROM games;\nDROP TABLE games;\n```") == "SELECT name FROM games"
    assert extract_sql("WITH t AS (SELECT 1) SELECT * FROM t") == "WITH t AS (SELECT 1) SELECT * FROM t"
    assert extract_sql("I can't help") is None
    # a ';' inside a literal or quoted identifier does not end the statement
    assert extract_sql("SELECT * FROM t WHERE a = 'x;y'; DROP TABLE t") == "SELECT * FROM t WHERE a = 'x;y'"
    assert extract_sql("SELECT 'it''s;' AS \"c;d\" FROM t; trailing prose") == "SELECT 'it''s;' AS \"c;d\" FROM t"


def test_sql_agent_train_generate_run(db):
    class LLM:
        def __init__(self):
            self.prompts = []

        def invoke(self, messages, **kw):
            self.prompts.append(messages[0]["content"])
            if len(messages) > 2:  # the correction round
                return "```sql\nSELECT name, players FROM games WHERE indie = 1 ORDER BY players DESC LIMIT 1\n```"
            if "indie" in messages[-1]["content"]:
                return "```sql\nSELECT name, player_count FROM games\n```"  # wrong column -> sqlite error
            if "Answer the user's question" in messages[0]["content"]:
                return "Beta has the most positive reviews."
            return "```sql\nSELECT name, positive FROM games ORDER BY positive DESC LIMIT 2\n```"

    llm = LLM()
    ag = SqlAgent(llm, VectorStore("sql", _Emb(), device="cpu"))
    ag.connect_to_sqlite(db)
    assert ag.train_schema() == 1
    doc_id = ag.train(documentation="indie = 1 marks independent games; players is the player base")
    ag.train(question="How many games are there?", sql="SELECT COUNT(*) FROM games")
    with pytest.raises(ValueError):
        ag.train(question="orphan")
    kinds = sorted(t["kind"] for t in ag.get_training_data())
    assert kinds == ["ddl", "documentation", "sql"]
    out = ag.ask("Which 2 games have the most positive reviews?", summarize=True)
    assert out["error"] is None and out["df"]["name"].tolist() == ["Beta", "Delta"]
    assert out["summary"].startswith("Beta")
    sys_prompt = llm.prompts[0]
    assert "CREATE TABLE games" in sys_prompt and "independent games" in sys_prompt and "COUNT(*)" in sys_prompt
    out = ag.ask("Which indie game has the biggest player base?")
    assert out["error"] is None and out["df"].iloc[0].tolist() == ["Gamma", 90000]  # fixed in the correction round
    assert ag.remove_training_data(doc_id) and not ag.remove_training_data(doc_id)
    assert "independent games" not in ag.prompt("indie")[0]["content"]


def test_sql_agent_read_only(db):
    ag = SqlAgent(None, VectorStore("sql2", _Emb(), device="cpu"))
    ag.connect_to_sqlite(db)
    for stmt in ("DROP TABLE games", "UPDATE games SET positive = 0", "DELETE FROM games",
                 "INSERT INTO games (name) VALUES ('x')", "ATTACH DATABASE ':memory:' AS x",
                 "CREATE TABLE t (a)", "PRAGMA writable_schema = 1"):
        with pytest.raises(sqlite3.DatabaseError):
            ag.run_sql(stmt)
    assert len(ag.run_sql("SELECT * FROM games")) == 4
    ag.query_timeout_s = 0.2  # an unbounded recursive CTE is interrupted at the deadline
    with pytest.raises(sqlite3.OperationalError):
        ag.run_sql("WITH RECURSIVE n(i) AS (SELECT 1 UNION ALL SELECT i + 1 FROM n) SELECT max(i) FROM n")
    ag.query_timeout_s = 30.0

    class Bad:
        def invoke(self, messages, **kw):
            return "```sql\nWITH doomed AS (SELECT id FROM games) DELETE FROM games WHERE id IN doomed\n```"

    ag.llm = Bad()
    out = ag.ask("delete everything", retries=1)
    assert out["df"] is None and "not authorized" in out["error"]
    assert len(ag.run_sql("SELECT * FROM games")) == 4


DF = pd.DataFrame({"region": ["north", "south", "north", "east", "south"], "sales": [10.0, 20.0, 30.0, 5.0, 15.0],
                   "units": [1, 2, 3, 1, 2]})


def test_plot_spec_validation_and_data():
    out = plot_data(DF, {"kind": "bar", "x": "region", "y": "sales", "agg": "sum", "title": "Sales"})
    assert out["rows"] == [{"x": "east", "y": 5.0}, {"x": "north", "y": 40.0}, {"x": "south", "y": 35.0}]
    assert out["vega_lite"]["mark"] == "bar" and out["vega_lite"]["title"] == "Sales"
    assert len(plot_data(DF, {"kind": "scatter", "x": "units", "y": "sales"})["rows"]) == 5
    assert sum(r["y"] for r in plot_data(DF, {"kind": "hist", "x": "region"})["rows"]) == 5
    for bad in ({"kind": "pie", "x": "region"}, {"kind": "bar", "x": "nope"}, {"kind": "bar", "x": "region",
                                                                              "y": "sales", "agg": "exec"}):
        with pytest.raises(ValueError):
            plot_data(DF, bad)


def test_data_analysis_agent():
    class LLM:
        def invoke(self, messages, **kw):
            sys_ = messages[0]["content"]
            if sys_ == da.UNDERSTAND:
                return "no"
            if sys_.startswith("You are given") and "Describe the plot" in sys_:
                return '{"kind": "line", "x": "units", "y": "sales", "agg": "mean", "title": "t"}'
            if sys_.startswith("You are given"):
                q = sys_.split("answer to:")[1]
                if "import" in q:
                    return "__import__('os').system('echo hacked')"
                return "```python\ndf.groupby('region')['sales'].sum()\n```"
            if sys_ == da.REASON:
                return "<think>north is largest</think>North sells the most."
            return "A sales table by region."

    ag = DataAnalysisAgent(LLM(), DF)
    out = ag.answer("Total sales per region?")
    assert out["result"] == {"east": 5.0, "north": 40.0, "south": 35.0} and out["plot"] is None
    assert out["thinking"] == "north is largest" and out["explanation"] == "North sells the most."
    out = ag.answer("Plot mean sales by units")
    assert out["plot"]["spec"]["kind"] == "line" and out["plot"]["rows"][0] == {"x": 1, "y": 7.5}
    out = ag.answer("import something please")
    assert out["error"] is not None and out["result"] is None
    assert ag.insights() == "A sales table by region."
    assert split_thinking("plain") == ("", "plain")
