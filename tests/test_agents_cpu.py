"""Bash tool-calling agent loop (W11/W12), PandasAI adapter (C8), API client script (C9)."""
import json
import os
import subprocess
import sys

from generativeaiexamples_amd.examples.agents.bash_agent import BashTool, run_agent, system_prompt

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bash_tool_allowlist_and_jail(tmp_path):
    (tmp_path / "a.txt").write_text("x")
    (tmp_path / "b.txt").write_text("y")
    t = BashTool(str(tmp_path))
    assert "a.txt" in t("ls")
    assert t("rm a.txt").startswith("error") and (tmp_path / "a.txt").exists()
    assert t("ls | wc -l").startswith("error")
    assert t("cat a.txt; rm b.txt").startswith("error") and (tmp_path / "b.txt").exists()
    assert BashTool(str(tmp_path), confirm=lambda c: False)("ls").startswith("error: the user declined")


def test_agent_loop_executes_tool_calls(tmp_path):
    for i in range(3):
        (tmp_path / f"f{i}.txt").write_text("z")
    script = [{"content": None, "tool_calls": [{"id": "c1", "type": "function",
                                                "function": {"name": "exec_bash_command", "arguments": json.dumps({"cmd": "ls"})}}]},
              {"content": "There are 3 text files."}]
    seen = []

    def chat(messages, tools):
        seen.append([dict(m) for m in messages])
        return script[len(seen) - 1]
    ans = run_agent("how many txt files?", chat, BashTool(str(tmp_path)), thinking="off")
    assert ans == "There are 3 text files."
    tool_msg = seen[1][-1]
    assert tool_msg["role"] == "tool" and "f2.txt" in tool_msg["content"]
    assert seen[0][0]["content"].startswith("detailed thinking off")
    assert system_prompt("/x", None).startswith("You are")


def test_pandasai_adapter_routes_to_llm():
    from generativeaiexamples_amd.integrations.pandasai_llm import MI355XPandasLLM

    class FakeLLM:
        def invoke(self, msgs):
            return "df.shape[0]"

    class Prompt:
        def to_string(self):
            return "Write pandas code counting rows"

    llm = MI355XPandasLLM(model="m", llm=FakeLLM())
    assert llm.call(Prompt()) == "df.shape[0]" and llm.last_prompt == "Write pandas code counting rows"
    assert llm.type == "mi355x-llm" and llm._default_params["model"] == "m"


def test_api_client_script_help():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "RAG/src/chain_server/api_client.py"), "--help"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "--docs" in r.stdout


def test_faiss_compat_roundtrip(tmp_path):
    """Notebook-style FAISS usage with a LangChain-style embeddings object (embed_documents/embed_query)."""
    import hashlib

    from generativeaiexamples_amd.integrations.faiss_compat import FAISS

    class LCEmb:
        def _v(self, t):
            h = hashlib.sha256(t.encode()).digest()
            return [b / 255.0 for b in h[:16]]

        def embed_documents(self, texts):
            return [self._v(t) for t in texts]

        def embed_query(self, text):
            return self._v(text)

    texts = [f"fact number {i}" for i in range(20)]
    db = FAISS.from_texts(texts, LCEmb(), metadatas=[{"i": i} for i in range(20)], device="cpu")
    top = db.similarity_search("fact number 7", k=1)[0]
    assert top.page_content == "fact number 7" and top.metadata["i"] == 7  # exact match has distance 0
    db.save_local(str(tmp_path / "faiss"))
    db2 = FAISS.load_local(str(tmp_path / "faiss"), LCEmb(), allow_dangerous_deserialization=True, device="cpu")
    assert db2.similarity_search("fact number 13", k=1)[0].page_content == "fact number 13"
    assert len(db2.as_retriever(search_kwargs={"k": 3}).invoke("fact number 2")) == 3


def test_bash_tool_rejects_escapes(tmp_path):
    (tmp_path / "a.txt").write_text("x")
    t = BashTool(str(tmp_path))
    assert t("find . -name '*.txt' -exec rm {} +").startswith("error: find predicate '-exec'")
    assert t("find . -delete").startswith("error: find predicate '-delete'")
    assert t("find / -execdir sh -c id +").startswith("error")
    assert "outside the working directory" in t("cat /etc/shadow")
    assert "outside the working directory" in t("ls ../")
    assert "outside the working directory" in t("head ~/.bashrc")
    assert (tmp_path / "a.txt").exists()
    assert t("cat a.txt") == "x"
    assert "a.txt" in t("find . -name *.txt")
    # attached short-option values and GNU abbreviated long options (advisor round 2)
    assert t("sort -o/home/u/.bashrc a.txt").startswith("error: option -o")
    assert t("grep -f/etc/shadow x .").startswith("error: option -f")
    assert t("sort --compress-prog=sh -S 1K a.txt").startswith("error: option --compress-prog")
    assert t("sort --output=/tmp/x a.txt").startswith("error")
    assert t("uniq a.txt b.txt").startswith("error: too many operands")  # 2nd operand = output file
    assert t("du -L .").startswith("error: option -L")
    assert t("find . -newer /etc/passwd").startswith("error") and "outside" in t("find . -newer /etc/passwd")
    assert t("head -n1 a.txt") == "x" and t("head -n 1 a.txt") == "x"
    assert t("grep -c x a.txt") == "1" and t("sort -r -k 1 a.txt") == "x"


def test_pandas_sandbox_allowlist():
    import pandas as pd
    import pytest

    from generativeaiexamples_amd.examples.structured_data import safe_pandas_eval

    df = pd.DataFrame({"a": [1, 2, 3], "b": ["x", "y", "x"]})
    assert safe_pandas_eval("df.groupby('b')['a'].sum().to_dict()", df) == {"x": 4, "y": 2}
    assert safe_pandas_eval("df[df['a'] > 1].shape[0]", df) == 2
    assert safe_pandas_eval("df['a'].mean()", df) == 2.0
    for bad in ("pd.read_pickle('x.pkl')", "pd.read_csv('data.csv')", "df.to_json('/tmp/x')",
                "df.to_markdown(buf='out.md')", "df.to_hdf('x.h5', key='k')", "df.apply(print)",
                "df.eval('a+1')", "df.query('a>1')", "df.pipe(len)", "df.__class__",
                "df.to_string(buf='f')", "pd.io", "df['a'].map(print)"):
        with pytest.raises(ValueError):
            safe_pandas_eval(bad, df)
