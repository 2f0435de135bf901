"""Event-driven CVE triage community app (reference community/event-driven-rag-cve-analysis): checklist
parsing, version ordering (PEP 440 / Debian), SBOM and code-search tools, the ReAct loop and the concurrent scan
engine + /scan service, driven by a scripted LLM on the CPU."""
import json
import threading
import time
import zlib

import pytest
import torch

from generativeaiexamples_amd.chain_server.connectors import Embeddings
from generativeaiexamples_amd.chain_server.vectorstore import VectorStore
from generativeaiexamples_amd.community.cve_agent import (CodeSearch, CVEEngine, ReActAgent, SBOMChecker, create_app,
                                                          debian_compare, parse_checklist, parse_step,
                                                          version_comparison)
from generativeaiexamples_amd.community.cve_agent.checklist import CHECKLIST_PROMPT
from generativeaiexamples_amd.community.cve_agent.pipeline import SUMMARY_PROMPT, timing_table
from generativeaiexamples_amd.community.cve_agent.tools import default_tools
from generativeaiexamples_amd.index.hbm_index import Document

CHECKLIST_REPLY = ('Here is the checklist:\n["Check for lxml: verify the image\'s "lxml" dependency.", '
                   '"Check the lxml version: versions up to 4.9.1 are vulnerable."]')


def test_parse_checklist_variants():
    assert parse_checklist(CHECKLIST_REPLY) == ['Check for lxml: verify the image\'s "lxml" dependency.',
                                                "Check the lxml version: versions up to 4.9.1 are vulnerable."]
    assert parse_checklist('```json\n["a b", ["c d"]]\n```') == ["a b", "c d"]
    assert parse_checklist("1. Check the version\n2) Check usage of iterwalk\n- Review mitigations") == [
        "Check the version", "Check usage of iterwalk", "Review mitigations"]
    assert parse_checklist("['only one item'") == ["only one item"]  # unterminated list is closed
    assert parse_checklist("") == []


@pytest.mark.parametrize("a,b,want", [
    ("1.0~rc1", "1.0", -1), ("1.0", "1.0-1", -1), ("1.2.3", "1.2.3-0", 0), ("1:0.9", "2.0", 1),
    ("2.9.10+dfsg-1", "2.9.14+dfsg-1", -1), ("1.0a", "1.0", 1), ("1.0+", "1.0a", 1), ("1.0.10", "1.0.9", 1),
    ("2.36-9+deb12u4", "2.36-9+deb12u10", -1), ("0.9~~", "0.9~", -1)])
def test_debian_ordering(a, b, want):
    assert debian_compare(a, b) == want and debian_compare(b, a) == -want


def test_version_comparison_contract():
    assert version_comparison("4.9.1,4.9.1") is True and version_comparison("4.9.2,4.9.1") is False
    assert version_comparison("2.9.12, 2.9.10, 2.9.14") is True
    assert version_comparison("1:2.9.10-1,2.9.10,2.9.14") is False  # Debian epoch outranks upstream
    assert version_comparison("2.9.10-1ubuntu0.2,2.9.10,2.9.14") is True
    assert version_comparison("1.2,1.0,1.1,1.2") is True and version_comparison("1.3,1.0,1.1,1.2") is False
    assert isinstance(version_comparison("1.0"), str)


def test_sbom_and_code_tools(tmp_path):
    p = tmp_path / "sbom.csv"
    p.write_text("package,version\nlxml,4.9.1\nLibXML2,2.9.12\n")
    sb = SBOMChecker.from_csv(str(p))
    assert sb("lxml") == "4.9.1" and sb(" libxml2 ") == "2.9.12" and sb("'lxml'") == "4.9.1"
    assert "not found" in sb("aiohttp") and "name only" in sb("lxml version please")

    class HashEmb(Embeddings):
        dim = 32

        def embed_tensor(self, texts, input_type):
            out = torch.zeros(len(texts), self.dim)
            for i, t in enumerate(texts):
                for w in t.lower().replace("(", " ").replace(".", " ").split():
                    out[i, zlib.crc32(w.encode()) % self.dim] += 1
            return torch.nn.functional.normalize(out + 1e-3, dim=-1)

    store = VectorStore("code", HashEmb(), device="cpu")
    assert "No source code" in CodeSearch(store)("iterwalk")
    store.add_documents([Document("from lxml import etree\nfor ev, el in etree.iterwalk(root): pass",
                                  {"source": "app/parse.py"}),
                         Document("def add(a, b):\n    return a + b", {"source": "app/math.py"})])
    assert CodeSearch(store, k=1)("etree iterwalk").startswith("[app/parse.py]")
    tools = default_tools(sb, CodeSearch(store))
    assert [t.name for t in tools] == ["Version Comparator", "SBOM Package Checker", "Container Code Search"]
    assert tools[0]("oops") .startswith("Could not compare")


class _LLM:
    """Checklist -> two items; agent: SBOM lookup then a final answer; summary -> fixed text."""

    def __init__(self, delay=0.0):
        self.delay, self.lock, self.inflight, self.peak = delay, threading.Lock(), 0, 0

    def invoke(self, messages, **kw):
        with self.lock:
            self.inflight += 1
            self.peak = max(self.peak, self.inflight)
        try:
            time.sleep(self.delay)
            sys_, user = messages[0]["content"], messages[-1]["content"]
            if sys_ == CHECKLIST_PROMPT:
                return "not a list at all" if "BROKEN" in user else CHECKLIST_REPLY
            if sys_ == SUMMARY_PROMPT:
                return "The container appears vulnerable."
            if "Observation:" not in user:
                assert kw.get("stop") == ["\nObservation:"]
                return "Thought: I should look in the SBOM.\nAction: SBOM Package Checker\nAction Input: lxml\n"
            return "Thought: the SBOM lists it.\nFinal Answer: lxml 4.9.1 is installed."
        finally:
            with self.lock:
                self.inflight -= 1


def test_parse_step():
    assert parse_step("Thought: x\nFinal Answer: yes") == ("yes", None, None)
    assert parse_step("Thought: x\nAction: [SBOM Package Checker]\nAction Input: \"lxml\"") == (
        None, "SBOM Package Checker", "lxml")
    assert parse_step("Action: A\nAction Input: b\nFinal Answer: c") == (None, "A", "b")  # the earlier one wins
    assert parse_step("just prose") == (None, None, None)


def test_react_agent_loop():
    sb = SBOMChecker({"lxml": "4.9.1"})
    r = ReActAgent(_LLM(), default_tools(sb)).run("Check for lxml")
    assert r.finished and r.answer == "lxml 4.9.1 is installed." and r.steps == [("SBOM Package Checker", "lxml",
                                                                                  "4.9.1")]

    class Chatty:
        def __init__(self):
            self.seen = []

        def invoke(self, messages, **kw):
            self.seen.append(messages[-1]["content"])
            if len(self.seen) == 1:
                return "I think it is fine."  # no protocol: reminded
            if len(self.seen) == 2:
                return "Thought: try\nAction: Nonexistent Tool\nAction Input: x"
            return "Thought: still looking\nAction: Version Comparator\nAction Input: 1.0,2.0"

    c = Chatty()
    r = ReActAgent(c, default_tools(sb), max_steps=4).run("Check the version")
    assert "did not follow the format" in c.seen[1] and "is not a tool" in c.seen[2]
    assert not r.finished and r.answer == "still looking" and r.steps[-1][2] == "True"


def test_engine_scan_concurrent_and_ordered():
    llm = _LLM(delay=0.05)
    eng = CVEEngine(llm, tools=default_tools(SBOMChecker({"lxml": "4.9.1"})), max_concurrency=16)
    cves = ["CVE-A lxml iterwalk crash", "BROKEN input", "CVE-A lxml iterwalk crash"]
    res = eng.scan(cves)
    assert [r.cve_info for r in res] == cves
    assert res[0].checklist[1].startswith("Check the lxml version") and res[0].response == [
        "lxml 4.9.1 is installed."] * 2
    assert res[0].summary == "The container appears vulnerable." and res[0].error is None
    assert res[1].checklist == ["not a list at all"] and len(res[1].response) == 1
    assert llm.peak >= 4  # CVEs and checklist items in flight together
    assert all(r.latency_ms > 0 for r in res)
    rows = timing_table(eng, cves[:1], counts=(1, 3))
    assert [r["cves"] for r in rows] == [1, 3] and rows[1]["avg_ms"] < rows[1]["total_ms"]


def test_engine_error_is_per_cve():
    class Bad(_LLM):
        def invoke(self, messages, **kw):
            if "explode" in messages[-1]["content"]:
                raise RuntimeError("model down")
            return super().invoke(messages, **kw)

    res = CVEEngine(Bad(), tools=default_tools(SBOMChecker({}))).scan(["explode", "CVE-B"])
    assert res[0].error == "RuntimeError: model down" and res[1].error is None and res[1].checklist


def test_scan_service():
    from fastapi.testclient import TestClient

    eng = CVEEngine(_LLM(), tools=default_tools(SBOMChecker({"lxml": "4.9.1"})), summarize=False)
    c = TestClient(create_app(lambda: eng))
    out = c.post("/scan", json=[{"cve_info": "CVE-1"}, {"cve_info": "CVE-2"}]).json()
    assert [o["cve_info"] for o in out] == ["CVE-1", "CVE-2"] and out[0]["summary"] == ""
    lines = [json.loads(x) for x in c.post("/scan/stream", json=[{"cve_info": "CVE-3"}]).text.splitlines() if x]
    assert len(lines) == 1 and lines[0]["response"] == ["lxml 4.9.1 is installed."] * 2
