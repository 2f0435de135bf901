"""Event-driven CVE triage (reference: /root/reference/community/event-driven-rag-cve-analysis/cyber_dev_day/
pipeline.py:44-137, pipeline_utils.py:115-132 and notebooks/cyber-dev-day.ipynb - a Morpheus LLM engine per CVE:
checklist node -> agent node over every checklist item, outputs ``checklist`` + ``response`` columns; an HTTP source
``POST /scan`` with ``[{"cve_info": ...}, ...]`` for the microservice form; latency measured for 1 / 5 / 10 CVEs).

``CVEEngine.scan`` runs CVEs concurrently and, inside each CVE, every checklist item's agent concurrently (one thread
per in-flight model call): the in-process LLM engine's continuous batcher turns those calls into one decode batch,
which is what makes 10 CVEs cost about as much wall time as 1 (the reference notebook's concurrency table). Each result
carries its own latency. ``create_app`` serves ``POST /scan`` (results as JSON) and ``POST /scan/stream`` (NDJSON, one
line per finished CVE).

  python -m generativeaiexamples_amd.community.cve_agent.pipeline --sbom sbom.csv --cve "An issue was ..."
"""
from __future__ import annotations

import argparse
import json
import time
from concurrent.futures import ThreadPoolExecutor, as_completed
from dataclasses import asdict, dataclass, field
from typing import Callable, Iterator, List, Optional, Sequence

from pydantic import BaseModel

from .agent import ReActAgent
from .checklist import generate_checklist
from .tools import CodeSearch, SBOMChecker, Tool, default_tools

SUMMARY_PROMPT = (
    "Summarise a container exploitability investigation in two or three sentences: state whether the container "
    "appears vulnerable to the CVE, not vulnerable, or undetermined, and cite the decisive checklist findings.")


class ScanItem(BaseModel):
    """One event of the reference's /scan payload ``[{"cve_info": ...}, ...]``."""
    cve_info: str


@dataclass
class CVEResult:
    cve_info: str
    checklist: List[str] = field(default_factory=list)
    response: List[str] = field(default_factory=list)
    summary: str = ""
    latency_ms: float = 0.0
    error: Optional[str] = None


class CVEEngine:
    def __init__(self, checklist_llm, agent_llm=None, tools: Optional[Sequence[Tool]] = None,
                 max_concurrency: int = 64, summarize: bool = True, max_steps: int = 8):
        self.checklist_llm, self.agent_llm = checklist_llm, agent_llm or checklist_llm
        self.tools = list(tools) if tools is not None else default_tools()
        self.max_concurrency, self.summarize, self.max_steps = max_concurrency, summarize, max_steps

    def _agent(self) -> ReActAgent:
        return ReActAgent(self.agent_llm, self.tools, max_steps=self.max_steps)

    def _one(self, cve_info: str, pool: ThreadPoolExecutor) -> CVEResult:
        t0 = time.perf_counter()
        res = CVEResult(cve_info)
        try:
            res.checklist = generate_checklist(cve_info, self.checklist_llm)
            futs = [pool.submit(self._agent().run, item) for item in res.checklist]
            res.response = [f.result().answer for f in futs]
            if self.summarize and res.checklist:
                findings = "\n".join(f"- {c}\n  Finding: {r}" for c, r in zip(res.checklist, res.response))
                r = self.agent_llm.invoke(
                    [{"role": "system", "content": SUMMARY_PROMPT},
                     {"role": "user", "content": f"CVE: {cve_info}\n\nChecklist findings:\n{findings}"}],
                    temperature=0.0, max_tokens=200)
                res.summary = str(getattr(r, "content", r) or "")  # message objects and plain strings alike
        except Exception as e:  # noqa: BLE001 - one bad CVE does not fail the batch
            res.error = f"{type(e).__name__}: {e}"
        res.latency_ms = (time.perf_counter() - t0) * 1e3
        return res

    def _indexed(self, cves: Sequence[str]) -> Iterator[tuple]:
        if not cves:
            return
        # item agents run on their own pool so a CVE waiting on its items never starves them of workers
        with ThreadPoolExecutor(max_workers=self.max_concurrency) as items, \
                ThreadPoolExecutor(max_workers=max(1, min(len(cves), self.max_concurrency))) as outer:
            futs = {outer.submit(self._one, c, items): i for i, c in enumerate(cves)}
            for f in as_completed(futs):
                yield futs[f], f.result()

    def scan_iter(self, cves: Sequence[str]) -> Iterator[CVEResult]:
        """Results in completion order."""
        for _, r in self._indexed(cves):
            yield r

    def scan(self, cves: Sequence[str]) -> List[CVEResult]:
        """Results in input order."""
        out: List[Optional[CVEResult]] = [None] * len(cves)
        for i, r in self._indexed(cves):
            out[i] = r
        return out  # type: ignore[return-value]


def timing_table(engine: CVEEngine, cves: Sequence[str], counts=(1, 5, 10)) -> List[dict]:
    """The reference notebook's benchmark: total and per-CVE wall time for batches of 1 / 5 / 10 CVEs."""
    rows = []
    for n in counts:
        batch = [cves[i % len(cves)] for i in range(n)]
        t0 = time.perf_counter()
        engine.scan(batch)
        total = (time.perf_counter() - t0) * 1e3
        rows.append({"cves": n, "total_ms": total, "avg_ms": total / n})
    return rows


def create_app(engine_factory: Callable[[], CVEEngine]):
    from fastapi import FastAPI
    from fastapi.responses import StreamingResponse
    from starlette.concurrency import iterate_in_threadpool, run_in_threadpool

    app = FastAPI(title="CVE exploitability triage")

    @app.post("/scan")
    async def scan(items: List[ScanItem]):
        res = await run_in_threadpool(engine_factory().scan, [i.cve_info for i in items])
        return [asdict(r) for r in res]

    @app.post("/scan/stream")
    async def scan_stream(items: List[ScanItem]):
        it = engine_factory().scan_iter([i.cve_info for i in items])
        return StreamingResponse(iterate_in_threadpool(json.dumps(asdict(r)) + "\n" for r in it),
                                 media_type="application/x-ndjson")

    return app


def _default_engine(sbom: Optional[str], code_collection: Optional[str]) -> CVEEngine:
    from ...chain_server.utils import get_llm, get_vectorstore

    code = CodeSearch(get_vectorstore(collection=code_collection)) if code_collection else None
    return CVEEngine(get_llm(), tools=default_tools(SBOMChecker.from_csv(sbom) if sbom else None, code))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sbom", help="CSV with package,version columns")
    ap.add_argument("--code-collection", help="HBM collection holding the container's source code")
    ap.add_argument("--cve", action="append", default=[], help="CVE description (repeatable)")
    ap.add_argument("--serve", action="store_true", help="serve POST /scan instead of scanning --cve")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=26302)
    a = ap.parse_args()
    if a.serve:
        import uvicorn

        engine = _default_engine(a.sbom, a.code_collection)
        uvicorn.run(create_app(lambda: engine), host=a.host, port=a.port)
        return
    for r in _default_engine(a.sbom, a.code_collection).scan(a.cve):
        print(json.dumps(asdict(r), indent=1))


if __name__ == "__main__":
    main()
