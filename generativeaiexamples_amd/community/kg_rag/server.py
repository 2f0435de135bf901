"""Backend of the knowledge-graph RAG app (reference: /root/reference/community/knowledge_graph_rag/backend/server.py
and routers/{ui_backend,chat,evaluation,visualization}.py):

  GET  /get-models/                   served chat models
  POST /process-documents/            {directory, model_id}: split + extract triples in the background, index the chunks
                                      in the hybrid collection, write entities / relations / triples CSVs, documents.csv
                                      and knowledge_graph.graphml under ``data_dir``
  GET  /progress/                     fraction of chunks processed
  GET  /check-file-exists/            whether the GraphML graph exists
  POST /chat/                         {user_input, use_kg, model_id} -> answer with graph + passage context
  POST /create-qa-pairs/              {num_data, model_id}: synthetic QA pairs (NDJSON stream, also qa_data.csv)
  POST /run-evaluation/               {questions_list, answers_list, model_id}: text / graph / combined answers (NDJSON)
  POST /run-scoring_llm_as_a_judge/   {combined_results}: 1-4 judge ratings per variant (NDJSON)
  POST /run-scoring-RAGAS/            {combined_results}: answer relevancy + context precision per variant (NDJSON)
  POST /run-scoring/                  {combined_results}: reward-model scores per variant, when a reward model is given
  GET  /visualization                 the graph as {nodes, edges} JSON (optionally around one entity)

Models come from the framework's service hub (``llm_factory(model_id)``), the chunks live in an HBM collection with
BM25 fusion, and the graph is the in-process ``KnowledgeGraph`` (re-read from GraphML at start-up when present).

  python -m generativeaiexamples_amd.community.kg_rag.server --data-dir ./data --port 8000
"""
from __future__ import annotations

import argparse
import asyncio
import csv
import json
import os
import threading
from typing import Callable, Dict, List, Optional

from fastapi import BackgroundTasks, FastAPI, HTTPException
from fastapi.responses import JSONResponse, StreamingResponse
from pydantic import BaseModel
from starlette.concurrency import iterate_in_threadpool

from ...index.hbm_index import Document
from .extract import generate_qa_pair, judge_answer, process_documents, sample_documents
from .graph import KnowledgeGraph
from .rag import KGRag

SCORE_COLUMNS = (("gt", "gt_answer", "combined_RAG_context_response"),
                 ("textRAG", "textRAG_answer", "text_RAG_context_response"),
                 ("graphRAG", "graphRAG_answer", "graph_RAG_context_response"),
                 ("combinedRAG", "combined_answer", "combined_RAG_context_response"))


class DirectoryRequest(BaseModel):
    directory: str
    model_id: str = ""


class ChatRequest(BaseModel):
    user_input: str
    use_kg: bool = True
    model_id: str = ""


class QAPairsRequest(BaseModel):
    num_data: int
    model_id: str = ""


class QARequest(BaseModel):
    questions_list: list
    answers_list: list
    model_id: str = ""


class ScoreRequest(BaseModel):
    combined_results: list


def _contexts(v) -> List[str]:
    if isinstance(v, list):
        return [str(x) for x in v]
    return [s.strip() for s in str(v or "").split(",") if s.strip()]


def create_app(llm_factory: Callable[[str], object], store, data_dir: str, models: Callable[[], list] = lambda: [],
               ranker=None, judge_llm_factory: Optional[Callable[[], object]] = None, embed=None,
               reward_fn: Optional[Callable[[str, str], Optional[Dict[str, float]]]] = None,
               max_workers: int = 8) -> FastAPI:
    app = FastAPI(title="Knowledge-graph RAG")

    @app.on_event("startup")
    async def _worker_threads():
        # streamed responses hold a worker thread per waiting stream: anyio's default 40 would queue a burst
        import anyio

        anyio.to_thread.current_default_thread_limiter().total_tokens = int(os.environ.get("GAI_SERVER_THREADS", "256"))
    os.makedirs(data_dir, exist_ok=True)
    graphml = os.path.join(data_dir, "knowledge_graph.graphml")
    state = {"graph": KnowledgeGraph.read_graphml(graphml) if os.path.exists(graphml) else KnowledgeGraph(),
             "progress": 0.0, "error": None}
    lock = threading.Lock()
    judge_factory = judge_llm_factory or (lambda: llm_factory(""))

    def rag(model_id: str) -> KGRag:
        return KGRag(llm_factory(model_id), state["graph"], store, ranker)

    @app.get("/get-models/")
    async def get_models():
        return {"models": list(models())}

    def ingest(directory: str, model_id: str):
        def progress(done, total):
            state["progress"] = done / max(total, 1)

        try:
            chunks, graph = process_documents(directory, llm_factory(model_id), max_workers=max_workers,
                                              update_progress=progress)
            if chunks:
                store.add_documents([Document(c.page_content, {k: v for k, v in c.metadata.items() if k != "triples"})
                                     for c in chunks])
            with open(os.path.join(data_dir, "documents.csv"), "w", newline="") as f:
                w = csv.writer(f)
                w.writerow(["content"])
                w.writerows([c.page_content] for c in chunks)
            with lock:
                # merged into a copy and swapped in: chat requests read the current graph without the lock
                merged = KnowledgeGraph()
                merged.merge(state["graph"])
                merged.merge(graph)
                merged.to_csvs(data_dir)
                merged.write_graphml(graphml)
                state["graph"] = merged
            state["progress"] = 1.0
        except Exception as e:  # noqa: BLE001 - surfaced through /progress/
            state["error"] = str(e)

    @app.post("/process-documents/")
    async def process_documents_endpoint(req: DirectoryRequest, background_tasks: BackgroundTasks):
        if not os.path.isdir(req.directory):
            raise HTTPException(404, f"directory {req.directory!r} not found")
        state["progress"], state["error"] = 0.0, None
        background_tasks.add_task(ingest, req.directory, req.model_id)
        return {"message": "Processing started"}

    @app.get("/progress/")
    async def get_progress():
        out = {"progress": str(state["progress"])}
        if state["error"]:
            out["error"] = state["error"]
        return out

    @app.get("/check-file-exists/")
    async def check_file_exists():
        return JSONResponse({"file_exists": os.path.exists(graphml)})

    @app.post("/chat/")
    async def chat(req: ChatRequest):
        return await asyncio.to_thread(rag(req.model_id).chat, req.user_input, req.use_kg)

    def _ndjson(rows):
        # the rows come from blocking model calls: produced in the thread pool, never on the event loop
        async def gen():
            async for row in iterate_in_threadpool(rows()):
                yield json.dumps(row) + "\n"
        return StreamingResponse(gen(), media_type="text/event-stream")

    @app.post("/create-qa-pairs/")
    async def create_qa_pairs(req: QAPairsRequest):
        path = os.path.join(data_dir, "documents.csv")
        if not os.path.exists(path):
            raise HTTPException(404, "Documents not found. Please process documents first.")
        with open(path, newline="") as f:
            docs = [Document(r["content"], {}) for r in csv.DictReader(f)]
        llm = llm_factory(req.model_id)

        def rows():
            pairs = []
            for d in sample_documents(docs, req.num_data):
                try:
                    p = generate_qa_pair(d.page_content, llm)
                except Exception as e:  # noqa: BLE001
                    yield {"error": str(e)}
                    continue
                if p:
                    pairs.append(p)
                    yield p
            with open(os.path.join(data_dir, "qa_data.csv"), "w", newline="") as f:
                w = csv.DictWriter(f, fieldnames=["question", "answer"])
                w.writeheader()
                w.writerows(pairs)
        return _ndjson(rows)

    @app.post("/run-evaluation/")
    async def run_evaluation(req: QARequest):
        r = rag(req.model_id)

        def rows():
            path = os.path.join(data_dir, "combined_results.csv")
            for q, a in zip(req.questions_list, req.answers_list):
                res = r.evaluate_question(q, a)
                new = not os.path.exists(path) or os.path.getsize(path) == 0
                with open(path, "a", newline="") as f:
                    w = csv.DictWriter(f, fieldnames=list(res.keys()))
                    if new:
                        w.writeheader()
                    w.writerow({k: json.dumps(v) if isinstance(v, list) else v for k, v in res.items()})
                yield res
        return _ndjson(rows)

    @app.post("/run-scoring_llm_as_a_judge/")
    async def run_scoring_judge(req: ScoreRequest):
        llm = judge_factory()

        def rows():
            for row in req.combined_results:
                try:
                    for name, col, _ in SCORE_COLUMNS:
                        for k, v in judge_answer(row["question"], row[col], llm).items():
                            row[f"{name}_{k}"] = v
                    yield row
                except Exception as e:  # noqa: BLE001
                    yield {"error": str(e)}
        return _ndjson(rows)

    @app.post("/run-scoring-RAGAS/")
    async def run_scoring_ragas(req: ScoreRequest):
        from ...evaluation.ragas_llm import RagasJudge

        llm = judge_factory()

        def judge_fn(messages, schema=None):
            kw = {"response_format": {"type": "json_schema", "json_schema": {"schema": schema}}} if schema else {}
            try:
                r = llm.invoke(messages, temperature=0.0, max_tokens=300, **kw)
            except TypeError:
                r = llm.invoke(messages)
            return getattr(r, "content", r)

        judge = RagasJudge(judge_fn, embed)

        def rows():
            for row in req.combined_results:
                try:
                    for name, col, ctx_col in SCORE_COLUMNS:
                        ctxs = _contexts(row.get(ctx_col))
                        if embed is not None:
                            row[f"{name}_answer_relevancy"] = judge.answer_relevancy(row["question"], row[col])
                        row[f"{name}_context_precision"] = judge.context_precision(row["question"], row["gt_answer"],
                                                                                   ctxs)
                    yield row
                except Exception as e:  # noqa: BLE001
                    yield {"error": str(e)}
        return _ndjson(rows)

    @app.post("/run-scoring/")
    async def run_scoring(req: ScoreRequest):
        if reward_fn is None:
            raise HTTPException(501, "no reward model is configured")

        def rows():
            for row in req.combined_results:
                for name, col, _ in SCORE_COLUMNS:
                    for k, v in (reward_fn(row["question"], row[col]) or {}).items():
                        row[f"{name}_{k}"] = v
                yield row
        return _ndjson(rows)

    @app.get("/visualization")
    async def visualization(entity: Optional[str] = None, depth: int = 2, limit: int = 2000):
        g = state["graph"]
        if entity:
            facts = set(g.entity_knowledge(entity, depth=depth, both_directions=True))
            edges = [e for e in g.triples() if f"{e[0]} {e[1]} {e[2]}" in facts]
        else:
            edges = g.triples()
        edges = edges[:limit]
        names = sorted({e[0] for e in edges} | {e[2] for e in edges})
        types = {n: g.types.get(n.lower(), "Unknown") for n in names}
        return {"nodes": [{"id": n, "type": types[n]} for n in names],
                "edges": [{"source": s, "relation": r, "target": t} for s, r, t in edges]}

    app.state.kg = state
    return app


def default_app(data_dir: str) -> FastAPI:
    """Wired to the chain-server factories: the configured LLM, a hybrid HBM collection, the ranker."""
    from ...chain_server.utils import get_config, get_embedding_model, get_hub, get_llm, get_ranking_model
    from ...chain_server.vectorstore import VectorStore

    store = VectorStore(os.environ.get("KG_COLLECTION", "kg_rag_hybrid"), get_embedding_model(), hybrid=True,
                        persist_dir=os.environ.get("APP_VECTORSTORE_PERSISTDIR"))

    def models():
        try:
            name = get_config().llm.model_name
            return [name] if get_hub().llm(name) is not None else []
        except Exception:  # noqa: BLE001
            return []

    return create_app(lambda model_id: get_llm(), store, data_dir, models, get_ranking_model())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8000)
    ap.add_argument("--data-dir", default=os.environ.get("DATA_DIR", "data"))
    a = ap.parse_args()
    import uvicorn

    uvicorn.run(default_app(a.data_dir), host=a.host, port=a.port)


if __name__ == "__main__":
    main()
