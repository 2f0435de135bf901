"""RAG server of the RAG-Blueprint-2.x API with the sizing advisor's extensions (reference: /root/reference/community/
vgpu-sizing-advisor/src/server.py:131-1760):

  GET  /health                 service + collection health
  POST /generate               chat messages -> SSE ``data: {ChainResponse}`` chunks (OpenAI chunk shape; citations on
                               the first chunk, usage + finish_reason "stop" on the last); per-request collection,
                               vdb_top_k / reranker_top_k, query rewriting, reranker, guardrails, citations switches
  POST /chat/completions       alias of /generate
  POST /search                 retrieval only -> Citations
  POST /generate_structured    a deployment recommendation as structured JSON: the model (with retrieved context)
                               picks model / GPUs / concurrency / token budgets, the MI355X sizing planner
                               (``generativeaiexamples_amd.sizing.plan``) turns them into memory + latency figures
  GET  /available-models       the framework's LLM presets with parameter counts
  GET  /detect-gpu             the local GPU (HIP runtime)
  POST /test-configuration     SSE: plan, then a measured run of the configuration on this engine (``deploy.py``)
  POST /apply-configuration    SSE: start the framework's OpenAI server with the configuration (``deploy.py``)
  GET  /api/download-citation  a source file of a collection (basename only)
"""
from __future__ import annotations

import json
import os
import re
import threading
import time
import uuid
from typing import Callable, Iterator, List, Literal, Optional

from fastapi import FastAPI, HTTPException
from fastapi.responses import FileResponse, JSONResponse, StreamingResponse
from pydantic import BaseModel, Field
from starlette.concurrency import iterate_in_threadpool, run_in_threadpool

from ...chain_server.connectors import rerank
from ...index.hbm_index import Document
from .store import CollectionManager

DEFAULT_COLLECTION = os.environ.get("COLLECTION_NAME", "multimodal_data")
RAG_SYSTEM = ("You are a helpful assistant. Answer the user's question using the context below; if the context does "
              "not contain the answer, say so. Context:\n{context}")
CHAT_SYSTEM = "You are a helpful assistant."
REWRITE_SYSTEM = ("Rewrite the user's last question as a single standalone search query, resolving references to the "
                  "earlier conversation. Reply with the query only.")
STRUCTURED_SYSTEM = (
    "You recommend a GPU deployment for serving an LLM on AMD Instinct GPUs. From the request and the context, choose "
    "values and reply with JSON only: {{\"model\": <one of {models}>, \"num_gpus\": <1|2|4|8 or null to let the "
    "planner choose>, \"concurrency\": <concurrent requests>, \"prompt_tokens\": <int>, \"response_tokens\": <int>, "
    "\"dtype\": \"bf16\"|\"fp8\", \"kv_dtype\": \"bf16\"|\"fp8\", \"reasoning\": <one sentence>}}.\nContext:\n"
    "{context}")


class Message(BaseModel):
    role: Optional[Literal["user", "assistant", "system"]] = "user"
    content: str = ""


class Prompt(BaseModel):
    messages: List[Message]
    use_knowledge_base: bool = True
    temperature: float = Field(0.2, ge=0.0, le=2.0)
    top_p: float = Field(0.7, ge=0.0, le=1.0)
    max_tokens: int = Field(1024, ge=1, le=131072)
    reranker_top_k: int = Field(4, ge=0, le=25)
    vdb_top_k: int = Field(10, ge=1, le=400)
    collection_name: str = DEFAULT_COLLECTION
    enable_query_rewriting: bool = False
    enable_reranker: bool = True
    enable_guardrails: bool = False
    enable_citations: bool = True
    model: str = ""
    stop: List[str] = Field(default_factory=list)


class DocumentSearch(BaseModel):
    query: str
    reranker_top_k: int = Field(4, ge=0, le=25)
    vdb_top_k: int = Field(10, ge=1, le=400)
    collection_name: str = DEFAULT_COLLECTION
    messages: List[Message] = Field(default_factory=list)
    enable_query_rewriting: bool = False
    enable_reranker: bool = True


class DeploymentConfig(BaseModel):
    model: str = "llama3-8b"
    num_gpus: Optional[int] = None
    concurrency: int = Field(64, ge=1, le=4096)
    prompt_tokens: int = Field(2400, ge=1, le=131072)
    response_tokens: int = Field(256, ge=1, le=32768)
    dtype: Literal["bf16", "fp8"] = "bf16"
    kv_dtype: Literal["bf16", "fp8"] = "bf16"


class ConfigurationRequest(BaseModel):
    configuration: DeploymentConfig = Field(default_factory=DeploymentConfig)
    deployment_mode: Literal["local"] = "local"
    measure: bool = True
    measure_concurrency: Optional[int] = Field(None, ge=1, le=512)
    port: int = 8000


def _count_tokens(llm, text: str) -> int:
    tok = getattr(getattr(llm, "engine", None), "tokenizer", None)
    try:
        return len(tok.encode(text)) if tok is not None else len(text.split())
    except Exception:  # noqa: BLE001
        return len(text.split())


def _citations(hits: List[Document], enable: bool = True) -> dict:
    if not enable:
        return {"total_results": 0, "results": []}
    res = []
    for d in hits:
        md = d.metadata
        res.append({"document_id": str(md.get("row", md.get("id", ""))), "content": d.page_content,
                    "document_name": md.get("filename", md.get("source", "")),
                    "document_type": md.get("type", "text") if md.get("type") in ("image", "table", "chart")
                    else "text", "score": float(md.get("relevance_score", md.get("score", 0.0))),
                    "metadata": {"page_number": int(md.get("page", 0) or 0), "language": md.get("language", ""),
                                 "description": md.get("description", "")}})
    return {"total_results": len(res), "results": res}


def _chunk(resp_id: str, model: str, delta: str, acc: str, finish: Optional[str] = None, citations=None,
           usage=None) -> str:
    body = {"id": resp_id, "object": "chat.completion.chunk", "model": model, "created": int(time.time()),
            "choices": [{"index": 0, "message": {"role": "assistant", "content": acc},
                         "delta": {"role": None, "content": delta}, "finish_reason": finish}]}
    if citations is not None:
        body["citations"] = citations
    if usage is not None:
        body["usage"] = usage
    return "data: " + json.dumps(body) + "\n\n"


class BlueprintRag:
    """Retrieval + generation shared by the /generate, /search and /generate_structured routes."""

    def __init__(self, llm_factory: Callable[[str], object], manager: CollectionManager, ranker=None,
                 guardrails=None):
        self.llm_factory, self.manager, self.ranker, self.guardrails = llm_factory, manager, ranker, guardrails

    def rewrite(self, llm, messages: List[Message], query: str) -> str:
        history = [m for m in messages[:-1] if m.content.strip()]
        if not history:
            return query
        convo = "\n".join(f"{m.role}: {m.content}" for m in history) + f"\nuser: {query}"
        out = llm.invoke([{"role": "system", "content": REWRITE_SYSTEM}, {"role": "user", "content": convo}],
                         temperature=0.0, max_tokens=96)
        return (out or "").strip().splitlines()[0].strip() if (out or "").strip() else query

    def retrieve(self, query: str, collection: str, vdb_top_k: int, reranker_top_k: int,
                 use_reranker: bool) -> List[Document]:
        try:
            hits = self.manager.search(collection, query, vdb_top_k)
        except KeyError:
            return []
        docs = [Document(d.page_content, dict(d.metadata, relevance_score=float(s))) for d, s in hits]
        k = reranker_top_k or len(docs)
        if use_reranker and self.ranker is not None and docs:
            docs = rerank(self.ranker, docs, query, k)
        return docs[:k]

    def _messages(self, p: Prompt, query: str, docs: List[Document]) -> List[dict]:
        system = RAG_SYSTEM.format(context="\n\n".join(d.page_content for d in docs)) if p.use_knowledge_base \
            else CHAT_SYSTEM
        sys_extra = [m.content for m in p.messages if m.role == "system" and m.content.strip()]
        if sys_extra:
            system = "\n".join(sys_extra) + "\n" + system
        hist = [{"role": m.role, "content": m.content} for m in p.messages[:-1]
                if m.role in ("user", "assistant") and m.content.strip()]
        return [{"role": "system", "content": system}] + hist + [{"role": "user", "content": query}]

    def stream(self, p: Prompt) -> Iterator[str]:
        resp_id, llm = str(uuid.uuid4()), self.llm_factory(p.model)
        users = [m for m in p.messages if m.role == "user"]
        query = users[-1].content if users else ""
        docs: List[Document] = []
        if p.use_knowledge_base:
            q = self.rewrite(llm, p.messages, query) if p.enable_query_rewriting else query
            docs = self.retrieve(q, p.collection_name, p.vdb_top_k, p.reranker_top_k, p.enable_reranker)
        msgs = self._messages(p, query, docs)

        def gen():
            return iter(llm.stream(msgs, temperature=p.temperature, top_p=p.top_p, max_tokens=p.max_tokens,
                                   stop=p.stop or None))

        pieces = self.guardrails.generate(query, gen) if (p.enable_guardrails and self.guardrails) else gen()
        acc, first = "", True
        for piece in pieces:
            if not piece:
                continue
            acc += piece
            yield _chunk(resp_id, p.model, piece, acc, citations=_citations(docs, p.enable_citations) if first
                         else None)
            first = False
        usage = {"prompt_tokens": sum(_count_tokens(llm, m["content"]) for m in msgs),
                 "completion_tokens": _count_tokens(llm, acc)}
        usage["total_tokens"] = usage["prompt_tokens"] + usage["completion_tokens"]
        yield _chunk(resp_id, p.model, "", "", finish="stop",
                     citations=_citations(docs, p.enable_citations) if first else None, usage=usage)

    def structured(self, p: Prompt) -> dict:
        from ... import sizing
        from ...models.registry import LLM_PRESETS

        llm = self.llm_factory(p.model)
        users = [m for m in p.messages if m.role == "user"]
        query = users[-1].content if users else ""
        docs = self.retrieve(query, p.collection_name, p.vdb_top_k, p.reranker_top_k, p.enable_reranker) \
            if p.use_knowledge_base else []
        presets = [k for k in LLM_PRESETS if not k.startswith("tiny")]
        reply = llm.invoke([{"role": "system", "content": STRUCTURED_SYSTEM.format(
            models=", ".join(presets), context="\n\n".join(d.page_content for d in docs) or "(none)")},
            {"role": "user", "content": query}], temperature=0.0, max_tokens=256)
        cfg, reasoning = _structured_config(reply or "", query, presets)
        plan = sizing.plan(cfg.model, "MI355X", cfg.num_gpus, cfg.concurrency, cfg.prompt_tokens,
                           cfg.response_tokens, cfg.dtype, cfg.kv_dtype)
        return {"structured_output": {"title": "generate_mi355x_config", "description": reasoning,
                                      "configuration": cfg.model_dump(), "parameters": plan},
                "citations": _citations(docs, p.enable_citations), "model": p.model, "created": int(time.time()),
                "id": str(uuid.uuid4())}


def _structured_config(reply: str, query: str, presets: List[str]):
    """Model JSON when it parses and names a known preset; otherwise the request text is scanned for a preset name and
    numbers (the reference wraps unparseable replies in a fixed schema instead)."""
    from ..fm_asr.chains import first_json_object

    obj = first_json_object(reply) or {}
    fields = {k: obj.get(k) for k in ("model", "num_gpus", "concurrency", "prompt_tokens", "response_tokens",
                                      "dtype", "kv_dtype") if obj.get(k) is not None}
    low = query.lower()
    if fields.get("model") not in presets:
        fields["model"] = next((p for p in sorted(presets, key=len, reverse=True) if p in low), "llama3-8b")
        for key, pat in (("concurrency", r"(\d+)\s*(?:concurrent|users|requests|sessions)"),
                         ("num_gpus", r"(\d+)\s*(?:x\s*)?(?:gpus?|mi3\d\dx?)")):
            m = re.search(pat, low)
            if m and key not in fields:
                fields[key] = int(m.group(1))
        if "fp8" in low:
            fields.setdefault("dtype", "fp8")
    if fields.get("num_gpus") not in (None, 1, 2, 4, 8):
        fields["num_gpus"] = None
    try:
        cfg = DeploymentConfig(**fields)
    except Exception:  # noqa: BLE001 - out-of-range model values: keep only the model choice
        cfg = DeploymentConfig(model=fields["model"])
    return cfg, str(obj.get("reasoning") or f"Sizing for {cfg.model} at {cfg.concurrency} concurrent requests.")


def _available_models() -> List[dict]:
    from ... import sizing
    from ...models.registry import LLM_PRESETS

    out = []
    for key, (name, _) in LLM_PRESETS.items():
        if key.startswith("tiny"):
            continue
        try:
            size = f"{sizing.ModelSpec.from_preset(key).params_b:.1f}B"
        except Exception:  # noqa: BLE001 - non-Llama geometry (OPT / hybrid) without a params formula
            m = re.search(r"(\d+(?:\.\d+)?)[Bb]", name)
            size = m.group(0) if m else ""
        out.append({"id": key, "name": name.split("/")[-1], "label": name.split("/")[-1].replace("-", " "),
                    "size": size, "modelTag": name})
    return out


def create_rag_app(llm_factory: Callable[[str], object], manager: CollectionManager, ranker=None, guardrails=None,
                   models: Callable[[], list] = lambda: [],
                   measure_fn: Optional[Callable[..., dict]] = None,
                   launch_fn: Optional[Callable[..., Iterator[dict]]] = None,
                   detect_fn: Optional[Callable[[], Optional[dict]]] = None) -> FastAPI:
    from . import deploy

    rag = BlueprintRag(llm_factory, manager, ranker, guardrails)
    measure_fn = measure_fn or deploy.measure_config
    launch_fn = launch_fn or deploy.launch_server
    detect_fn = detect_fn or deploy.detect_gpu
    app = FastAPI(title="RAG server (sizing advisor)")

    @app.on_event("startup")
    async def _worker_threads():
        # streamed responses hold a worker thread per waiting stream: anyio's default 40 would queue a burst
        import anyio

        anyio.to_thread.current_default_thread_limiter().total_tokens = int(os.environ.get("GAI_SERVER_THREADS", "256"))

    @app.get("/health")
    async def health():
        cols = manager.list()["collections"]
        return {"message": "Service is up.",
                "databases": [{"service": "hbm-index", "url": "in-process", "status": "healthy",
                               "collections": len(cols)}],
                "object_storage": [], "nim": [{"service": "llm", "model": m, "status": "healthy"} for m in models()]}

    async def _sse(p: Prompt):
        return StreamingResponse(iterate_in_threadpool(rag.stream(p)), media_type="text/event-stream")

    @app.post("/generate")
    async def generate(p: Prompt):
        return await _sse(p)

    @app.post("/chat/completions")
    async def chat_completions(p: Prompt):
        return await _sse(p)

    @app.post("/search")
    async def search(s: DocumentSearch):
        def run():
            q = s.query
            if s.enable_query_rewriting and s.messages:
                q = rag.rewrite(llm_factory(""), s.messages + [Message(role="user", content=s.query)], s.query)
            return _citations(rag.retrieve(q, s.collection_name, s.vdb_top_k, s.reranker_top_k, s.enable_reranker))
        return await run_in_threadpool(run)

    @app.post("/generate_structured")
    async def generate_structured(p: Prompt):
        try:
            return await run_in_threadpool(rag.structured, p)
        except KeyError as e:
            return JSONResponse({"error": f"unknown model preset {e}"}, status_code=400)

    @app.get("/available-models")
    async def available_models():
        return {"models": _available_models()}

    @app.get("/detect-gpu")
    async def detect_gpu():
        info = await run_in_threadpool(detect_fn)
        if info is None:
            return JSONResponse({"error": "No GPU detected"}, status_code=404)
        return info

    measure_lock = threading.Lock()

    def _events(it: Iterator[dict]):
        return StreamingResponse(iterate_in_threadpool(f"data: {json.dumps(e)}\n\n" for e in it),
                                 media_type="text/event-stream", headers={"Cache-Control": "no-cache"})

    @app.post("/test-configuration")
    async def test_configuration(req: ConfigurationRequest):
        from ... import sizing

        c = req.configuration

        def events():
            yield {"status": "planning"}
            try:
                plan = sizing.plan(c.model, "MI355X", c.num_gpus, c.concurrency, c.prompt_tokens, c.response_tokens,
                                   c.dtype, c.kv_dtype)
            except KeyError:
                yield {"status": "error", "message": f"unknown model preset {c.model!r}"}
                return
            yield {"status": "plan", "plan": plan}
            if not req.measure:
                yield {"status": "done"}
                return
            gpu = detect_fn()
            if gpu is None:
                yield {"status": "skipped", "message": "no GPU on this host; the plan is analytic only"}
                return
            if plan["tp"] > 1:
                yield {"status": "skipped", "message": f"the plan needs TP={plan['tp']}: use /apply-configuration "
                                                       "and a served benchmark"}
                return
            n = req.measure_concurrency or min(c.concurrency, plan["max_concurrent_sequences"] or 1)
            # a measurement loads the model on this process's GPU: one at a time, never two models side by side
            if not measure_lock.acquire(blocking=False):
                yield {"status": "busy", "message": "another configuration is being measured; retry when it ends"}
                return
            try:
                yield {"status": "measuring", "gpu": gpu, "concurrency": n}
                m = measure_fn(c.model, concurrency=n, prompt=c.prompt_tokens, response=c.response_tokens)
            except Exception as e:  # noqa: BLE001
                yield {"status": "error", "message": "measurement failed", "error": str(e)}
                return
            finally:
                measure_lock.release()
            yield {"status": "done", "measured": m,
                   "estimated": {"tpot_ms": plan["tpot_ms"], "ttft_s_single": plan["ttft_s_single"]}}

        return _events(events())

    @app.post("/apply-configuration")
    async def apply_configuration(req: ConfigurationRequest):
        from ... import sizing

        c = req.configuration
        try:
            tp = sizing.plan(c.model, "MI355X", c.num_gpus, c.concurrency, c.prompt_tokens, c.response_tokens,
                             c.dtype, c.kv_dtype)["tp"]
        except KeyError:
            raise HTTPException(400, f"unknown model preset {c.model!r}")
        preset = c.model + ("-fp8" if c.dtype == "fp8" else "")
        extra = ["--kv-cache-dtype", "fp8"] if c.kv_dtype == "fp8" else []
        return _events(launch_fn(preset, tp=tp, port=req.port, max_num_seqs=c.concurrency, extra_args=extra))

    @app.get("/api/download-citation")
    async def download_citation(source: str, collection_name: str = DEFAULT_COLLECTION):
        path = os.path.join(manager.upload_dir, os.path.basename(collection_name), os.path.basename(source))
        if not os.path.isfile(path):
            raise HTTPException(404, "file not found")
        return FileResponse(path, filename=os.path.basename(source))

    app.state.rag = rag
    return app


def main():
    import argparse

    import uvicorn

    from ...chain_server.utils import get_config, get_embedding_model, get_llm, get_ranking_model
    from .ingestor import create_ingestor_app

    ap = argparse.ArgumentParser(description="RAG server (port) + ingestor server (ingestor-port) in ONE process, "
                                             "sharing the in-HBM collections (the reference runs two containers "
                                             "around an external Milvus)")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8081)
    ap.add_argument("--ingestor-port", type=int, default=8082)
    ap.add_argument("--data-dir", default=os.environ.get("APP_VECTORSTORE_PERSISTDIR", "data"))
    a = ap.parse_args()
    mgr = CollectionManager(get_embedding_model(), os.path.join(a.data_dir, "uploads"),
                            persist_dir=os.path.join(a.data_dir, "collections"))
    rag_app = create_rag_app(lambda model: get_llm(), mgr, get_ranking_model(),
                             models=lambda: [get_config().llm.model_name])
    servers = [uvicorn.Server(uvicorn.Config(app, host=a.host, port=port))
               for app, port in ((rag_app, a.port), (create_ingestor_app(mgr), a.ingestor_port))]

    import asyncio

    async def serve():
        await asyncio.gather(*(s.serve() for s in servers))

    asyncio.run(serve())


if __name__ == "__main__":
    main()
