"""Chain server of the FM-radio streaming RAG app (reference: /root/reference/community/fm-asr-streaming-rag/
chain-server/server.py:37-74): ``POST /storeStreamingText`` feeds transcripts to the text accumulator,
``GET|POST /generate`` streams an answer (intent-routed, ``chains.py``), ``GET /serverStatus`` and
``GET /availableNvidiaModels`` as in the reference. The models come from the framework's in-process service hub
(or a remote endpoint, per the APP_* configuration) and the stream's chunks live in the HBM vector index.

  python -m generativeaiexamples_amd.community.fm_asr.server --port 8081
"""
from __future__ import annotations

import argparse
import datetime as _dt
import os
from typing import Callable, Optional

from fastapi import FastAPI, HTTPException, Request
from fastapi.responses import JSONResponse, StreamingResponse
from pydantic import BaseModel, Field, ValidationError
from starlette.concurrency import run_in_threadpool

from .chains import StreamQuery, StreamRagChain
from .stream_store import StreamRetriever, TextAccumulator, TimestampDatabase


class TextEntry(BaseModel):
    transcript: str = Field(..., description="Streaming text to store")
    source_id: str = Field("fm-radio", description="Source of the text")
    timestamp: Optional[_dt.datetime] = Field(None, description="Timestamp of the text (arrival time is used)")


class StreamConfig(BaseModel):
    question: str = Field(..., description="The input query/prompt to the pipeline.")
    context: Optional[str] = Field(None, description="Additional context for the question (optional)")
    name: Optional[str] = Field(None, description="Name of the LLM to use (the served model when omitted)")
    engine: Optional[str] = Field(None, description="Engine of the LLM (informational)")
    use_knowledge_base: bool = Field(True, description="Whether to use the transcript store")
    allow_summary: bool = Field(False, description="Use recursive summarization to reduce long contexts")
    temperature: float = Field(0.2, ge=0.0, le=2.0, description="Temperature of the LLM response")
    max_docs: int = Field(8, ge=1, le=256, description="Maximum number of transcript chunks in the context")
    num_tokens: int = Field(512, ge=1, le=32768, description="Maximum number of tokens in the response")


def create_app(llm_factory: Callable[[], object], accumulator: TextAccumulator, retriever: StreamRetriever,
               models: Callable[[], list] = lambda: []) -> FastAPI:
    app = FastAPI(title="FM radio streaming RAG")

    @app.get("/serverStatus")
    async def server_status():
        return {"is_ready": True}

    @app.get("/availableNvidiaModels")
    async def available_models():
        return JSONResponse({"local_models": list(models()), "cloud_models": []})

    @app.post("/storeStreamingText")
    async def store_streaming_text(data: TextEntry):
        # the accumulator embeds the finished chunks: a blocking model call, kept off the event loop
        return JSONResponse(await run_in_threadpool(accumulator.update, data.source_id, data.transcript))

    async def _generate(cfg: StreamConfig):
        q = StreamQuery(question=cfg.question, use_knowledge_base=cfg.use_knowledge_base,
                        allow_summary=cfg.allow_summary, temperature=cfg.temperature, max_docs=cfg.max_docs,
                        num_tokens=cfg.num_tokens, context=cfg.context)
        chain = StreamRagChain(llm_factory(), accumulator, retriever)
        return StreamingResponse(chain.answer(q), media_type="text/plain")

    @app.get("/generate")
    async def generate_get(request: Request):
        # the reference's client sends the config as a JSON body on GET
        body = await request.body()
        try:
            cfg = StreamConfig.model_validate_json(body) if body else StreamConfig(**dict(request.query_params))
        except ValidationError as e:
            raise HTTPException(422, e.errors(include_url=False, include_context=False)) from e
        return await _generate(cfg)

    @app.post("/generate")
    async def generate_post(cfg: StreamConfig):
        return await _generate(cfg)

    app.state.accumulator, app.state.retriever = accumulator, retriever
    return app


def default_app() -> FastAPI:
    """Wired to the chain-server factories: the configured LLM, embedder (passages into an HBM collection), ranker."""
    from ...chain_server.utils import get_config, get_hub, get_llm, get_ranking_model, get_vectorstore

    store = get_vectorstore(collection=os.environ.get("FM_COLLECTION", "FM_Radio_Stream_Collection"))
    retriever = StreamRetriever(store, get_ranking_model())
    acc = TextAccumulator(retriever, chunk_size=int(os.environ.get("DB_CHUNK_SIZE", 256)),
                          chunk_overlap=int(os.environ.get("DB_CHUNK_OVERLAP", 32)),
                          timestamp_db=TimestampDatabase(os.environ.get("FM_TIMESERIES_DB", ":memory:")))

    def models():
        try:
            return [get_config().llm.model_name] if get_hub().llm(get_config().llm.model_name) is not None else []
        except Exception:
            return []

    return create_app(lambda: get_llm(), acc, retriever, models)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8081)
    a = ap.parse_args()
    import uvicorn

    uvicorn.run(default_app(), host=a.host, port=a.port)


if __name__ == "__main__":
    main()
