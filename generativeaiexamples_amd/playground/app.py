"""RAG Playground web UI (the reference's Gradio-in-FastAPI playground, RAG/src/rag_playground/default/).

Pages: ``/`` and ``/converse`` (chat with a "Use knowledge base" switch, streamed answers, the
retrieved context shown next to the chat; the page calls /search before /generate when the
knowledge base is on, like pages/converse.py:100-119) and ``/kb`` (upload, list - refreshed every
5 s - and delete documents). The browser talks to this server's ``/api/*`` routes, which forward to
the chain server through :class:`ChatClient`, so the chain server needs no CORS exposure.
Config: ``APP_SERVERURL`` / ``APP_SERVERPORT`` / ``APP_MODELNAME`` (same names as the reference).
``/speech`` is the reference's speech playground (rag_playground/speech): microphone -> streaming ASR into
the question box, answers read back by TTS, through the pluggable backend of :mod:`.speech`
(``RIVA_API_URI``; routes ``/api/speech/status``, ``/api/speech/asr`` (WAV in), ``/api/speech/tts``
(WAV out)). ``/prompt-design`` is the community prompt-design helper (:mod:`.prompt_designer`: per-model system
prompt, few-shot examples and sampling settings in a YAML file (``PROMPT_DESIGN_CONFIG``), generate / compare models,
optional retrieved context).
"""
from __future__ import annotations

import os
import tempfile
from pathlib import Path

from fastapi import FastAPI, Request
from fastapi.responses import FileResponse, JSONResponse, RedirectResponse, StreamingResponse
from fastapi.staticfiles import StaticFiles
from starlette.concurrency import iterate_in_threadpool, run_in_threadpool

from ..chain_server.multipart import parse_multipart
from .chat_client import ChatClient

STATIC = Path(__file__).parent / "static"


def create_app(server_url: str | None = None, model_name: str | None = None,
               client: ChatClient | None = None, speech=None, designer=None) -> FastAPI:
    host = server_url or os.environ.get("APP_SERVERURL", "http://localhost")
    port = os.environ.get("APP_SERVERPORT", "8081")
    if server_url is None and ":" not in host.split("//")[-1]:
        host = f"{host}:{port}"
    client = client or ChatClient(host, model_name or os.environ.get("APP_MODELNAME", "meta/llama3-8b-instruct"))
    app = FastAPI(title="RAG Playground")
    app.state.client = client
    from .speech import backend_from_env, pcm_chunks, pcm_to_wav, wav_to_pcm16

    speech = speech if speech is not None else backend_from_env()
    app.state.speech = speech
    app.mount("/static", StaticFiles(directory=STATIC), name="static")

    @app.get("/")
    async def root():
        return RedirectResponse("/converse")

    @app.get("/converse")
    async def converse():
        return FileResponse(STATIC / "converse.html")

    @app.get("/kb")
    async def kb():
        return FileResponse(STATIC / "kb.html")

    @app.post("/api/search")
    async def search(req: Request):
        body = await req.json()
        chunks = await run_in_threadpool(client.search, body.get("query", ""), int(body.get("top_k", 4)))
        return {"chunks": chunks}

    @app.post("/api/generate")
    async def generate(req: Request):
        body = await req.json()
        gen = client.predict(body.get("query", ""), bool(body.get("use_knowledge_base", False)),
                             int(body.get("max_tokens", 1024)), body.get("history") or [])

        async def chunks():
            async for c in iterate_in_threadpool(gen):
                yield c

        return StreamingResponse(chunks(), media_type="text/plain; charset=utf-8")

    @app.get("/api/documents")
    async def documents():
        return {"documents": await run_in_threadpool(client.get_uploaded_documents)}

    @app.delete("/api/documents")
    async def delete(filename: str):
        return {"message": await run_in_threadpool(client.delete_documents, filename)}

    @app.post("/api/documents")
    async def upload(req: Request):
        parts = parse_multipart(req.headers.get("content-type", ""), await req.body())
        names = []
        with tempfile.TemporaryDirectory() as d:
            paths = []
            for p in parts:
                if p.filename:
                    fp = os.path.join(d, os.path.basename(p.filename))
                    with open(fp, "wb") as f:
                        f.write(p.data)
                    paths.append(fp)
            try:
                names = await run_in_threadpool(client.upload_documents, paths)
            except Exception as e:
                return JSONResponse(status_code=500, content={"message": str(e)})
        return {"uploaded": names}

    @app.get("/speech")
    async def speech_page():
        return FileResponse(STATIC / "speech.html")

    @app.get("/api/speech/status")
    async def speech_status():
        ok = speech.available()
        return {"asr": ok, "tts": ok, "message": "" if ok else
                "Speech is unavailable: set RIVA_API_URI to a Riva server with ASR / TTS enabled."}

    @app.post("/api/speech/asr")
    async def speech_asr(req: Request):
        if not speech.available():
            return JSONResponse(status_code=503, content={"message": "no ASR service configured"})
        lang = req.query_params.get("language", "en-US")
        pcm = wav_to_pcm16(await req.body(), 16000)

        def run():
            last = ""
            for last in speech.transcribe(pcm_chunks(pcm, 16000), lang, 16000):
                pass
            return last

        try:
            return {"transcript": await run_in_threadpool(run)}
        except Exception as e:
            return JSONResponse(status_code=502, content={"message": f"ASR failed: {e}"})

    @app.post("/api/speech/tts")
    async def speech_tts(req: Request):
        if not speech.available():
            return JSONResponse(status_code=503, content={"message": "no TTS service configured"})
        body = await req.json()
        text = (body.get("text") or "").strip()
        if not text:
            return JSONResponse(status_code=400, content={"message": "no text to synthesize"})

        def run():
            return b"".join(speech.synthesize(text, body.get("language", "en-US"), body.get("voice", "")))

        try:
            pcm = await run_in_threadpool(run)
        except Exception as e:
            return JSONResponse(status_code=502, content={"message": f"TTS failed: {e}"})
        from fastapi.responses import Response

        return Response(pcm_to_wav(pcm, speech.sample_rate_tts), media_type="audio/wav")

    from .prompt_designer import PromptConfigStore, PromptDesigner, add_routes

    designer = designer if designer is not None else PromptDesigner(
        PromptConfigStore(os.environ.get("PROMPT_DESIGN_CONFIG")))
    app.state.designer = designer
    add_routes(app, designer)

    @app.get("/health")
    async def health():
        return {"message": "Service is up.", "chain_server": await run_in_threadpool(client.health)}

    return app
