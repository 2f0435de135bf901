"""Chain-server REST API (contract of RAG/src/chain_server/server.py:249-491 and
docs/api_reference/openapi_schema.json): /health, /documents (POST multipart, GET, DELETE),
/generate (SSE), /search.

Behaviour kept byte-compatible: request schemas and ranges (422 on violation, ``detail`` list
without the offending ``input``), HTML sanitisation of every text field, the last ``user``
message becomes the query and the rest the history, SSE frames ``data: <ChainResponse>\\n\\n``
with a terminal ``finish_reason: "[DONE]"`` frame, errors as a 500 SSE frame, CORS ``*``.

Internals fixed: ingest, retrieval and generation run in worker threads,
never on the event loop; the example is instantiated once; uploads use a per-request temp name.
"""
from __future__ import annotations

import importlib.util
import inspect
import logging
import os
import shutil
import tempfile
import uuid
from typing import Any, Dict, List

from fastapi import FastAPI, Query, Request
from fastapi.encoders import jsonable_encoder
from fastapi.exceptions import RequestValidationError
from fastapi.middleware.cors import CORSMiddleware
from fastapi.responses import JSONResponse, StreamingResponse
from pydantic import BaseModel, Field, constr, field_validator
from starlette.concurrency import iterate_in_threadpool, run_in_threadpool

from . import tracing
from .multipart import parse_multipart
from .sanitize import clean

logging.basicConfig(level=os.environ.get("LOGLEVEL", "INFO").upper())
log = logging.getLogger(__name__)

_REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
EXAMPLE_DIR = os.environ.get("EXAMPLE_DIR") or (
    "RAG/examples/" if os.path.isdir("RAG/examples") else os.path.join(_REPO, "RAG", "examples"))
UPLOAD_DIR = os.environ.get("UPLOAD_DIR", "/tmp-data/uploaded_files")

# FastAPI's default title / version, as the reference's ``FastAPI()`` (docs/api_reference/openapi_schema.json "info")
app = FastAPI()
app.add_middleware(CORSMiddleware, allow_origins=["*"], allow_credentials=False, allow_methods=["*"],
                   allow_headers=["*"])


# ------------------------------------------------------------------------------------ schemas
class Message(BaseModel):
    """Definition of the Chat Message type."""

    role: str = Field(description="Role for a message AI, User and System", default="user", max_length=256,
                      pattern=r"[\s\S]*")
    content: str = Field(description="The input query/prompt to the pipeline.",
                         default="I am going to Paris, what should I see?", max_length=131072, pattern=r"[\s\S]*")

    @field_validator("role")
    @classmethod
    def _role(cls, v):
        v = clean(v)
        if v.lower() not in ("user", "assistant", "system"):
            raise ValueError("Role must be one of 'user', 'assistant', or 'system'")
        return v.lower()

    @field_validator("content")
    @classmethod
    def _content(cls, v):
        return clean(v)


class Prompt(BaseModel):
    """Definition of the Prompt API data type."""

    messages: List[Message] = Field(
        ..., max_length=50000,
        description="A list of messages comprising the conversation so far. The roles of the messages must be "
                    "alternating between user and assistant. The last input message should have role user. A message "
                    "with the the system role is optional, and must be the very first message if it is present.")
    use_knowledge_base: bool = Field(..., description="Whether to use a knowledge base")
    temperature: float = Field(
        0.2, ge=0.1, le=1.0,
        description="The sampling temperature to use for text generation. The higher the temperature value is, the "
                    "less deterministic the output text will be. It is not recommended to modify both temperature and "
                    "top_p in the same call.")
    top_p: float = Field(
        0.7, ge=0.1, le=1.0,
        description="The top-p sampling mass used for text generation. The top-p value determines the probability "
                    "mass that is sampled at sampling time. For example, if top_p = 0.2, only the most likely tokens "
                    "(summing to 0.2 cumulative probability) will be sampled. It is not recommended to modify both "
                    "temperature and top_p in the same call.")
    max_tokens: int = Field(
        1024, ge=0, le=1024, json_schema_extra={"format": "int64"},
        description="The maximum number of tokens to generate in any given call. Note that the model is not aware of "
                    "this value, and generation will simply stop at the number of tokens specified.")
    stop: List[constr(max_length=256, pattern=r"[\s\S]*")] = Field(
        max_length=256, default=[],
        description="A string or a list of strings where the API will stop generating further tokens. The returned "
                    "text will not contain the stop sequence.")

    @field_validator("use_knowledge_base", mode="before")
    @classmethod
    def _kb(cls, v):
        s = clean(str(v))
        m = {"True": True, "False": False, "true": True, "false": False}
        if s not in m:
            raise ValueError("use_knowledge_base must be a boolean value")
        return m[s]

    @field_validator("temperature", "top_p", mode="before")
    @classmethod
    def _num(cls, v):
        return float(clean(str(v)))


class ChainResponseChoices(BaseModel):
    """Definition of Chain response choices"""

    index: int = Field(default=0, ge=0, le=256, json_schema_extra={"format": "int64"})
    message: Message = Field(default=Message(role="assistant", content=""))
    finish_reason: str = Field(default="", max_length=4096, pattern=r"[\s\S]*")


class ChainResponse(BaseModel):
    """Definition of Chain APIs resopnse data type"""

    id: str = Field(default="", max_length=100000, pattern=r"[\s\S]*")
    choices: List[ChainResponseChoices] = Field(default=[], max_length=256)


class DocumentSearch(BaseModel):
    """Definition of the DocumentSearch API data type."""

    query: str = Field(description="The content or keywords to search for within documents.", max_length=131072,
                       pattern=r"[\s\S]*", default="")
    top_k: int = Field(description="The maximum number of documents to return in the response.", default=4, ge=0,
                       le=25, json_schema_extra={"format": "int64"})


class DocumentChunk(BaseModel):
    """Represents a chunk of a document."""

    content: str = Field(description="The content of the document chunk.", max_length=131072, pattern=r"[\s\S]*",
                         default="")
    filename: str = Field(description="The name of the file the chunk belongs to.", max_length=4096,
                          pattern=r"[\s\S]*", default="")
    score: float = Field(..., description="The relevance score of the chunk.")


class DocumentSearchResponse(BaseModel):
    """Represents a response from a document search."""

    chunks: List[DocumentChunk] = Field(..., description="List of document chunks.", max_length=256)


class DocumentsResponse(BaseModel):
    """Represents the response containing a list of documents."""

    documents: List[constr(max_length=131072, pattern=r"[\s\S]*")] = Field(
        description="List of filenames.", max_length=1000000, default=[])


class HealthResponse(BaseModel):
    message: str = Field(max_length=4096, pattern=r"[\s\S]*", default="")


# ------------------------------------------------------------------------------------ example loading
def _has_contract(cls) -> bool:
    return all(hasattr(cls, m) for m in ("ingest_docs", "llm_chain", "rag_chain"))


def load_example(example_path: str | None = None):
    """Import every .py under RAG/examples/$EXAMPLE_PATH; instantiate the first class implementing the
    BaseExample contract (skipping BaseExample itself)."""
    root = os.path.join(EXAMPLE_DIR, example_path or os.environ.get("EXAMPLE_PATH", "basic_rag/langchain"))
    for dirpath, _dirs, files in os.walk(root):
        for fn in sorted(files):
            if not fn.endswith(".py"):
                continue
            spec = importlib.util.spec_from_file_location(f"gai_example_{uuid.uuid4().hex[:8]}",
                                                          os.path.join(dirpath, fn))
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)  # type: ignore[union-attr]
            for name, cls in inspect.getmembers(mod, inspect.isclass):
                if name == "BaseExample" or inspect.isabstract(cls) or not _has_contract(cls):
                    continue
                try:
                    return cls()
                except Exception as e:
                    raise ValueError(f"Class {name} is not implemented and could not be instantiated.") from e
    raise NotImplementedError(f"Could not find a valid example class in {root}")


def example():
    ex = getattr(app.state, "example", None)
    if ex is None:
        ex = app.state.example = load_example()
    return ex


@app.on_event("startup")
def _startup() -> None:
    if os.environ.get("GAI_LAZY_EXAMPLE", "0") != "1":
        example()


@app.on_event("startup")
async def _worker_threads() -> None:
    # every streaming /generate holds a worker thread while it waits for its next token, and retrieval / prompt
    # building run in worker threads too: with anyio's default of 40, a 64-request burst would queue behind the streams
    # already running (benchmarks/served.py measured with 256)
    import anyio

    anyio.to_thread.current_default_thread_limiter().total_tokens = int(os.environ.get("GAI_SERVER_THREADS", "256"))


@app.exception_handler(RequestValidationError)
async def _validation(request: Request, exc: RequestValidationError) -> JSONResponse:
    return JSONResponse(status_code=422, content={"detail": jsonable_encoder(exc.errors(), exclude={"input", "ctx"})})


# ------------------------------------------------------------------------------------ routes
# every route documents its 500 like the reference (server.py:248-257 and the other decorators)
_ERR500 = {500: {"description": "Internal Server Error",
                 "content": {"application/json": {"example": {"detail": "Internal server error occurred"}}}}}
_VALIDATION_ERROR = {"description": "Validation Error",
                     "content": {"application/json": {"schema": {"$ref": "#/components/schemas/HTTPValidationError"}}}}
# POST /documents takes ``file: UploadFile = File(...)`` in the reference (server.py:280). python-multipart is not
# importable here, so the body is parsed by chain_server/multipart.py and the multipart requestBody that FastAPI
# would derive from File(...) is declared explicitly (schema added to components in _openapi below).
_UPLOAD_BODY_SCHEMA = {"properties": {"file": {"type": "string", "format": "binary", "title": "File"}},
                       "type": "object", "required": ["file"], "title": "Body_upload_document_documents_post"}
_UPLOAD_OPENAPI = {"requestBody": {"required": True, "content": {"multipart/form-data": {
    "schema": {"$ref": "#/components/schemas/Body_upload_document_documents_post"}}}}}


@app.get("/health", response_model=HealthResponse, responses=_ERR500)
async def health_check():
    """
    Perform a Health Check

    Returns 200 when service is up. This does not check the health of downstream services.
    """
    return HealthResponse(message="Service is up.")


def _missing_file() -> JSONResponse:
    """The 422 FastAPI gives a ``File(...)`` parameter whose part is absent (the reference's behaviour)."""
    return JSONResponse(status_code=422, content={"detail": [
        {"type": "missing", "loc": ["body", "file"], "msg": "Field required"}]})


@app.post("/documents", responses={422: _VALIDATION_ERROR, **_ERR500}, openapi_extra=_UPLOAD_OPENAPI)
@tracing.instrumentation_wrapper
async def upload_document(request: Request) -> JSONResponse:
    """Upload a document to the vector store."""
    ctype = request.headers.get("content-type", "")
    body = await request.body()
    try:
        parts = parse_multipart(ctype, body)
    except Exception:
        parts = []
    f = next((p for p in parts if p.name == "file"), None)
    if f is None:
        return _missing_file()
    if not f.filename:  # a file part without a name: the reference's 200 "No files provided" (server.py:283-284)
        return JSONResponse(content={"message": "No files provided"}, status_code=200)
    try:
        name = os.path.basename(f.filename)
        os.makedirs(UPLOAD_DIR, exist_ok=True)
        path = os.path.join(UPLOAD_DIR, name)
        tmp = tempfile.NamedTemporaryFile(dir=UPLOAD_DIR, delete=False)
        with tmp:
            tmp.write(f.data)
        shutil.move(tmp.name, path)
        await run_in_threadpool(example().ingest_docs, path, name)
        return JSONResponse(content={"message": "File uploaded successfully"}, status_code=200)
    except Exception as e:
        log.exception("ingest failed")
        return JSONResponse(content={"message": str(e)}, status_code=500)


def _frame(content: str, finish: str = "", rid: str | None = None) -> str:
    r = ChainResponse(id=rid or str(uuid.uuid4()),
                      choices=[ChainResponseChoices(index=0, message=Message(role="assistant", content=content),
                                                    finish_reason=finish)])
    return "data: " + r.model_dump_json() + "\n\n"


@app.post("/generate", response_model=ChainResponse, responses=_ERR500)
@tracing.instrumentation_wrapper
async def generate_answer(request: Request, prompt: Prompt) -> StreamingResponse:
    """Generate and stream the response to the provided prompt."""
    try:
        msgs = [m.model_dump() for m in prompt.messages]
        query, idx = None, None
        for i in range(len(msgs) - 1, -1, -1):
            if msgs[i]["role"] == "user":
                query, idx = msgs[i]["content"], i
                break
        history = [m for j, m in enumerate(msgs) if j != idx]
        settings = prompt.model_dump(exclude={"messages", "use_knowledge_base"})
        ex = example()
        if query is None:
            query = ""
        chain = ex.rag_chain if prompt.use_knowledge_base else ex.llm_chain
        # conversation state keyed by an explicit session (X-Session-Id header) for chains that keep memory
        sid = request.headers.get("x-session-id")
        if sid and "session_id" in inspect.signature(chain).parameters:
            settings["session_id"] = clean(sid)[:256]
        # retrieval + prompt building run in a worker thread (concurrent queries coalesce into one embed and
        # one index scan there); the token stream is then awaited on the event loop when the chain returns
        # an async-iterable stream (in-process engine), so no thread is held per open stream
        gen = await run_in_threadpool(chain, query, history, **settings)
        if hasattr(gen, "__aiter__"):
            chunks = tracing.traced_astream("llm_stream", gen)
        else:
            chunks = iterate_in_threadpool(tracing.traced_stream("llm_stream", iter(gen)))

        async def frames():
            rid = str(uuid.uuid4())
            try:
                async for chunk in chunks:
                    if chunk:
                        yield _frame(chunk, "", rid)
                yield _frame("", "[DONE]", rid)
            except Exception as e:  # mid-stream failure: report it as the last frame
                log.exception("generation failed")
                yield _frame(f"Error from chain server. Please check chain-server logs for more details. {e}",
                             "[DONE]", rid)

        return StreamingResponse(frames(), media_type="text/event-stream")
    except Exception as e:
        log.exception("generate failed")
        msg = str(e)
        if "vector" in msg.lower() and "store" in msg.lower():
            msg = "Error from vector store. Please check chain-server logs for more details."
        else:
            msg = f"Error from chain server. Please check chain-server logs for more details. {msg}"
        return StreamingResponse(iter([_frame(msg, "[DONE]")]), media_type="text/event-stream", status_code=500)


@app.post("/search", response_model=DocumentSearchResponse, responses=_ERR500)
@tracing.instrumentation_wrapper
async def document_search(request: Request, data: DocumentSearch) -> Dict[str, List[Dict[str, Any]]]:
    """Search for the most relevant documents for the given search parameters."""
    try:
        ex = example()
        if not hasattr(ex, "document_search"):
            raise NotImplementedError("Example class has not implemented the document_search method.")
        res = await run_in_threadpool(ex.document_search, data.query, data.top_k)
        chunks = [DocumentChunk(content=r.get("content", ""), filename=r.get("filename", ""),
                                score=float(r.get("score", 0.0))) for r in res]
        return DocumentSearchResponse(chunks=chunks)
    except Exception as e:
        log.exception("search failed")
        return JSONResponse(content={"message": f"Error occurred while searching documents. {e}"}, status_code=500)


@app.get("/documents", response_model=DocumentsResponse, responses=_ERR500)
@tracing.instrumentation_wrapper
async def get_documents(request: Request) -> DocumentsResponse:
    """List available documents."""
    try:
        docs = await run_in_threadpool(example().get_documents)
        return DocumentsResponse(documents=docs)
    except Exception as e:
        log.exception("list documents failed")
        return JSONResponse(content={"message": f"Error occurred while fetching documents: {e}"}, status_code=500)


@app.delete("/documents", responses=_ERR500)
@tracing.instrumentation_wrapper
async def delete_document(request: Request, filename: str = Query(...)) -> JSONResponse:
    """Delete a document."""
    try:
        ok = await run_in_threadpool(example().delete_documents, [filename])
        if not ok:
            raise Exception(f"Error in deleting document {filename}")
        return JSONResponse(content={"message": f"Document {filename} deleted successfully"}, status_code=200)
    except Exception as e:
        log.exception("delete failed")
        return JSONResponse(content={"message": f"Failed to delete document {filename}. {e}"}, status_code=500)


def _openapi() -> Dict[str, Any]:
    """FastAPI's schema plus the multipart body component of POST /documents (see _UPLOAD_OPENAPI)."""
    if app.openapi_schema is None:
        from fastapi.openapi.utils import get_openapi

        schema = get_openapi(title=app.title, version=app.version, openapi_version=app.openapi_version,
                             description=app.description, routes=app.routes)
        schema.setdefault("components", {}).setdefault("schemas", {})[
            "Body_upload_document_documents_post"] = _UPLOAD_BODY_SCHEMA
        app.openapi_schema = schema
    return app.openapi_schema


app.openapi = _openapi
