"""Ingestor server of the RAG-Blueprint-2.x API (reference: /root/reference/community/vgpu-sizing-advisor/src/
ingestor_server/server.py:204-701):

  GET    /health
  POST   /documents     multipart ``documents`` files + form field ``data`` = {"collection_name", "blocking",
                        "split_options": {"chunk_size", "chunk_overlap"}} -> upload result, or {"task_id"} when
                        ``blocking`` is false
  GET    /status        ?task_id= -> {"state": PENDING | FINISHED | FAILED | UNKNOWN, "result"}
  PATCH  /documents     same body as POST; existing documents of the same names are replaced
  GET    /documents     ?collection_name= -> document names
  DELETE /documents     ?collection_name=&document_names=a&document_names=b
  GET    /collections   names + entity counts
  POST   /collections   ?collection_names=a&collection_names=b (JSON list body also accepted)
  DELETE /collections   ?collection_names=...
"""
from __future__ import annotations

import json
import os
from typing import List, Optional

from fastapi import FastAPI, HTTPException, Query, Request
from fastapi.responses import JSONResponse
from pydantic import BaseModel, Field
from starlette.concurrency import run_in_threadpool

from ...chain_server.multipart import parse_multipart
from .store import _NAME, CollectionManager, TaskHandler

DEFAULT_COLLECTION = os.environ.get("COLLECTION_NAME", "multimodal_data")


class SplitOptions(BaseModel):
    chunk_size: int = Field(512, ge=16, le=65536)
    chunk_overlap: int = Field(150, ge=0, le=16384)


class DocumentUploadRequest(BaseModel):
    collection_name: str = DEFAULT_COLLECTION
    blocking: bool = False
    split_options: SplitOptions = Field(default_factory=SplitOptions)


def _parse(data: str) -> DocumentUploadRequest:
    try:
        return DocumentUploadRequest(**json.loads(data or "{}"))
    except json.JSONDecodeError as e:
        raise HTTPException(400, "Invalid JSON format") from e
    except Exception as e:  # noqa: BLE001 - pydantic validation
        raise HTTPException(422, str(e)) from e


async def _names(request: Request, names: Optional[List[str]]) -> List[str]:
    if names:
        return names
    try:
        body = await request.json()
    except Exception:  # noqa: BLE001 - no / non-JSON body
        body = None
    if isinstance(body, list):
        return [str(x) for x in body]
    return [DEFAULT_COLLECTION]


def create_ingestor_app(manager: CollectionManager, tasks: Optional[TaskHandler] = None) -> FastAPI:
    tasks = tasks or TaskHandler()
    app = FastAPI(title="Ingestor server")

    @app.get("/health")
    async def health():
        return {"message": "Ingestion Service is up."}

    async def _upload(request: Request, replace: bool):
        # multipart body parsed by chain_server/multipart.py (python-multipart, which FastAPI's File() needs, is not
        # in this image): ``documents`` file parts + a ``data`` JSON form field, as the reference's clients send
        try:
            parts = parse_multipart(request.headers.get("content-type", ""), await request.body())
        except ValueError as e:
            raise HTTPException(400, str(e)) from e
        data = next((p.data.decode("utf-8", "replace") for p in parts if p.name == "data" and p.filename is None),
                    "{}")
        req = _parse(data)
        if not _NAME.match(req.collection_name or ""):
            raise HTTPException(400, f"invalid collection name {req.collection_name!r}")
        files = [p for p in parts if p.name == "documents"]
        if not files:
            raise HTTPException(400, "No files provided for uploading.")
        paths = []
        for f in files:
            name = os.path.basename(f.filename or "")
            if not name:
                raise HTTPException(400, "Error parsing uploaded filename.")
            paths.append(manager.save_upload(req.collection_name, name, f.data))

        def job():
            return manager.ingest(req.collection_name, paths, req.split_options.chunk_size,
                                  req.split_options.chunk_overlap, replace=replace)

        if not req.blocking:
            return {"message": "Ingestion started in background", "task_id": tasks.submit(job)}
        return await run_in_threadpool(job)

    @app.post("/documents")
    async def upload(request: Request):
        return await _upload(request, replace=False)

    @app.patch("/documents")
    async def replace(request: Request):
        return await _upload(request, replace=True)

    @app.get("/status")
    async def status(task_id: str):
        return tasks.status(task_id)

    @app.get("/documents")
    async def list_documents(collection_name: str = DEFAULT_COLLECTION):
        return manager.documents(collection_name)

    @app.delete("/documents")
    async def delete_documents(collection_name: str = DEFAULT_COLLECTION,
                               document_names: List[str] = Query(default=[])):
        try:
            return await run_in_threadpool(manager.delete_documents, collection_name, document_names)
        except KeyError as e:
            return JSONResponse({"message": str(e.args[0])}, status_code=404)

    @app.get("/collections")
    async def list_collections():
        return manager.list()

    @app.post("/collections")
    async def create_collections(request: Request, collection_names: Optional[List[str]] = Query(default=None),
                                 collection_type: str = "text", embedding_dimension: int = 2048):
        # the index dimension follows the served embedder; the requested dimension is accepted for API parity
        return manager.create(await _names(request, collection_names))

    @app.delete("/collections")
    async def delete_collections(request: Request, collection_names: Optional[List[str]] = Query(default=None)):
        return manager.delete(await _names(request, collection_names))

    app.state.manager, app.state.tasks = manager, tasks
    return app
