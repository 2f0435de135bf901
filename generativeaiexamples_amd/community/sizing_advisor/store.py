"""Named document collections + background ingestion tasks for the RAG-Blueprint-2.x style servers (reference:
/root/reference/community/vgpu-sizing-advisor/src/ingestor_server/server.py:88-701 - collections created / listed /
deleted in Milvus, files uploaded per collection, split with ``split_options``, ingested blocking or as a background
task polled through ``/status``).

Each collection is a chain-server ``VectorStore`` (one HBM index, optionally persisted under ``persist_dir``) embedded
by the shared embedder, so every collection's search is the same on-GPU exact scan. Uploaded files are kept under
``upload_dir/<collection>/`` so citations can be downloaded.
"""
from __future__ import annotations

import os
import re
import shutil
import threading
import uuid
from concurrent.futures import Future, ThreadPoolExecutor
from typing import Callable, Dict, List, Optional, Tuple

from ...index.hbm_index import Document
from ...rag.text_splitter import RecursiveCharacterTextSplitter

UNSUPPORTED = (".rst", ".rtf", ".org")
_NAME = re.compile(r"^[A-Za-z_][A-Za-z0-9_]{0,254}$")  # Milvus' collection-name rule, kept for client parity


class CollectionManager:
    def __init__(self, embeddings, upload_dir: str, persist_dir: Optional[str] = None, device=None,
                 hybrid: bool = False, store_factory: Optional[Callable[[str], object]] = None):
        from ...chain_server.vectorstore import VectorStore

        self.emb, self.upload_dir, self.persist_dir = embeddings, upload_dir, persist_dir
        self.factory = store_factory or (lambda name: VectorStore(name, embeddings, device=device,
                                                                  persist_dir=persist_dir, hybrid=hybrid))
        self.stores: Dict[str, object] = {}
        self.lock = threading.RLock()
        if persist_dir and os.path.isdir(persist_dir):  # reopen persisted collections
            for name in sorted(os.listdir(persist_dir)):
                if os.path.exists(os.path.join(persist_dir, name, "index.json")):
                    self.stores[name] = self.factory(name)

    # ---- collections
    def create(self, names: List[str]) -> dict:
        ok, failed = [], []
        with self.lock:
            for n in names:
                if not n or not _NAME.match(n):
                    failed.append({"collection_name": n or "", "error_message": "invalid collection name"})
                elif n in self.stores:
                    ok.append(n)  # creating an existing collection is a no-op, as in the reference
                else:
                    self.stores[n] = self.factory(n)
                    ok.append(n)
        return {"message": "Collection creation process completed.", "successful": ok, "failed": failed,
                "total_success": len(ok), "total_failed": len(failed)}

    def delete(self, names: List[str]) -> dict:
        ok, failed = [], []
        with self.lock:
            for n in names:
                if n not in self.stores:
                    failed.append({"collection_name": n, "error_message": f"collection {n} not found"})
                    continue
                self.stores.pop(n)
                for d in (os.path.join(self.persist_dir, n) if self.persist_dir else None,
                          os.path.join(self.upload_dir, n)):
                    if d and os.path.isdir(d):
                        shutil.rmtree(d, ignore_errors=True)
                ok.append(n)
        return {"message": "Collection deletion process completed.", "successful": ok, "failed": failed,
                "total_success": len(ok), "total_failed": len(failed)}

    def list(self) -> dict:
        with self.lock:
            cols = [{"collection_name": n, "num_entities": len(s)} for n, s in sorted(self.stores.items())]
        return {"message": "Successfully obtained collections", "total_collections": len(cols), "collections": cols}

    def get(self, name: str, create: bool = False):
        with self.lock:
            if name not in self.stores:
                if not create:
                    raise KeyError(f"collection {name} does not exist")
                if not _NAME.match(name or ""):
                    raise ValueError(f"invalid collection name {name!r}")
                self.create([name])
            return self.stores[name]

    # ---- documents
    def documents(self, name: str) -> dict:
        names = sorted(self.get(name).filenames()) if name in self.stores else []
        return {"message": "Document listing successfully completed.", "total_documents": len(names),
                "documents": [{"document_name": n} for n in names]}

    def delete_documents(self, name: str, document_names: List[str]) -> dict:
        store = self.get(name)
        gone = [n for n in document_names if store.delete_filename(n)]
        for n in gone:
            p = os.path.join(self.upload_dir, name, os.path.basename(n))
            if os.path.exists(p):
                os.remove(p)
        return {"message": "Files deleted successfully" if gone else "No matching documents found",
                "total_documents": len(gone), "documents": [{"document_name": n} for n in gone]}

    def save_upload(self, name: str, filename: str, data: bytes) -> str:
        if not _NAME.match(name or ""):  # the name becomes a directory: never a path
            raise ValueError(f"invalid collection name {name!r}")
        d = os.path.join(self.upload_dir, name)
        os.makedirs(d, exist_ok=True)
        p = os.path.join(d, os.path.basename(filename))
        with open(p, "wb") as f:
            f.write(data)
        return p

    def ingest(self, name: str, paths: List[str], chunk_size: int = 512, chunk_overlap: int = 150,
               replace: bool = False) -> dict:
        """Load + split + embed each file into collection ``name``; per-file failures are reported, not raised."""
        from ...rag.loaders import load

        store = self.get(name, create=True)
        splitter = RecursiveCharacterTextSplitter(chunk_size, chunk_overlap)
        existing = set(store.filenames())
        done, failed = [], []
        for p in paths:
            fn = os.path.basename(p)
            try:
                if fn.lower().endswith(UNSUPPORTED):
                    raise ValueError(f"File format for {fn} is not supported.")
                if fn in existing:
                    if not replace:
                        raise ValueError(f"Document {fn} already exists. Use PATCH /documents to replace it.")
                    store.delete_filename(fn)
                docs = [Document(d.page_content, dict(d.metadata, filename=fn)) for d in load(p, fn)]
                chunks = [c for c in splitter.split_documents(docs) if c.page_content.strip()]
                if not chunks:
                    raise ValueError(f"No text could be extracted from {fn}.")
                store.add_documents(chunks)
                done.append({"document_name": fn})
            except Exception as e:  # noqa: BLE001
                failed.append({"document_name": fn, "error_message": str(e)})
        return {"message": "Document upload job successfully completed.", "total_documents": len(paths),
                "documents": done, "failed_documents": failed}

    def search(self, name: str, query: str, k: int) -> List[Tuple[Document, float]]:
        store = self.get(name)
        return store.similarity_search_with_relevance_scores(query, k) if len(store) else []


class TaskHandler:
    """Background ingestion tasks: PENDING -> FINISHED (result) | FAILED (message)."""

    def __init__(self, workers: int = 2):
        self.pool = ThreadPoolExecutor(max_workers=workers)
        self.tasks: Dict[str, Future] = {}

    MAX_TASKS = 4096  # finished tasks kept for /status; the oldest finished ones are forgotten first

    def submit(self, fn: Callable[[], dict]) -> str:
        tid = str(uuid.uuid4())
        if len(self.tasks) >= self.MAX_TASKS:
            for old in [t for t, f in self.tasks.items() if f.done()][: len(self.tasks) - self.MAX_TASKS + 1]:
                self.tasks.pop(old, None)
        self.tasks[tid] = self.pool.submit(fn)
        return tid

    def status(self, tid: str) -> dict:
        f = self.tasks.get(tid)
        if f is None:
            return {"state": "UNKNOWN", "result": {"message": "Task not found"}}
        if not f.done():
            return {"state": "PENDING", "result": {}}
        if f.exception() is not None:
            return {"state": "FAILED", "result": {"message": str(f.exception())}}
        return {"state": "FINISHED", "result": f.result()}
