"""Prompt designer (reference: /root/reference/community/llm-prompt-design-helper - chat_ui.py:91-322 and
chat_ui_utils.py: per-model system prompt, few-shot examples and sampling settings kept in a YAML file with a
``default`` entry, edited in the UI and written back; generation against OpenAI-compatible endpoints; optional
retrieval context from a local FAISS store of uploaded files / URLs).

``PromptConfigStore`` reads / writes that YAML shape (``yaml.safe_load`` / ``safe_dump``; a model without an entry
inherits ``default``). ``PromptDesigner`` builds the message list (system prompt + retrieved context, few-shot turns,
history, input), streams one model's answer, and compares several models on the same input concurrently (against the
in-process server they share decode batches). Context comes from a chain-server VectorStore of pasted / uploaded text.
"""
from __future__ import annotations

import os
import threading
from concurrent.futures import ThreadPoolExecutor
from typing import Callable, Dict, Iterator, List, Optional

import yaml
from fastapi import Request  # module level: the route annotations below are resolved against these globals

DEFAULT_SETTINGS = {"system_prompt": "You are an assistant to help answer the user's question. Answer politely and "
                                     "accurately.",
                    "few_shot_examples": [], "temperature": 0.0, "top_p": 0.7, "max_tokens": 1024, "seed": 42}
_KEYS = tuple(DEFAULT_SETTINGS) + ("base_url",)


class PromptConfigStore:
    def __init__(self, path: Optional[str] = None):
        self.path, self.lock = path, threading.Lock()
        self.data: Dict[str, dict] = {"default": dict(DEFAULT_SETTINGS)}
        if path and os.path.exists(path):
            with open(path) as f:
                loaded = yaml.safe_load(f) or {}
            if not isinstance(loaded, dict):
                raise ValueError(f"{path}: expected a mapping of model name -> settings")
            for name, s in loaded.items():
                self.data[str(name)] = {k: v for k, v in (s or {}).items() if k in _KEYS}
            self.data.setdefault("default", dict(DEFAULT_SETTINGS))

    def get(self, model: str) -> dict:
        with self.lock:
            out = dict(DEFAULT_SETTINGS)
            out.update({k: v for k, v in self.data.get("default", {}).items() if v is not None})
            out.update({k: v for k, v in self.data.get(model, {}).items() if v is not None})
        out["few_shot_examples"] = [e for e in (out.get("few_shot_examples") or [])
                                    if isinstance(e, dict) and e.get("role") in ("user", "assistant")
                                    and isinstance(e.get("content"), str)]
        return out

    def update(self, model: str, settings: dict, save: bool = True) -> dict:
        bad = set(settings) - set(_KEYS)
        if bad:
            raise ValueError(f"unknown settings {sorted(bad)}")
        with self.lock:
            self.data.setdefault(model, {}).update(settings)
        if save and self.path:
            self.save()
        return self.get(model)

    def models(self) -> List[str]:
        return [m for m in self.data if m != "default"]

    def save(self, path: Optional[str] = None) -> None:
        with self.lock, open(path or self.path, "w") as f:
            yaml.safe_dump(self.data, f, sort_keys=False, allow_unicode=True)


def build_messages(settings: dict, user_input: str, context: Optional[List[str]] = None,
                   history: Optional[List[dict]] = None) -> List[dict]:
    system = settings.get("system_prompt") or ""
    if context:
        system += "\n\nUse the following context when it is relevant:\n" + "\n\n".join(context)
    msgs = [{"role": "system", "content": system}] if system else []
    msgs += [{"role": e["role"], "content": e["content"]} for e in settings.get("few_shot_examples") or []]
    msgs += [m for m in history or [] if m.get("role") in ("user", "assistant")]
    return msgs + [{"role": "user", "content": user_input}]


class PromptDesigner:
    def __init__(self, store: PromptConfigStore, llm_for: Optional[Callable[[str, dict], object]] = None,
                 context_store=None):
        self.store, self.context_store = store, context_store
        self.llm_for = llm_for or self._remote

    @staticmethod
    def _remote(model: str, settings: dict):
        from ..chain_server.connectors import RemoteChatLLM

        base = settings.get("base_url") or os.environ.get("APP_LLM_SERVERURL", "http://localhost:8000")
        return RemoteChatLLM(base, model)

    def context(self, query: str, k: int = 4) -> List[str]:
        if self.context_store is None or len(self.context_store) == 0:
            return []
        return [d.page_content for d, _ in self.context_store.similarity_search_with_relevance_scores(query, k)]

    def add_context(self, texts: List[str], source: str = "pasted") -> int:
        from ..index.hbm_index import Document
        from ..rag.text_splitter import RecursiveCharacterTextSplitter

        if self.context_store is None:
            raise RuntimeError("no context store configured")
        sp = RecursiveCharacterTextSplitter(1000, 100)
        chunks = [c for t in texts for c in sp.split_text(t) if c.strip()]
        if chunks:
            self.context_store.add_documents([Document(c, {"filename": source}) for c in chunks])
        return len(chunks)

    def stream(self, model: str, user_input: str, use_context: bool = False, history=None, k: int = 4
               ) -> Iterator[str]:
        s = self.store.get(model)
        msgs = build_messages(s, user_input, self.context(user_input, k) if use_context else None, history)
        llm = self.llm_for(model, s)
        yield from llm.stream(msgs, temperature=s["temperature"], top_p=s["top_p"], max_tokens=s["max_tokens"],
                              seed=s.get("seed"))

    def compare(self, models: List[str], user_input: str, use_context: bool = False) -> Dict[str, str]:
        with ThreadPoolExecutor(max_workers=max(1, min(8, len(models)))) as ex:  # request-sized list: bounded
            futs = {m: ex.submit(lambda m=m: "".join(self.stream(m, user_input, use_context))) for m in models}
            out = {}
            for m, f in futs.items():
                try:
                    out[m] = f.result()
                except Exception as e:  # noqa: BLE001 - one unreachable model does not fail the comparison
                    out[m] = f"[error: {e}]"
            return out


def add_routes(app, designer: PromptDesigner) -> None:
    """``/prompt-design`` page and its ``/api/prompt/*`` routes on the playground app."""
    from fastapi.responses import FileResponse, JSONResponse, StreamingResponse
    from starlette.concurrency import iterate_in_threadpool, run_in_threadpool

    from .app import STATIC

    @app.get("/prompt-design")
    async def page():
        return FileResponse(STATIC / "prompt_design.html")

    @app.get("/api/prompt/config")
    async def get_config(model: str = "default"):
        return {"model": model, "settings": designer.store.get(model), "models": designer.store.models()}

    @app.put("/api/prompt/config")
    async def put_config(req: Request):
        body = await req.json()
        try:
            s = await run_in_threadpool(designer.store.update, body.get("model", "default"), body.get("settings", {}))
        except ValueError as e:
            return JSONResponse(status_code=400, content={"message": str(e)})
        return {"model": body.get("model", "default"), "settings": s}

    @app.post("/api/prompt/generate")
    async def generate(req: Request):
        b = await req.json()
        it = designer.stream(b.get("model", "default"), b.get("input", ""), bool(b.get("use_context")),
                             b.get("history") or [])
        return StreamingResponse(iterate_in_threadpool(it), media_type="text/plain; charset=utf-8")

    @app.post("/api/prompt/compare")
    async def compare(req: Request):
        b = await req.json()
        return await run_in_threadpool(designer.compare, list(b.get("models") or []), b.get("input", ""),
                                       bool(b.get("use_context")))

    @app.post("/api/prompt/context")
    async def context(req: Request):
        b = await req.json()
        try:
            n = await run_in_threadpool(designer.add_context, [str(t) for t in b.get("texts") or []],
                                        b.get("source", "pasted"))
        except RuntimeError as e:
            return JSONResponse(status_code=400, content={"message": str(e)})
        return {"chunks": n}
