"""Client of the chain-server REST API (the role of RAG/src/rag_playground/default/chat_client.py:29-177).

Used by the playground pages, the evaluation tool and the load generator. ``predict`` streams
``POST /generate`` and parses the SSE frames (``data: `` prefix, 6 characters) into text chunks.
"""
from __future__ import annotations

import json
import logging
import os
from typing import Dict, Iterator, List, Optional

import httpx

from ..chain_server import tracing

log = logging.getLogger(__name__)


class ChatClient:
    def __init__(self, server_url: str, model_name: str = "", timeout: float = 600.0,
                 http: Optional[httpx.Client] = None):
        if not server_url.startswith("http"):
            server_url = "http://" + server_url
        self.server_url = server_url.rstrip("/")
        self.model_name = model_name
        self.timeout = timeout
        # any httpx.Client works (tests pass a starlette TestClient bound to the chain-server app)
        self.http = http or httpx.Client(timeout=timeout)

    # ------------------------------------------------------------------ search / generate
    def search(self, prompt: str, top_k: int = 4) -> List[Dict]:
        r = self.http.post(f"{self.server_url}/search", json={"query": prompt, "top_k": top_k},
                       headers=tracing.inject({"accept": "application/json"}))
        r.raise_for_status()
        return r.json().get("chunks", [])

    def predict(self, query: str, use_knowledge_base: bool, num_tokens: int = 1024, history=None,
                temperature: float = 0.2, top_p: float = 0.7, stop: Optional[List[str]] = None) -> Iterator[str]:
        messages = list(history or []) + [{"role": "user", "content": query}]
        body = {"messages": messages, "use_knowledge_base": use_knowledge_base, "temperature": temperature,
                "top_p": top_p, "max_tokens": num_tokens, "stop": stop or []}
        with self.http.stream("POST", f"{self.server_url}/generate", json=body, headers=tracing.inject({})) as r:
            if r.status_code != 200 and r.status_code != 500:
                r.raise_for_status()
            for line in r.iter_lines():
                if not line.startswith("data: "):
                    continue
                frame = json.loads(line[6:])
                ch = frame["choices"][0]
                if ch.get("finish_reason") == "[DONE]":
                    content = ch["message"]["content"]
                    if content:
                        yield content
                    break
                yield ch["message"]["content"]

    # ------------------------------------------------------------------ documents
    def upload_documents(self, file_paths: List[str]) -> List[str]:
        done = []
        for p in file_paths:
            with open(p, "rb") as f:
                r = self.http.post(f"{self.server_url}/documents", files={"file": (os.path.basename(p), f)},
                               headers=tracing.inject({}))
            if r.status_code != 200:
                raise RuntimeError(f"upload of {p} failed: {r.status_code} {r.text}")
            done.append(os.path.basename(p))
        return done

    def delete_documents(self, filename: str) -> str:
        r = self.http.delete(f"{self.server_url}/documents", params={"filename": filename})
        r.raise_for_status()
        return r.json().get("message", "")

    def get_uploaded_documents(self) -> List[str]:
        r = self.http.get(f"{self.server_url}/documents")
        r.raise_for_status()
        return r.json().get("documents", [])

    def health(self) -> bool:
        try:
            return self.http.get(f"{self.server_url}/health", timeout=10).status_code == 200
        except httpx.HTTPError:
            return False
