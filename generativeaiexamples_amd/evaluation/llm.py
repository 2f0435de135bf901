"""Minimal OpenAI-compatible chat client used by the generator / judge (any /v1 server: ours or remote)."""
from __future__ import annotations

import os
from typing import Callable, List, Optional

import httpx


class ChatFn:
    """callable(messages) -> str over POST {base_url}/v1/chat/completions (non-streaming)."""

    def __init__(self, base_url: str, model: str, temperature: float = 0.1, max_tokens: int = 512, top_p: float = 1.0,
                 api_key: Optional[str] = None, http: Optional[httpx.Client] = None, timeout: float = 600.0):
        if not base_url.startswith("http"):
            base_url = "http://" + base_url
        self.url = base_url.rstrip("/") + ("" if base_url.rstrip("/").endswith("/v1") else "/v1") + "/chat/completions"
        self.model, self.kw = model, dict(temperature=temperature, max_tokens=max_tokens, top_p=top_p)
        key = api_key or os.environ.get("NVIDIA_API_KEY")
        self.headers = {"Authorization": f"Bearer {key}"} if key else {}
        self.http = http or httpx.Client(timeout=timeout)

    def __call__(self, messages: List[dict], schema: Optional[dict] = None) -> str:
        """``schema``: JSON schema the reply must follow (``response_format: json_schema``; the model server
        enforces it with constrained decoding)."""
        body = dict(model=self.model, messages=messages, stream=False, **self.kw)
        if schema is not None:
            body["response_format"] = {"type": "json_schema", "json_schema": {"name": "reply", "schema": schema}}
        r = self.http.post(self.url, json=body, headers=self.headers)
        r.raise_for_status()
        return r.json()["choices"][0]["message"]["content"] or ""


LLMFn = Callable[[List[dict]], str]
