"""Model-service clients used by the example pipelines (the roles of ChatNVIDIA, NVIDIAEmbeddings and
NVIDIARerank in the reference, RAG/src/chain_server/utils.py:364-471).

Two transports behind one interface:
* in-process (``model_engine = mi355x``): calls the MI355X engines of this process's ServiceHub -
  no HTTP hop on the query path;
* remote (``nvidia-ai-endpoints`` / ``openai``): HTTP to any NIM/OpenAI-compatible ``/v1`` server
  (e.g. ``python -m generativeaiexamples_amd.serving`` on another node), SSE streaming.
"""
from __future__ import annotations

import json
import logging
import threading
from typing import Any, Dict, Iterator, List, Optional, Sequence

import httpx

from ..engine.sampling import SamplingParams
from ..engine.tokenizer import apply_chat_template
from ..index.hbm_index import Document

log = logging.getLogger(__name__)


def _base(url: str) -> str:
    url = url.rstrip("/")
    if not url.startswith("http"):
        url = "http://" + url
    return url if url.endswith("/v1") else url + "/v1"


# ------------------------------------------------------------------------------------------ LLM
from . import tracing  # noqa: E402


class ChatLLM:
    model: str = ""

    def __init__(self, temperature: float = 0.2, top_p: float = 0.7, max_tokens: int = 1024,
                 stop: Optional[Sequence[str]] = None, **extra):
        self.settings = dict(temperature=temperature, top_p=top_p, max_tokens=max_tokens, stop=list(stop or []))
        self.settings.update({k: v for k, v in extra.items() if v is not None})

    def stream(self, messages: List[Dict[str, Any]], **override) -> Iterator[str]:
        raise NotImplementedError

    def traced_stream(self, messages: List[Dict[str, Any]], **override) -> Iterator[str]:
        """stream() inside an 'llm' span with model, prompt size and first_token_time_ms (TTFT)."""
        n_prompt = sum(len(str(m.get("content") or "")) for m in messages)
        return tracing.traced_stream("llm.stream", self.stream(messages, **override),
                                     **{"llm.model": getattr(self, "model", ""), "llm.prompt_chars": n_prompt})

    def invoke(self, messages: List[Dict[str, Any]], **override) -> str:
        return "".join(self.stream(messages, **override))

    def _params(self, override) -> SamplingParams:
        s = dict(self.settings)
        s.update({k: v for k, v in override.items() if v is not None})
        return SamplingParams(temperature=float(s.get("temperature", 0.2)), top_p=float(s.get("top_p", 0.7)),
                              max_tokens=int(s.get("max_tokens", 1024)), stop=list(s.get("stop") or []),
                              seed=s.get("seed"), ignore_eos=bool(s.get("ignore_eos", False)))


class EngineStream:
    """Token-text stream of one in-process generation. Iterated synchronously (a worker thread blocks per
    chunk, e.g. an example that post-processes the stream) or asynchronously (``async for``: the
    chain-server SSE route awaits the engine's asyncio queue and holds no thread while waiting). The
    request is submitted to the engine when iteration starts."""

    def __init__(self, engine, ids: List[int], params: SamplingParams):
        self.engine, self.ids, self.params = engine, ids, params

    def __iter__(self) -> Iterator[str]:
        for it in self.engine.generate_sync(self.ids, self.params):
            if it.delta:
                yield it.delta

    async def _agen(self):
        async for it in self.engine.generate(self.ids, self.params):
            if it.delta:
                yield it.delta

    def __aiter__(self):
        return self._agen()


class LocalChatLLM(ChatLLM):
    def __init__(self, engine, model: str, **settings):
        super().__init__(**settings)
        self.engine, self.model = engine, model

    def stream(self, messages, **override) -> EngineStream:
        ids = apply_chat_template(messages, self.engine.tokenizer)
        return EngineStream(self.engine, ids, self._params(override))


class RemoteChatLLM(ChatLLM):
    def __init__(self, base_url: str, model: str, api_key: Optional[str] = None, timeout: float = 600.0, **settings):
        super().__init__(**settings)
        self.base, self.model = _base(base_url), model
        self.headers = {"Authorization": f"Bearer {api_key}"} if api_key else {}
        self.timeout = timeout

    def stream(self, messages, **override) -> Iterator[str]:
        p = self._params(override)
        body = {"model": self.model, "messages": messages, "temperature": p.temperature, "top_p": p.top_p,
                "max_tokens": p.max_tokens, "stream": True}
        if p.stop:
            body["stop"] = p.stop
        with httpx.stream("POST", f"{self.base}/chat/completions", json=body, headers=self.headers,
                          timeout=self.timeout) as r:
            r.raise_for_status()
            for line in r.iter_lines():
                if not line.startswith("data:"):
                    continue
                data = line[5:].strip()
                if data == "[DONE]":
                    break
                obj = json.loads(data)
                for ch in obj.get("choices", []):
                    d = ch.get("delta", {}).get("content")
                    if d:
                        yield d


# ------------------------------------------------------------------------------------------ embeddings
class Embeddings:
    dim: int = 0

    def embed_documents(self, texts: List[str]) -> List[List[float]]:
        raise NotImplementedError

    def embed_query(self, text: str) -> List[float]:
        raise NotImplementedError

    # tensor fast path (in-process): avoids host round trips when indexing into HBM
    def embed_tensor(self, texts: List[str], input_type: str):
        import torch

        fn = self.embed_documents if input_type == "passage" else (lambda t: [self.embed_query(x) for x in t])
        return torch.tensor(fn(texts), dtype=torch.float32)


class LocalEmbeddings(Embeddings):
    def __init__(self, embedder, truncate: str = "END"):
        self.e, self.truncate = embedder, truncate
        self.dim = embedder.dim

    def embed_tensor(self, texts, input_type):
        # concurrent callers (retrieval threads, ingest) coalesce into one encoder call (DynamicBatcher)
        if hasattr(self.e, "embed_coalesced"):
            return self.e.embed_coalesced(texts, input_type, self.truncate)
        return self.e.embed(texts, input_type, self.truncate)

    def embed_documents(self, texts):
        return self.embed_tensor(texts, "passage").float().cpu().tolist()

    def embed_query(self, text):
        return self.embed_tensor([text], "query").float().cpu()[0].tolist()


class RemoteEmbeddings(Embeddings):
    def __init__(self, base_url: str, model: str, truncate: str = "END", api_key: Optional[str] = None,
                 batch: int = 64, timeout: float = 600.0):
        self.base, self.model, self.truncate, self.batch = _base(base_url), model, truncate, batch
        self.headers = {"Authorization": f"Bearer {api_key}"} if api_key else {}
        self.timeout = timeout

    def _call(self, texts, input_type):
        out = []
        for i in range(0, len(texts), self.batch):
            r = httpx.post(f"{self.base}/embeddings", json={"model": self.model, "input": texts[i:i + self.batch],
                                                             "input_type": input_type, "truncate": self.truncate,
                                                             "encoding_format": "float"},
                           headers=self.headers, timeout=self.timeout)
            r.raise_for_status()
            out += [d["embedding"] for d in sorted(r.json()["data"], key=lambda d: d["index"])]
        return out

    def embed_documents(self, texts):
        return self._call(texts, "passage")

    def embed_query(self, text):
        return self._call([text], "query")[0]


# ------------------------------------------------------------------------------------------ ranking
_FOREIGN_RANKER_LOCK = threading.Lock()


def rerank(ranker, documents: Sequence[Document], query: str, top_n: int) -> List[Document]:
    """``ranker.compress_documents`` keeping ``top_n`` documents. This framework's rankers take ``top_n`` per call; a
    foreign (LangChain-style) compressor keeps it as state, so it is set for the call and restored under a lock -
    one ranker object is shared by every request of a server."""
    if isinstance(ranker, Ranker):
        return ranker.compress_documents(documents, query, top_n=top_n)
    with _FOREIGN_RANKER_LOCK:
        saved, ranker.top_n = ranker.top_n, top_n
        try:
            return ranker.compress_documents(documents, query)
        finally:
            ranker.top_n = saved


class Ranker:
    def __init__(self, top_n: int = 4):
        self.top_n = top_n

    def rank(self, query: str, passages: List[str]) -> List[tuple]:
        raise NotImplementedError

    @tracing.traced("reranker")
    def compress_documents(self, documents: Sequence[Document], query: str,
                           top_n: Optional[int] = None) -> List[Document]:
        """Reorders documents by relevance, keeps ``top_n`` (default: the ranker's own), stores ``relevance_score`` in
        metadata. A per-call ``top_n`` leaves the shared ranker untouched, so concurrent requests can differ."""
        docs = list(documents)
        if not docs:
            return []
        ranked = self.rank(query, [d.page_content for d in docs])[: top_n or self.top_n]
        out = []
        for i, s in ranked:
            d = docs[i]
            md = dict(d.metadata)
            md["relevance_score"] = float(s)
            out.append(Document(d.page_content, md))
        return out


class LocalRanker(Ranker):
    def __init__(self, reranker, top_n: int = 4, truncate: str = "END"):
        super().__init__(top_n)
        self.r, self.truncate = reranker, truncate

    def rank(self, query, passages):
        return self.r.rank(query, passages, None, self.truncate)


class RemoteRanker(Ranker):
    def __init__(self, base_url: str, model: str, top_n: int = 4, truncate: str = "END",
                 api_key: Optional[str] = None):
        super().__init__(top_n)
        self.base, self.model, self.truncate = _base(base_url), model, truncate
        self.headers = {"Authorization": f"Bearer {api_key}"} if api_key else {}

    def rank(self, query, passages):
        r = httpx.post(f"{self.base}/ranking", json={"model": self.model, "query": {"text": query},
                                                     "passages": [{"text": p} for p in passages],
                                                     "truncate": self.truncate}, headers=self.headers, timeout=600)
        r.raise_for_status()
        return [(x["index"], x["logit"]) for x in r.json()["rankings"]]
