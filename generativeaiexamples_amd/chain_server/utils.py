"""Factories used by the example pipelines (the roles of RAG/src/chain_server/utils.py:173-715).

get_config / get_prompts / get_llm / get_embedding_model / get_ranking_model / get_text_splitter /
get_vectorstore / get_docs_vectorstore / del_docs_vectorstore. Model engines:
* ``mi355x`` (default) and ``huggingface``: the in-process MI355X engines of this process
  (built once from the ``engine`` config section / ``APP_ENGINE_*``),
* ``nvidia-ai-endpoints`` / ``openai``: a NIM-compatible server at ``server_url``.
"""
from __future__ import annotations

import logging
import os
import threading
from functools import lru_cache
from typing import Dict, List, Optional

import yaml

from ..rag.prompts import DEFAULT_PROMPTS
from ..rag.text_splitter import TokenTextSplitter
from .configuration import AppConfig
from .connectors import (ChatLLM, Embeddings, LocalChatLLM, LocalEmbeddings, LocalRanker, Ranker, RemoteChatLLM,
                         RemoteEmbeddings, RemoteRanker)
from .vectorstore import VectorStore, get_store

log = logging.getLogger(__name__)
LOCAL_ENGINES = {"mi355x", "local", "huggingface"}
REMOTE_ENGINES = {"nvidia-ai-endpoints", "openai", "nim"}


@lru_cache
def get_config() -> AppConfig:
    path = os.environ.get("APP_CONFIG_FILE", "/dev/null")
    cfg = AppConfig.from_file(path)
    log.info("chain-server config: %s", cfg)
    return cfg


def _merge(base: dict, over: dict) -> dict:
    out = dict(base)
    for k, v in (over or {}).items():
        out[k] = _merge(out[k], v) if isinstance(v, dict) and isinstance(out.get(k), dict) else v
    return out


def _example_dir() -> Optional[str]:
    from .server import EXAMPLE_DIR

    p = os.path.join(EXAMPLE_DIR, os.environ.get("EXAMPLE_PATH", "basic_rag/langchain"))
    return p if os.path.isdir(p) else None


@lru_cache
def get_prompts() -> Dict[str, str]:
    """Defaults <- example's prompt.yaml <- PROMPT_CONFIG_FILE (default /prompt.yaml), recursively merged."""
    prompts: Dict = dict(DEFAULT_PROMPTS)
    d = _example_dir()
    if d and os.path.isfile(os.path.join(d, "prompt.yaml")):
        with open(os.path.join(d, "prompt.yaml")) as f:
            prompts = _merge(prompts, yaml.safe_load(f) or {})
    user = os.environ.get("PROMPT_CONFIG_FILE", "/prompt.yaml")
    if os.path.isfile(user):
        with open(user) as f:
            prompts = _merge(prompts, yaml.safe_load(f) or {})
    return prompts


# --------------------------------------------------------------------------------- in-process hub
_HUB = None
_HUB_LOCK = threading.Lock()


def get_hub():
    """The process-wide ServiceHub (built on first use from the engine config section)."""
    global _HUB
    with _HUB_LOCK:
        if _HUB is None:
            from ..serving.hub import HubSpec, ServiceHub

            c = get_config()
            e = c.engine
            spec = HubSpec(llm=e.llm or None, llm_weights=e.llm_weights or None, embedder=e.embedder or None,
                           embedder_weights=e.embedder_weights or None, reranker=e.reranker or None,
                           reranker_weights=e.reranker_weights or None, served_llm_name=c.llm.model_name,
                           served_embedder_name=c.embeddings.model_name, served_reranker_name=c.ranking.model_name,
                           max_num_seqs=e.max_batch, max_model_len=e.max_model_len, kv_memory_fraction=e.kv_fraction,
                           device=e.device or None)
            _HUB = ServiceHub.build(spec)
        return _HUB


def set_hub(hub) -> None:
    """Inject a pre-built hub (tests, the combined server)."""
    global _HUB
    with _HUB_LOCK:
        _HUB = hub


# --------------------------------------------------------------------------------- factories
def get_llm(**kwargs) -> ChatLLM:
    c = get_config().llm
    settings = {k: kwargs.get(k) for k in ("temperature", "top_p", "max_tokens", "stop") if k in kwargs}
    if c.ignore_eos:
        settings["ignore_eos"] = True
    eng = c.model_engine.lower()
    if eng in REMOTE_ENGINES or (c.server_url and eng not in LOCAL_ENGINES):
        if not c.server_url and eng == "nvidia-ai-endpoints":
            base = "https://integrate.api.nvidia.com"
        else:
            base = c.server_url
        return RemoteChatLLM(base, c.model_name, api_key=os.environ.get("NVIDIA_API_KEY"), **settings)
    hub = get_hub()
    llm = hub.llm(c.model_name)
    if llm is None:
        raise RuntimeError(f"no in-process LLM serves '{c.model_name}'")
    return LocalChatLLM(llm, c.model_name, **settings)


def get_embedding_model() -> Embeddings:
    c = get_config().embeddings
    eng = c.model_engine.lower()
    if eng in REMOTE_ENGINES:
        return RemoteEmbeddings(c.server_url or "https://integrate.api.nvidia.com", c.model_name,
                                api_key=os.environ.get("NVIDIA_API_KEY"))
    emb = get_hub().embedder(c.model_name)
    if emb is None:
        raise RuntimeError(f"no in-process embedder serves '{c.model_name}'")
    return LocalEmbeddings(emb)


def get_ranking_model() -> Optional[Ranker]:
    """None when no reranker is available (pipelines then run without reranking)."""
    c, r = get_config().ranking, get_config().retriever
    try:
        if c.model_engine.lower() in REMOTE_ENGINES:
            if not c.server_url:
                return None
            return RemoteRanker(c.server_url, c.model_name, top_n=r.top_k)
        rr = get_hub().reranker(c.model_name)
        return LocalRanker(rr, top_n=r.top_k) if rr is not None else None
    except Exception as e:  # degrade gracefully like the reference
        log.warning("ranking model unavailable: %s", e)
        return None


def get_text_splitter():
    c = get_config().text_splitter
    tok = None
    try:
        emb = get_hub().embedder(get_config().embeddings.model_name)
        tok = emb.tok if emb is not None else None
    except Exception:
        tok = None
    if tok is None:
        from ..engine.tokenizer import bert_byte_tokenizer

        tok = bert_byte_tokenizer()
    return TokenTextSplitter(tok, tokens_per_chunk=max(8, c.chunk_size - 2), overlap=min(c.chunk_overlap, c.chunk_size - 3))


def collection_name(default: str = "vector_db") -> str:
    return os.environ.get("COLLECTION_NAME", default)


def get_vectorstore(embeddings: Optional[Embeddings] = None, collection: Optional[str] = None) -> VectorStore:
    c = get_config().vector_store
    embeddings = embeddings or get_embedding_model()
    dev = None
    try:
        if isinstance(embeddings, LocalEmbeddings):
            dev = embeddings.e.model.device
    except Exception:
        dev = None
    return get_store(collection or collection_name(), embeddings, c.metric, c.persist_dir or None, device=dev,
                     hybrid=bool(c.hybrid))


def get_docs_vectorstore(store: VectorStore) -> List[str]:
    return store.filenames()


def del_docs_vectorstore(store: VectorStore, filenames: List[str]) -> bool:
    ok = True
    for f in filenames:  # every filename (the reference stops after the first: SURVEY §7.7 item 5)
        ok = store.delete_filename(f) and ok
    return ok
