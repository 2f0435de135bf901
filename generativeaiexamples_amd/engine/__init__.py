"""Serving engines: LLM generator (continuous batching, paged KV, HIP graphs), embedder, reranker."""
from .llm_engine import EngineConfig, LLMEngine, Request, RequestOutput  # noqa: F401
from .sampling import SamplingParams  # noqa: F401
