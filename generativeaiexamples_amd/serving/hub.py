"""ServiceHub: the models one process serves (generator(s), embedder(s), reranker(s)) and their names.

The reference runs one container per model (LLM NIM :8000, embedding NIM :9080, ranking NIM
:1976 - docker-compose-nim-ms.yaml); here they share one process per GPU and one memory plan
(generator + embedder + reranker + index co-located in 288 GB of HBM).
Model names are the NIM names the reference's configs use, so ``APP_LLM_MODELNAME`` etc. work
unchanged. LoRA adapter names (multi-LoRA by model name, NIM_PEFT_SOURCE) alias their base model.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

from ..engine.embedder import Embedder, Reranker
from ..engine.llm_engine import EngineConfig, LLMEngine
from ..utils.metrics import METRICS
from .async_engine import AsyncLLMEngine


@dataclass
class HubSpec:
    llm: Optional[str] = "llama3-8b"
    llm_weights: Optional[str] = None
    embedder: Optional[str] = "e5-large-v2"
    embedder_weights: Optional[str] = None
    reranker: Optional[str] = None
    reranker_weights: Optional[str] = None
    served_llm_name: Optional[str] = None
    served_embedder_name: Optional[str] = None
    served_reranker_name: Optional[str] = None
    max_num_seqs: int = 256
    max_model_len: int = 8192
    max_batched_tokens: int = 16384
    use_graphs: bool = True
    kv_memory_fraction: float = 0.6
    lora_adapters: Dict[str, str] = field(default_factory=dict)
    device: Optional[str] = None
    # tensor parallelism of the generator across the ranks of this job (one process per GPU, RCCL):
    # rank 0 serves the API and plans every step, the other ranks execute its plans (LLMEngine.follow)
    tp: int = 1
    dtype: Optional[str] = None  # generator dtype override ("float32" for exact CPU rehearsals)
    kv_cache_dtype: str = "auto"  # "fp8": OCP e4m3fn paged KV cache (NIM / TRT-LLM kv_cache_dtype option)

    @staticmethod
    def from_env() -> "HubSpec":
        g = os.environ.get
        s = HubSpec()
        s.llm = g("APP_ENGINE_LLM", s.llm) or None
        s.llm_weights = g("APP_ENGINE_LLMWEIGHTS")
        s.embedder = g("APP_ENGINE_EMBEDDER", s.embedder) or None
        s.embedder_weights = g("APP_ENGINE_EMBEDDERWEIGHTS")
        s.reranker = g("APP_ENGINE_RERANKER") or None
        s.reranker_weights = g("APP_ENGINE_RERANKERWEIGHTS")
        s.served_llm_name = g("APP_LLM_MODELNAME")
        s.served_embedder_name = g("APP_EMBEDDINGS_MODELNAME")
        s.served_reranker_name = g("APP_RANKING_MODELNAME")
        s.max_num_seqs = int(g("APP_ENGINE_MAXBATCH", s.max_num_seqs))
        s.max_model_len = int(g("APP_ENGINE_MAXMODELLEN", s.max_model_len))
        s.device = g("APP_ENGINE_DEVICE")
        s.tp = int(g("APP_ENGINE_TP", s.tp))
        s.kv_cache_dtype = g("APP_ENGINE_KVCACHEDTYPE", s.kv_cache_dtype)
        return s


class ServiceHub:
    def __init__(self):
        self.follower_engine: Optional[LLMEngine] = None  # TP follower ranks: the engine they execute
        self.llms: Dict[str, AsyncLLMEngine] = {}
        self.embedders: Dict[str, Embedder] = {}
        self.rerankers: Dict[str, Reranker] = {}
        self.loras: Dict[str, str] = {}
        self.aliases: Dict[str, str] = {}
        self.default_llm_name: Optional[str] = None
        self.default_embedder_name: Optional[str] = None
        self.default_reranker_name: Optional[str] = None
        self.default_max_tokens = 1024

    # ---------------------------------------------------------------- registration
    def add_llm(self, name: str, engine: LLMEngine | AsyncLLMEngine):
        a = engine if isinstance(engine, AsyncLLMEngine) else AsyncLLMEngine(engine)
        self.llms[name] = a
        self.default_llm_name = self.default_llm_name or name

    def add_embedder(self, name: str, emb: Embedder):
        if hasattr(emb, "capture_graphs"):
            emb.capture_graphs()  # before serving: no graph capture beside the running engine thread
        self.embedders[name] = emb
        self.default_embedder_name = self.default_embedder_name or name

    def add_reranker(self, name: str, rr: Reranker):
        self.rerankers[name] = rr
        self.default_reranker_name = self.default_reranker_name or name

    def add_alias(self, alias: str, base: str):
        self.aliases[alias] = base

    def lora_for(self, name: Optional[str]) -> Optional[str]:
        """Adapter to apply when a request names ``name`` (None for base-model names)."""
        return self.loras.get(name) if name else None

    # ---------------------------------------------------------------- lookup
    def _pick(self, table: dict, name: Optional[str], default: Optional[str]):
        if not table:
            return None
        if name is None or name == "":
            return table.get(default)
        name = self.aliases.get(name, name)
        if name in table:
            return table[name]
        # the reference's clients send catalog names ("meta/llama3-8b-instruct", "NV-Embed-QA", ...):
        # a single-model table serves whatever name it is asked for
        return next(iter(table.values())) if len(table) == 1 else None

    def llm(self, name=None) -> Optional[AsyncLLMEngine]:
        return self._pick(self.llms, name, self.default_llm_name)

    def embedder(self, name=None) -> Optional[Embedder]:
        return self._pick(self.embedders, name, self.default_embedder_name)

    def reranker(self, name=None) -> Optional[Reranker]:
        return self._pick(self.rerankers, name, self.default_reranker_name)

    def model_list(self) -> List[Tuple[str, str]]:
        out = [(n, n) for n in list(self.llms) + list(self.embedders) + list(self.rerankers)]
        out += [(a, b) for a, b in self.aliases.items()]
        return out

    def max_model_len(self, name) -> Optional[int]:
        a = self.llms.get(self.aliases.get(name, name))
        return a.engine.cfg.max_model_len if a else None

    def ready(self) -> bool:
        return all(a.healthy for a in self.llms.values())

    def update_gauges(self):
        for a in self.llms.values():
            s = a.engine.sched
            METRICS.kv_usage.set(1.0 - s.num_free_blocks() / max(1, s.num_blocks()))

    def shutdown(self):
        for a in self.llms.values():
            a.shutdown()
            a.engine.release_followers(stop=True)  # TP: end the followers' plan loops

    @property
    def is_follower(self) -> bool:
        return self.follower_engine is not None

    def serve_follower(self) -> str:
        """TP follower ranks: execute rank 0's step plans until it stops serving."""
        op = "yield"
        while op == "yield":
            op = self.follower_engine.follow()
        return op

    # ---------------------------------------------------------------- construction
    @classmethod
    def build(cls, spec: HubSpec) -> "ServiceHub":
        from ..models.registry import build_embedder_service, build_llm, build_reranker_service, default_device

        import torch

        dev = torch.device(spec.device) if spec.device else default_device()
        hub = cls()
        if spec.tp > 1:
            from ..parallel.dist import init_distributed

            ctx = init_distributed(tp_size=spec.tp)
            if ctx.world_size != spec.tp:
                raise ValueError(f"tp={spec.tp} needs a job of exactly {spec.tp} ranks (WORLD_SIZE={ctx.world_size})")
            dev = ctx.device if dev.type == "cuda" else dev
        dtype = getattr(torch, spec.dtype) if spec.dtype else None
        if spec.llm:
            m, tok, name = build_llm(spec.llm, spec.llm_weights, device=dev, dtype=dtype)
            eng = LLMEngine(m, tok, EngineConfig(max_num_seqs=spec.max_num_seqs, max_model_len=spec.max_model_len,
                                                 max_batched_tokens=spec.max_batched_tokens,
                                                 use_graphs=spec.use_graphs and dev.type == "cuda",
                                                 kv_memory_fraction=spec.kv_memory_fraction,
                                                 kv_cache_dtype=spec.kv_cache_dtype))
            if not eng.leader:  # TP follower: no API, no embedder / reranker
                hub.follower_engine = eng
                return hub
            hub.add_llm(spec.served_llm_name or name, eng)
            for alias, path in spec.lora_adapters.items():
                hub.add_alias(alias, spec.served_llm_name or name)
                if path:  # a trained adapter directory: served unmerged, selected by model name
                    eng.add_lora(alias, path)
                    hub.loras[alias] = alias
        if spec.embedder:
            emb, name = build_embedder_service(spec.embedder, spec.embedder_weights, device=dev)
            hub.add_embedder(spec.served_embedder_name or name, emb)
        if spec.reranker:
            rr, name = build_reranker_service(spec.reranker, spec.reranker_weights, device=dev)
            hub.add_reranker(spec.served_reranker_name or name, rr)
        return hub
