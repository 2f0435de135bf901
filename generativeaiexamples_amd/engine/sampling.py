"""Sampling parameters (OpenAI / NIM request fields) and their per-batch device tensors."""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

import torch


@dataclass
class SamplingParams:
    temperature: float = 0.2          # chain-server default (server.py Prompt.temperature)
    top_p: float = 0.7                # chain-server default
    top_k: int = 0
    max_tokens: int = 1024
    stop: List[str] = field(default_factory=list)
    stop_token_ids: List[int] = field(default_factory=list)
    ignore_eos: bool = False
    seed: Optional[int] = None
    frequency_penalty: float = 0.0
    presence_penalty: float = 0.0
    repetition_penalty: float = 1.0
    min_tokens: int = 0
    logprobs: bool = False
    # constrained decoding (engine/guided.py): a compiled grammar / JSON-schema matcher, or None
    guided: Optional[object] = None
    # elastic re-queue (serving/router.py): tokens of this completion already delivered by a replica that
    # failed mid-stream. They extend the prompt, count for the penalties and are replayed into the grammar
    # matcher; the caller has already taken them off max_tokens / min_tokens.
    resume_ids: List[int] = field(default_factory=list)
    resume_sent_chars: Optional[int] = None  # characters of their text the client already has

    @property
    def greedy(self) -> bool:
        return self.temperature <= 0.0 or self.top_k == 1

    @property
    def has_penalty(self) -> bool:
        return self.frequency_penalty != 0.0 or self.presence_penalty != 0.0 or self.repetition_penalty != 1.0


class SamplingBatch:
    """Packs the per-row sampling parameters of one step into device tensors (one staged H2D copy)."""

    @staticmethod
    def arrays(params: List[SamplingParams], seeds: List[int]):
        """Host arrays (temperature fp32, top_p fp32, top_k int32, seeds int64) of one step's rows."""
        import numpy as np
        temp = np.fromiter((0.0 if p.top_k == 1 else p.temperature for p in params), np.float32, len(params))
        top_p = np.fromiter((p.top_p for p in params), np.float32, len(params))
        top_k = np.fromiter((p.top_k for p in params), np.int32, len(params))
        return [temp, top_p, top_k, np.asarray(seeds, dtype=np.int64)]

    def __init__(self, params: List[SamplingParams], seeds: List[int], device, stager=None):
        temp, top_p, top_k, sd = self.arrays(params, seeds)
        if stager is None:
            from .staging import HostStager
            stager = HostStager(device, 1024)
        self.temperature, self.top_p, self.top_k, self.seeds = stager.stage([temp, top_p, top_k, sd])
