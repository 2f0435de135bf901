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

    @property
    def greedy(self) -> bool:
        return self.temperature <= 0.0 or self.top_k == 1

    @property
    def has_penalty(self) -> bool:
        return self.frequency_penalty != 0.0 or self.presence_penalty != 0.0 or self.repetition_penalty != 1.0


class SamplingBatch:
    """Packs the per-row sampling parameters of one step into device tensors (one H2D copy)."""

    def __init__(self, params: List[SamplingParams], seeds: List[int], device):
        n = len(params)
        f = torch.empty(n, 2, dtype=torch.float32)
        k = torch.empty(n, dtype=torch.int32)
        s = torch.empty(n, dtype=torch.int64)
        for i, p in enumerate(params):
            f[i, 0] = 0.0 if p.top_k == 1 else p.temperature
            f[i, 1] = p.top_p
            k[i] = p.top_k
            s[i] = seeds[i]
        pin = device.type == "cuda"
        if pin:
            f, k, s = f.pin_memory(), k.pin_memory(), s.pin_memory()
        f = f.to(device, non_blocking=True)
        self.temperature = f[:, 0].contiguous()
        self.top_p = f[:, 1].contiguous()
        self.top_k = k.to(device, non_blocking=True)
        self.seeds = s.to(device, non_blocking=True)
