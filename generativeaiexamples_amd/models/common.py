"""Shared model-side plumbing: the per-step ForwardBatch and weight initialisation helpers."""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Optional

import torch


@dataclass
class ForwardBatch:
    """Device-side description of one engine step (prefill tokens first, then decode tokens).

    Produced by the engine from the native scheduler's StepBatch.
    """
    token_ids: torch.Tensor          # [T] int32
    positions: torch.Tensor          # [T] int32
    slots: torch.Tensor              # [T] int32 (KV slot = block*16 + offset)
    num_prefill_tokens: int = 0
    # prefill part (varlen, chunked over cached prefixes)
    cu_q: Optional[torch.Tensor] = None            # [P+1] int32
    prefill_ctx: Optional[torch.Tensor] = None     # [P] int32
    prefill_block_tables: Optional[torch.Tensor] = None  # [P, maxb] int32
    prefill_tiles: Optional[torch.Tensor] = None   # attention tiles (host-built)
    prefill_qlen: List[int] = field(default_factory=list)
    # decode part
    decode_ctx: Optional[torch.Tensor] = None      # [Dn] int32
    decode_block_tables: Optional[torch.Tensor] = None  # [Dn, maxb] int32
    max_decode_ctx: int = 0
    # rows of the flat token dim whose logits are needed (in output order)
    sample_rows: Optional[torch.Tensor] = None     # [S] int64

    @property
    def num_tokens(self) -> int:
        return int(self.token_ids.shape[0])

    @property
    def num_decode(self) -> int:
        return self.num_tokens - self.num_prefill_tokens


def init_linear_(w: torch.Tensor, gen: torch.Generator, fan_in: int) -> torch.Tensor:
    """Deterministic scaled-normal init done in fp32 on the CPU generator, then cast (random-init weights)."""
    std = 1.0 / math.sqrt(fan_in)
    tmp = torch.empty(w.shape, dtype=torch.float32)
    tmp.normal_(0.0, std, generator=gen)
    w.copy_(tmp)
    return w


def randn_like_(w: torch.Tensor, seed: int, std: float) -> torch.Tensor:
    """Fast on-device random init (for multi-GB benchmark models)."""
    g = torch.Generator(device=w.device)
    g.manual_seed(seed)
    if w.is_floating_point():
        w.normal_(0.0, std, generator=g)
    return w
