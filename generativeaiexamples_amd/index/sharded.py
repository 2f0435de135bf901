"""Data-parallel sharded index over RCCL ("10M-vector index sharded DP=8").

Every rank holds one :class:`HBMIndex` shard. A search
  1. all-gathers the per-rank query batches ([q_r, dim] bf16 - a few KB),
  2. runs the fused top-k kernel of the local shard over ALL gathered queries,
  3. all-gathers the per-rank candidates ([Q, k] fp32 relevance + int64 global row),
  4. merges them with one top-k over the N*k candidates per query, and each rank keeps the rows
     of its own queries.
Message sizes are tiny next to xGMI bandwidth, so the cost is the two collective latencies; the
scan itself is perfectly parallel and HBM-bound on every GPU.
"""
from __future__ import annotations

from typing import List, Tuple

import torch
import torch.distributed as dist

from ..parallel.fault import guard
from .hbm_index import HBMIndex


class ShardedIndex:
    def __init__(self, local: HBMIndex, group=None):
        self.local = local
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0

    def global_row(self, local_rows: torch.Tensor, shard: int) -> torch.Tensor:
        return local_rows + (shard << 40)

    @staticmethod
    def split_row(g: int) -> Tuple[int, int]:
        return g >> 40, g & ((1 << 40) - 1)

    def _comm_dev(self, t: torch.Tensor) -> torch.device:
        # gloo (CPU test tier / single-GPU rehearsal) only moves host tensors
        return t.device if dist.get_backend(self.group) == "nccl" else torch.device("cpu")

    def _all_gather(self, t: torch.Tensor) -> List[torch.Tensor]:
        dev = self._comm_dev(t)
        src = t.to(dev)
        if src.dtype == torch.bfloat16 and dev.type == "cpu":
            src = src.float()
        parts = [torch.empty_like(src) for _ in range(self.world)]
        with guard("index_all_gather", self.rank):
            dist.all_gather(parts, src.contiguous(), group=self.group)
        return [p.to(t.device, t.dtype) for p in parts]

    def _gather_var(self, t: torch.Tensor) -> Tuple[torch.Tensor, List[int]]:
        n = torch.tensor([t.shape[0]], device=t.device, dtype=torch.int64)
        counts = [int(x) for x in self._all_gather(n)]
        mx = max(counts)
        pad = torch.zeros(mx, *t.shape[1:], dtype=t.dtype, device=t.device)
        pad[: t.shape[0]] = t
        parts = self._all_gather(pad)
        return torch.cat([p[:c] for p, c in zip(parts, counts)]), counts

    def search_raw(self, queries: torch.Tensor, k: int):
        """Local queries [q, dim] -> (relevance [q, k], global rows [q, k]) merged over all shards."""
        if self.world == 1:
            rel, rows = self.local.search_raw(queries, k)
            return rel, rows
        allq, counts = self._gather_var(queries.to(self.local.dtype))
        rel, rows = self.local.search_raw(allq, k)
        kk = rel.shape[1]
        if kk < k:  # shard smaller than k: pad
            padn = k - kk
            rel = torch.cat([rel, rel.new_full((rel.shape[0], padn), float("-inf"))], 1)
            rows = torch.cat([rows, rows.new_full((rows.shape[0], padn), -1)], 1)
        rows = torch.where(rows >= 0, self.global_row(rows, self.rank), rows)
        R = torch.cat(self._all_gather(rel.float()), 1)  # [Q, world*k]
        I = torch.cat(self._all_gather(rows), 1)
        top, pos = torch.topk(R, k, dim=1)
        gi = torch.gather(I, 1, pos)
        start = sum(counts[: self.rank])
        return top[start:start + counts[self.rank]], gi[start:start + counts[self.rank]]
