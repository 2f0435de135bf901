"""Data-parallel sharded index over RCCL ("10M-vector index sharded DP=8").

Every rank holds one :class:`HBMIndex` shard. A search is two all-gathers and no host synchronisation:
  1. the per-rank query batches are all-gathered, each padded to ``max_queries`` rows (a bound every rank agrees on
     up front: the engine / benchmark batch), so no count exchange - and no device -> host read of counts - precedes
     the scan;
  2. the fused top-k kernel of the local shard runs over ALL gathered queries (padding rows are scanned and ignored);
  3. the per-rank candidates - fp32 relevance and int64 global row, packed into ONE int32 message - are all-gathered;
  4. each rank merges only its own queries' W candidate lists with the in-tree top-k merge kernel (ops.topk_merge:
     the second stage of the similarity top-k, topk.hip sim_topk_stage2).
Without ``max_queries`` the batches are exchanged at their true sizes after a count all-gather (one host sync).
Message sizes are tiny next to xGMI bandwidth, so the cost is the two collective latencies; the scan itself is
perfectly parallel and HBM-bound on every GPU.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
import torch.distributed as dist

from ..parallel.fault import guard
from .hbm_index import HBMIndex


class ShardedIndex:
    def __init__(self, local: HBMIndex, group=None, max_queries: Optional[int] = None):
        self.local = local
        self.group = group
        self.max_queries = max_queries
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
        counts = [int(x) for x in self._all_gather(n)]  # host sync: only without max_queries
        mx = max(counts)
        pad = torch.zeros(mx, *t.shape[1:], dtype=t.dtype, device=t.device)
        pad[: t.shape[0]] = t
        parts = self._all_gather(pad)
        return torch.cat([p[:c] for p, c in zip(parts, counts)]), counts

    def search_raw(self, queries: torch.Tensor, k: int):
        """Local queries [q, dim] -> (relevance [q, k], global rows [q, k]) merged over all shards. A collective:
        every rank of the group calls it (with ``max_queries``: at most that many queries each)."""
        from .. import ops

        if self.world == 1:
            rel, rows = self.local.search_raw(queries, k)
            return rel, rows
        q = queries.shape[0]
        if self.max_queries is not None:
            if q > self.max_queries:
                raise ValueError(f"{q} queries > max_queries {self.max_queries} of this sharded index")
            buf = torch.zeros(self.max_queries, queries.shape[1], dtype=self.local.dtype, device=queries.device)
            buf[:q] = queries
            allq = torch.cat(self._all_gather(buf))
            start = self.rank * self.max_queries
        else:
            allq, counts = self._gather_var(queries.to(self.local.dtype))
            start = sum(counts[: self.rank])
        rel, rows = self.local.search_raw(allq, k)
        kk = rel.shape[1]
        if kk < k:  # shard smaller than k: pad
            padn = k - kk
            rel = torch.cat([rel, rel.new_full((rel.shape[0], padn), float("-inf"))], 1)
            rows = torch.cat([rows, rows.new_full((rows.shape[0], padn), -1)], 1)
        rows = torch.where(rows >= 0, self.global_row(rows, self.rank), rows)
        # one message: [Q, k] fp32 relevance + [Q, k] int64 rows as [Q, 3k] int32
        packed = torch.cat([rel.float().contiguous().view(torch.int32), rows.contiguous().view(torch.int32)], 1)
        parts = [p[start:start + q] for p in self._all_gather(packed)]  # this rank's queries, from every shard
        R = torch.stack([p[:, :k].contiguous().view(torch.float32) for p in parts])  # [W, q, k]
        I = torch.stack([p[:, k:].contiguous().view(torch.int64) for p in parts])    # [W, q, k]
        top, pos = ops.topk_merge(R, k)
        gi = torch.gather(I.permute(1, 0, 2).reshape(q, self.world * k), 1, pos)
        return top, gi
