"""Bucketed data-parallel gradient all-reduce overlapped with the backward pass.

Parameters are grouped (in reverse registration order = the order backward produces their grads)
into ~``bucket_mb`` flat buckets. A post-accumulate-grad hook marks a parameter ready; when the last
parameter of a bucket is ready its gradients are copied into the flat buffer and an async
all-reduce is launched on the DP group, so communication of late layers overlaps the backward of
early layers. ``finish()`` waits for the outstanding work, averages and scatters the results back.
On xGMI rings, buckets of tens of MB amortise the per-collective latency.
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist


class GradBucketer:
    def __init__(self, params: List[torch.Tensor], group=None, bucket_mb: float = 25.0):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.params = [p for p in params if p.requires_grad]
        self.buckets: List[List[torch.Tensor]] = []
        cur, size = [], 0
        for p in reversed(self.params):
            cur.append(p)
            size += p.numel() * 4
            if size >= bucket_mb * (1 << 20):
                self.buckets.append(cur)
                cur, size = [], 0
        if cur:
            self.buckets.append(cur)
        self.owner = {}
        for bi, b in enumerate(self.buckets):
            for p in b:
                self.owner[id(p)] = bi
        self.flat = [torch.zeros(sum(p.numel() for p in b), device=b[0].device, dtype=torch.float32)
                     for b in self.buckets]
        self.pending = [0] * len(self.buckets)
        self.work: List[Optional[object]] = [None] * len(self.buckets)
        self.launched = 0
        self.sync = True  # set False for non-final micro-batches of a gradient-accumulation step
        if self.world > 1:
            for p in self.params:
                p.register_post_accumulate_grad_hook(self._hook)
        self.reset()

    def reset(self):
        self.pending = [len(b) for b in self.buckets]
        self.work = [None] * len(self.buckets)
        self.launched = 0

    def _hook(self, p: torch.Tensor):
        if not self.sync:
            return
        bi = self.owner[id(p)]
        self.pending[bi] -= 1
        if self.pending[bi] == 0:
            self._launch(bi)

    def _launch(self, bi: int):
        flat, o = self.flat[bi], 0
        for p in self.buckets[bi]:
            n = p.numel()
            flat[o:o + n].copy_(p.grad.reshape(-1) if p.grad is not None else torch.zeros(n, device=flat.device))
            o += n
        self.work[bi] = dist.all_reduce(flat, group=self.group, async_op=True)
        self.launched += 1

    def finish(self):
        """Call after backward (of the last micro-batch): wait, average, write back."""
        if self.world == 1:
            return
        for bi in range(len(self.buckets)):
            if self.work[bi] is None:  # a bucket whose params got no grad in this step
                self._launch(bi)
            self.work[bi].wait()
            flat, o = self.flat[bi], 0
            flat.div_(self.world)
            for p in self.buckets[bi]:
                n = p.numel()
                if p.grad is None:
                    p.grad = torch.zeros_like(p)
                p.grad.copy_(flat[o:o + n].view_as(p.grad))
                o += n
        self.reset()
