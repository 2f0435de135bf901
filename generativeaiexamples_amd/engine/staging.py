"""Per-step host->device staging without per-step allocations.

Every engine step ships a handful of small index arrays (token ids, positions, KV slots, block tables,
sampling parameters) to the GPU. Allocating pinned memory per step (``tensor.pin_memory()``) costs
host time on every decode step; instead one persistent pinned int32 buffer and one device buffer are
reused: ``stage`` bump-allocates regions of them within a step (8-byte aligned, so int64/fp32 arrays
can be reinterpreted), packs the arrays with numpy and issues ONE async H2D copy per call.
``reset()`` recycles the regions once the copies issued since the last ``fence()`` have executed
(the engine alternates two stagers between launches, so a pipelined run's copies can still be queued
behind the run in flight while the other bank is filled). A step that stages more than the capacity
gets an extra region for the rest of that step (regions already in flight never move); the next
``reset()`` folds the extra size into one larger buffer.
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np
import torch


class HostStager:
    def __init__(self, device, capacity: int = 1 << 18):
        self.device = torch.device(device)
        self.pin = self.device.type == "cuda"
        self._event = None
        self._retired: list = []  # regions replaced within the current step (copies may be in flight)
        self._grow_to = 0
        self._alloc(capacity)

    def _alloc(self, n: int):
        self.capacity = n
        self.host = torch.empty(n, dtype=torch.int32, pin_memory=self.pin)
        self.host_np = self.host.numpy()
        self.dev = torch.empty(n, dtype=torch.int32, device=self.device) if self.pin else self.host
        self.off = 0

    def fence(self):
        """Mark the end of a launch's copies (the next reset() waits for them)."""
        if self.pin:
            self._event = torch.cuda.Event()
            self._event.record()

    def reset(self):
        if self._event is not None:
            self._event.synchronize()
            self._event = None
        self._retired.clear()
        if self._grow_to > self.capacity:
            self._alloc(self._grow_to)
        self._grow_to = 0
        self.off = 0

    def stage(self, arrays: Sequence[np.ndarray]) -> List[torch.Tensor]:
        """arrays of int32 / float32 / int64 (any shape) -> device tensors of the same dtype and shape."""
        metas, total = [], 0
        for a in arrays:
            a = np.ascontiguousarray(a)
            if a.dtype not in (np.int32, np.float32, np.int64):
                a = a.astype(np.int32)
            words = a.size * (2 if a.dtype == np.int64 else 1)
            metas.append((a, total, words))
            total += (words + 1) & ~1  # keep every region 8-byte aligned
        start = self.off
        if start + total > self.capacity:
            # regions staged earlier in this step may be in flight: keep them alive, continue in a new region
            self._grow_to = max(self._grow_to, 2 * self.capacity, start + 2 * total)
            if start:
                self._retired.append((self.host, self.dev))
            self._alloc(max(2 * self.capacity, total))
            start = 0
        for a, o, words in metas:
            self.host_np[start + o:start + o + words] = a.reshape(-1).view(np.int32)
        if self.pin and total:
            self.dev[start:start + total].copy_(self.host[start:start + total], non_blocking=True)
        self.off = start + total
        out = []
        for a, o, words in metas:
            v = self.dev[start + o:start + o + words]
            if a.dtype == np.float32:
                v = v.view(torch.float32)
            elif a.dtype == np.int64:
                v = v.view(torch.int64)
            out.append(v.view(*a.shape) if a.ndim != 1 else v)
        return out
