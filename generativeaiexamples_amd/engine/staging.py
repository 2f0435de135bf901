"""Per-step host->device staging without per-step allocations.

Every engine step ships a handful of small index arrays (token ids, positions, KV slots, block tables,
sampling parameters) to the GPU. Allocating pinned memory per step (``tensor.pin_memory()``) costs
host time on every decode step; instead one persistent pinned int32 buffer and one device buffer are
reused: ``stage`` bump-allocates regions of them within a step (8-byte aligned, so int64/fp32 arrays
can be reinterpreted), packs the arrays with numpy and issues ONE async H2D copy per call.
``reset()`` at the start of a step recycles the regions - safe because the engine synchronises on
the sampled tokens at the end of every step, so no copy from the previous step is still in flight.
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np
import torch


class HostStager:
    def __init__(self, device, capacity: int = 1 << 18):
        self.device = torch.device(device)
        self.pin = self.device.type == "cuda"
        self._alloc(capacity)

    def _alloc(self, n: int):
        self.capacity = n
        self.host = torch.empty(n, dtype=torch.int32, pin_memory=self.pin)
        self.host_np = self.host.numpy()
        self.dev = torch.empty(n, dtype=torch.int32, device=self.device) if self.pin else self.host
        self.off = 0

    def reset(self):
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
            if start:  # this step already staged regions that are in flight: never move them
                raise RuntimeError("HostStager: step staging exceeds capacity; construct with a larger capacity")
            self._alloc(max(2 * self.capacity, total))
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
