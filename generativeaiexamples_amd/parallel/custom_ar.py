"""One-shot peer-memory all-reduce for latency-bound TP messages.

RCCL's ring all-reduce crosses ``world - 1`` hops one after another. On the fully connected xGMI
mesh of an MI355X node every rank can push its whole input to all peers concurrently (one link
each) and reduce locally, so a decode-size message (Llama-3-70B TP8, batch 64: 1 MiB per
all-reduce, 160 per token) costs one hop. The kernel is ``csrc/comm/custom_ar.hip``; this module
owns the IPC buffers:

* every rank allocates (uncached, so no GPU's L2 keeps a stale line) a data area of
  ``2 parity x world x max_bytes`` and a signal area, exports both with ``hipIpcGetMemHandle``;
* handles are exchanged with one ``all_gather_object`` on the TP group (works over RCCL or gloo);
* every rank maps its peers' areas (``hipIpcOpenMemHandle``).

The launch takes no per-call scalar (epochs live in a device counter per workgroup), so it is
captured into the decode HIP graph like any other kernel. Messages larger than ``max_bytes`` or not
a multiple of 16 bytes go to RCCL. A peer that never arrives makes the kernel give up after a
bounded spin and set an error word (checked by :meth:`check`), never hang the GPU.

Two more kernels share the machinery:

* two-shot (``algo="twoshot"``, auto above ``GAI_AR_TWOSHOT_MIN_KB`` = 512 KiB at world > 2):
  reduce-scatter then all-gather, both as direct peer writes, over a second buffer set - each xGMI
  link carries 2/W of the message instead of all of it, which is what bounds large messages on the
  point-to-point mesh;
* ``all_reduce_rmsnorm``: the one-shot exchange fused with the residual add and the next RMSNorm
  (``DistContext.tp_all_reduce_rmsnorm``, used at every TP block boundary of the Llama family), one
  kernel and one pass over the activations instead of all-reduce + add&norm.

Reference parity: the reference has no in-repo collective (NCCL is implicit inside TRT-LLM,
SURVEY §2.4 P1); this is the "custom one-shot xGMI all-reduce for <= 1 MiB" of its MI355X design.
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch
import torch.distributed as dist


def _native():
    from .. import ops

    return ops.native()


class CustomAllReduce:
    """Peer-memory all-reduce over one process group. All ranks must construct it together."""

    def __init__(self, group=None, device: Optional[torch.device] = None, max_bytes: int = 8 << 20,
                 a2a_max_bytes: int = 0):
        """max_bytes: largest all-reduce (<= AR_CHUNK x AR_MAX_BLOCKS = 8 MiB); a2a_max_bytes: largest all-to-all
        segment (the expert-parallel prefill slabs; the all-to-all kernel's blocks loop over chunks). Every
        collective uses one slot size, the larger of the two: the collectives share the epoch counters, and a
        peer may write call e + 1 while this rank still reads call e, so the parity regions of consecutive calls
        must not overlap."""
        C = _native()
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if not 2 <= self.world <= 8:
            raise ValueError("CustomAllReduce supports 2..8 ranks")
        max_bytes = min(int(max_bytes), C.AR_CHUNK * C.AR_MAX_BLOCKS)
        self.max_bytes = max_bytes - max_bytes % C.AR_CHUNK
        a2a = -(-max(int(a2a_max_bytes), self.max_bytes) // C.AR_CHUNK) * C.AR_CHUNK
        self.slot_bytes = a2a
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        with torch.cuda.device(self.device):
            self._data = C.ipc_malloc(2 * self.world * self.slot_bytes)
            self._sig = C.ipc_malloc(C.AR_MAX_BLOCKS * 8 * 4)
            handles = (C.ipc_get_handle(self._data), C.ipc_get_handle(self._sig))
            allh: List = [None] * self.world
            dist.all_gather_object(allh, handles, group=group)
            self._opened: List[int] = []
            self.data_ptrs, self.sig_ptrs = [], []
            for q, (hd, hs) in enumerate(allh):
                if q == self.rank:
                    self.data_ptrs.append(self._data)
                    self.sig_ptrs.append(self._sig)
                else:
                    pd, ps = C.ipc_open(hd), C.ipc_open(hs)
                    self._opened += [pd, ps]
                    self.data_ptrs.append(pd)
                    self.sig_ptrs.append(ps)
            self.counters = torch.zeros(C.AR_MAX_BLOCKS, dtype=torch.int32, device=self.device)
            self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
            # two-shot buffers: [2 parity][world src][2 regions][region] with region = max_bytes / world,
            # signals [block][2 phases][8], own epochs
            self.region_bytes = -(-self.max_bytes // self.world // C.AR_CHUNK) * C.AR_CHUNK
            self._data2 = C.ipc_malloc(2 * self.world * 2 * self.region_bytes)
            self._sig2 = C.ipc_malloc(C.AR_MAX_BLOCKS * 2 * 8 * 4)
            handles2 = (C.ipc_get_handle(self._data2), C.ipc_get_handle(self._sig2))
            allh2: List = [None] * self.world
            dist.all_gather_object(allh2, handles2, group=group)
            self.data2_ptrs, self.sig2_ptrs = [], []
            for q, (hd, hs) in enumerate(allh2):
                if q == self.rank:
                    self.data2_ptrs.append(self._data2)
                    self.sig2_ptrs.append(self._sig2)
                else:
                    pd, ps = C.ipc_open(hd), C.ipc_open(hs)
                    self._opened += [pd, ps]
                    self.data2_ptrs.append(pd)
                    self.sig2_ptrs.append(ps)
            self.counters2 = torch.zeros(C.AR_MAX_BLOCKS, dtype=torch.int32, device=self.device)
            # one-shot below this size, two-shot above (2 ranks: one-shot always - same bytes per link)
            self.twoshot_min = int(os.environ.get("GAI_AR_TWOSHOT_MIN_KB", "512")) << 10
        torch.cuda.synchronize(self.device)
        dist.barrier(group=group)  # every peer has mapped every buffer before the first launch
        self._closed = False

    def eligible(self, t: torch.Tensor) -> bool:
        nbytes = t.numel() * t.element_size()
        return (not self._closed and t.is_cuda and t.is_contiguous() and t.dtype in (torch.bfloat16, torch.float32)
                and 0 < nbytes <= self.max_bytes and nbytes % 16 == 0)

    def algo_for(self, nbytes: int) -> str:
        if self.world > 2 and nbytes >= self.twoshot_min and nbytes % (16 * self.world) == 0:
            return "twoshot"
        return "oneshot"

    def all_reduce(self, t: torch.Tensor, out: Optional[torch.Tensor] = None, algo: str = "auto") -> torch.Tensor:
        """Sum ``t`` over the group (in place unless ``out`` is given). Graph-capturable. ``algo``: oneshot
        (every rank pushes the whole message to every peer: one hop, latency-bound sizes), twoshot
        (reduce-scatter + all-gather over direct peer writes: 2/W of the message per link), auto."""
        out = t if out is None else out
        nbytes = t.numel() * t.element_size()
        if algo == "auto":
            algo = self.algo_for(nbytes)
        if algo == "twoshot":
            _native().custom_allreduce_twoshot(t, out, self.data2_ptrs, self.sig2_ptrs, self.counters2, self.err,
                                               self.rank, self.region_bytes)
        else:
            _native().custom_allreduce(t, out, self.data_ptrs, self.sig_ptrs, self.counters, self.err, self.rank,
                                       self.slot_bytes)
        return out

    def eligible_a2a(self, t: torch.Tensor) -> bool:
        """Equal-split all-to-all of ``t`` (dim 0 split into world segments) fits the one-shot buffers."""
        nbytes = t.numel() * t.element_size()
        return (not self._closed and t.is_cuda and t.is_contiguous() and nbytes % (16 * self.world) == 0
                and 0 < nbytes // self.world <= self.slot_bytes)

    def all_to_all(self, t: torch.Tensor, out: Optional[torch.Tensor] = None, send_rows: Optional[torch.Tensor] = None,
                   recv_rows: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Segment q of ``t`` (dim 0 in world equal parts) goes to rank q; segment q of the result came from rank
        q. Direct peer writes, one hop, graph-capturable (csrc/comm/custom_ar.hip a2a_oneshot_kernel).
        send_rows / recv_rows (device int32 [world], together): only the first send_rows[q] rows (dim-0 rows of
        ``t``) of segment q cross to rank q, and only the first recv_rows[q] rows of the result's segment q are
        written (the rest keep ``out``'s previous contents); the counts never leave the device."""
        out = torch.empty_like(t) if out is None else out
        row_bytes = t[0].numel() * t.element_size() if send_rows is not None else 0
        _native().custom_all_to_all(t, out, self.data_ptrs, self.sig_ptrs, self.counters, self.err, self.rank,
                                    self.slot_bytes, send_rows, recv_rows, row_bytes)
        return out

    def eligible_rmsnorm(self, t: torch.Tensor) -> bool:
        D = t.shape[-1]
        return (self.eligible(t) and t.dtype == torch.bfloat16 and D % 2048 == 0 and 16384 % (2 * D) == 0)

    def all_reduce_rmsnorm(self, t: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float,
                           out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """residual += all_reduce(t); return rmsnorm(residual) * w - one kernel (see custom_ar.hip)."""
        out = torch.empty_like(t) if out is None else out
        _native().custom_allreduce_rmsnorm(t, out, residual, w, eps, self.data_ptrs, self.sig_ptrs, self.counters,
                                           self.err, self.rank, self.slot_bytes)
        return out

    def check(self) -> None:
        """Raise :class:`RankFailure` if a launch timed out waiting for a peer (host sync). The error word
        stays set, and the caller (``DistContext.check_comm``) retires this all-reduce: its per-block epochs
        are out of step with the peers' after a timeout, so later calls could not be trusted either."""
        if int(self.err.item()):
            from .fault import RankFailure
            raise RankFailure(f"custom all-reduce on rank {self.rank}: a peer did not arrive within the bounded "
                              "spin; the reduced activations of that step are invalid")

    def close(self) -> None:
        if self._closed:
            return
        C = _native()
        torch.cuda.synchronize(self.device)
        for p in self._opened:
            C.ipc_close(p)
        C.ipc_free(self._data)
        C.ipc_free(self._sig)
        C.ipc_free(self._data2)
        C.ipc_free(self._sig2)
        self._closed = True


def maybe_create(group, world: int, device: torch.device) -> Optional[CustomAllReduce]:
    """The TP group's custom all-reduce, or None (CPU, one rank, GAI_CUSTOM_AR=0, or setup failure)."""
    if world < 2 or world > 8 or device.type != "cuda" or os.environ.get("GAI_CUSTOM_AR", "1") == "0":
        return None
    mb = int(os.environ.get("GAI_CUSTOM_AR_MAX_MB", "8"))
    return CustomAllReduce(group, device, max_bytes=mb << 20)
