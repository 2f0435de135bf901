"""Rank-0 -> follower broadcast of engine step plans for tensor-parallel serving.

A TP=N generator is ONE serving instance: rank 0 owns the C++ scheduler, the request table, sampling
decisions and the HTTP front; ranks 1..N-1 own only their weight / KV shards. Every engine step rank 0
serialises the *step plan* (token ids, positions, KV slots, varlen metadata, block tables, sampling
parameters, multi-step run length) and publishes it here; the followers execute exactly that plan, so
all ranks issue the same kernels and the same RCCL / peer-memory collectives in the same order, and no
rank makes a scheduling decision of its own (no lock-step drift, aborts and disconnects are handled once,
on rank 0, by simply leaving the request out of the next plan).

Transport: ranks of one TP group share an MI355X node, so the plan goes through a native POSIX
shared-memory broadcast ring (``_rt.ShmChannel``, csrc/runtime/shm_channel.cpp): ~3 us per message,
nothing queued on the GPU streams. Followers detect a dead rank 0 (writer pid gone) and raise
:class:`~.fault.RankFailure`.

Wire format: msgpack maps whose numpy arrays are tagged ``{"__nd__": dtype, "s": shape, "b": bytes}``.
"""
from __future__ import annotations

import os
import uuid
from typing import Any, Optional

import msgpack
import numpy as np

from .fault import RankFailure

_ND = "__nd__"


def _enc(o: Any):
    if isinstance(o, np.ndarray):
        a = np.ascontiguousarray(o)
        return {_ND: a.dtype.str, "s": list(a.shape), "b": a.tobytes()}
    if isinstance(o, np.generic):
        return o.item()
    raise TypeError(f"step plan: cannot serialise {type(o).__name__}")


def _dec(d: dict):
    if _ND in d:
        return np.frombuffer(d["b"], dtype=np.dtype(d[_ND])).reshape(d["s"])
    return d


def pack(msg: dict) -> bytes:
    return msgpack.packb(msg, default=_enc, use_bin_type=True)


def unpack(b: bytes) -> dict:
    return msgpack.unpackb(b, object_hook=_dec, raw=False, strict_map_key=False)


class StepChannel:
    """Broadcast channel of one TP group: rank 0 (tp_rank 0) sends, the other members receive.

    All members of the group construct it together (the segment name is agreed through one
    ``broadcast_object_list`` on the TP group)."""

    def __init__(self, ctx, slot_bytes: int = 16 << 20, num_slots: int = 4, timeout_s: Optional[float] = None):
        import torch.distributed as dist

        from .. import _rt

        self.ctx = ctx
        self.leader = ctx.tp_rank == 0
        self.timeout_s = float(os.environ.get("GAI_STEP_TIMEOUT_S", "-1")) if timeout_s is None else timeout_s
        local = int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")))
        if ctx.tp_size > local:
            raise RuntimeError("StepChannel: a TP group must live on one node (shared-memory plan broadcast)")
        name = [f"/gai_step_{os.getpid()}_{uuid.uuid4().hex[:8]}" if self.leader else None]
        src = ctx.rank - ctx.tp_rank  # global rank of this group's tp_rank 0
        if self.leader:
            self.ch = _rt.ShmChannel.create(name[0], ctx.tp_size - 1, slot_bytes, num_slots)
        dist.broadcast_object_list(name, src=src, group=ctx.tp_group)
        self.name = name[0]
        if not self.leader:
            self.ch = _rt.ShmChannel.open(self.name, ctx.tp_rank - 1, 120.0)
        dist.barrier(group=ctx.tp_group)  # every follower attached before the first publish
        self.sent = 0

    def send(self, msg: dict) -> None:
        assert self.leader
        b = pack(msg)
        if len(b) > self.ch.slot_bytes:
            raise ValueError(f"step plan of {len(b)} bytes exceeds the {self.ch.slot_bytes}-byte channel slot")
        if not self.ch.send(b, self.timeout_s):
            raise RankFailure(f"step channel: a follower did not consume plan {self.sent} within {self.timeout_s}s")
        self.sent += 1

    def recv(self) -> dict:
        assert not self.leader
        try:
            b = self.ch.recv(self.timeout_s)
        except RuntimeError as e:  # writer process gone
            raise RankFailure(f"step channel on rank {self.ctx.rank}: {e}") from e
        if b is None:
            raise RankFailure(f"step channel on rank {self.ctx.rank}: no plan from rank 0 within {self.timeout_s}s")
        return unpack(b)
