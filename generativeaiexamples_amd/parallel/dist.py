"""Process groups and collectives.

MI355X topology: 8 GPUs, fully connected by xGMI, 7 point-to-point links of
~153 GB/s per GPU. One process per GPU; ``torch.distributed`` with backend ``nccl`` is RCCL on
ROCm. Sub-groups: ``tp`` (generator tensor parallel), ``dp`` (embedder / index shards) and ``ep``
(MoE experts). The TP group's RCCL collectives run on a high-priority stream; prefill row-parallel
projections overlap their all-reduce with the next row chunk's GEMM (``tp_linear_all_reduce``).

On the CPU test tier the same code runs over ``gloo`` (world_size 2, 127.0.0.1 rendezvous).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass, field
from typing import Optional

import torch
import torch.distributed as dist

from .fault import RankFailure, guard  # noqa: F401  (re-exported)


@dataclass
class DistContext:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    tp_size: int = 1
    dp_size: int = 1
    backend: str = "none"
    device: torch.device = field(default_factory=lambda: torch.device("cpu"))
    tp_group: Optional[object] = None
    dp_group: Optional[object] = None
    world_group: Optional[object] = None
    # Megatron-style sequence parallelism inside the TP group: between the row-parallel and
    # the next column-parallel GEMM the activations stay sharded along tokens, each all-reduce becomes a
    # reduce-scatter + all-gather pair (same bytes on the xGMI ring) and the residual adds / norms run on
    # T / tp rows per rank.
    sequence_parallel: bool = False
    # one-shot peer-memory all-reduce for TP messages <= GAI_CUSTOM_AR_MAX_MB (parallel/custom_ar.py)
    custom_ar: Optional[object] = None

    @property
    def tp_rank(self) -> int:
        return self.rank % self.tp_size

    @property
    def dp_rank(self) -> int:
        return self.rank // self.tp_size

    @property
    def is_distributed(self) -> bool:
        return self.world_size > 1

    # ---------------- collectives (no-ops when the group has one member) ----------------
    def tp_all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        if self.tp_size > 1:
            car = self.custom_ar
            if car is not None and car.eligible(t):  # latency-bound sizes: one-shot xGMI push
                with guard("tp_custom_all_reduce", self.rank):  # fault injection + error mapping
                    return car.all_reduce(t)
            with guard("tp_all_reduce", self.rank):
                if t.is_cuda or t.dtype in (torch.float32, torch.float64):
                    dist.all_reduce(t, group=self.tp_group)
                else:  # gloo (CPU test tier): reduce reduced-precision tensors in fp32
                    f = t.float()
                    dist.all_reduce(f, group=self.tp_group)
                    t.copy_(f)
        return t

    def tp_linear_all_reduce(self, x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None,
                             chunks: Optional[int] = None) -> torch.Tensor:
        """Row-parallel projection ``x @ w^T (+ bias)`` followed by its TP all-reduce, pipelined over row
        chunks for prefill-sized inputs: chunk i's all-reduce is issued asynchronously (RCCL runs it on
        its own high-priority stream, see ``init_distributed``) as soon as chunk i's GEMM is enqueued, so
        it overlaps chunk i+1's GEMM on the compute stream; the compute stream waits for every chunk's
        all-reduce before the result is used. Decode-sized inputs (and TP = 1) take the plain path.
        Same math as ``linear`` + ``tp_all_reduce`` (rows are independent)."""
        from .. import ops

        M = x.shape[0]
        if chunks is None:
            chunks = min(4, M // int(os.environ.get("GAI_TP_OVERLAP_CHUNK_ROWS", "1024")))
        if self.tp_size == 1 or chunks <= 1:
            return self.tp_all_reduce(ops.linear(x, w, bias=bias))
        out = torch.empty(M, w.shape[0], dtype=x.dtype, device=x.device)
        step = -(-M // chunks)
        asynchronous = x.is_cuda or x.dtype in (torch.float32, torch.float64)
        works = []
        with guard("tp_linear_all_reduce", self.rank):
            for a in range(0, M, step):
                part = out[a:a + step]
                ops.linear(x[a:a + step], w, bias=bias, out=part)
                if asynchronous:
                    works.append(dist.all_reduce(part, group=self.tp_group, async_op=True))
                else:  # gloo with reduced precision (CPU test tier): synchronous fp32 reduce per chunk
                    self.tp_all_reduce(part)
            for wk in works:
                wk.wait()
        return out

    def tp_all_reduce_rmsnorm(self, h: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float
                              ) -> torch.Tensor:
        """The TP block boundary: all-reduce the row-parallel partial sums ``h``, add them to ``residual``
        (in place) and return rmsnorm(residual) * w. On the custom all-reduce this is ONE kernel (peer push,
        reduce, residual add and norm over whole rows), otherwise the all-reduce plus the fused add+norm
        kernel; both round like the unfused path."""
        from .. import ops

        car = self.custom_ar
        if self.tp_size > 1 and car is not None and car.eligible_rmsnorm(h):
            with guard("tp_custom_all_reduce_rmsnorm", self.rank):
                return car.all_reduce_rmsnorm(h, residual, w, eps)
        self.tp_all_reduce(h)
        return ops.rms_norm(h, w, eps, residual=residual)

    def check_comm(self) -> None:
        """Poll the device-side error word of the custom all-reduce; call at a point that has already
        synchronised with the stream (the engine does it after copying the sampled tokens to the host). A
        set word means a peer missed the bounded spin: the custom all-reduce is retired (later messages go
        to RCCL) and :class:`RankFailure` is raised so serving marks the step's requests failed."""
        car = self.custom_ar
        if car is None:
            return
        try:
            car.check()
        except RankFailure:
            self.custom_ar = None
            raise

    def tp_all_gather_last(self, t: torch.Tensor) -> torch.Tensor:
        """Concatenate the per-rank shards along the last dim (vocab-parallel logits)."""
        if self.tp_size == 1:
            return t
        parts = [torch.empty_like(t) for _ in range(self.tp_size)]
        with guard("tp_all_gather", self.rank):
            dist.all_gather(parts, t.contiguous(), group=self.tp_group)
        return torch.cat(parts, dim=-1)

    def tp_reduce_scatter_rows(self, t: torch.Tensor) -> torch.Tensor:
        """Partial sums [T, D] (T divisible by tp) -> this rank's summed rows [T / tp, D]."""
        if self.tp_size == 1:
            return t
        n = t.shape[0] // self.tp_size
        with guard("tp_reduce_scatter", self.rank):
            if t.is_cuda:
                out = torch.empty(n, *t.shape[1:], dtype=t.dtype, device=t.device)
                dist.reduce_scatter_tensor(out, t.contiguous(), group=self.tp_group)
                return out
            f = t.float()  # gloo has no reduce-scatter: all-reduce + keep the local slice
            dist.all_reduce(f, group=self.tp_group)
            return f[self.tp_rank * n:(self.tp_rank + 1) * n].to(t.dtype).contiguous()

    def tp_all_gather_rows(self, t: torch.Tensor) -> torch.Tensor:
        """Row shards [T / tp, D] -> [T, D] in TP-rank order."""
        if self.tp_size == 1:
            return t
        with guard("tp_all_gather_rows", self.rank):
            if t.is_cuda:
                out = torch.empty(t.shape[0] * self.tp_size, *t.shape[1:], dtype=t.dtype, device=t.device)
                dist.all_gather_into_tensor(out, t.contiguous(), group=self.tp_group)
                return out
            parts = [torch.empty_like(t) for _ in range(self.tp_size)]
            dist.all_gather(parts, t.contiguous(), group=self.tp_group)
            return torch.cat(parts)

    def all_gather_obj(self, obj, group=None):
        if not self.is_distributed:
            return [obj]
        out = [None] * (dist.get_world_size(group) if group is not None else self.world_size)
        with guard("all_gather_object", self.rank):
            dist.all_gather_object(out, obj, group=group)
        return out

    def barrier(self):
        if self.is_distributed:
            with guard("barrier", self.rank):
                if self.backend == "nccl":
                    dist.barrier(device_ids=[self.local_rank])
                else:
                    dist.barrier()


_CTX: DistContext | None = None


def get_context() -> DistContext:
    global _CTX
    if _CTX is None:
        _CTX = DistContext()
        if torch.cuda.is_available():
            _CTX.device = torch.device("cuda", 0)
    return _CTX


def init_distributed(tp_size: int = 1, backend: str | None = None, timeout_s: int | None = None,
                     sequence_parallel: bool | None = None) -> DistContext:
    """Initialise from torchrun-style env vars (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR/PORT).

    Falls back to a single-process context when WORLD_SIZE is unset or 1.
    """
    global _CTX
    timeout_s = timeout_s or int(os.environ.get("GAI_DIST_TIMEOUT_S", "600"))
    # a hung RCCL collective aborts the communicator (-> RankFailure) instead of blocking forever
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    use_gpu = torch.cuda.is_available()
    if backend is None:
        # RCCL refuses two ranks on one device: a single-GPU rehearsal (GAI_SINGLE_DEVICE=1) uses gloo
        single = os.environ.get("GAI_SINGLE_DEVICE") == "1"
        backend = os.environ.get("GAI_DIST_BACKEND") or ("nccl" if use_gpu and not single else "gloo")
    ctx = DistContext(rank=rank, world_size=world, local_rank=local, backend=backend if world > 1 else "none")
    if sequence_parallel is None:
        sequence_parallel = os.environ.get("GAI_SEQUENCE_PARALLEL") == "1"
    ctx.sequence_parallel = bool(sequence_parallel)
    if use_gpu:
        # GAI_SINGLE_DEVICE=1: every rank on cuda:0 (gloo rehearsal of a multi-rank run on one GPU)
        dev_idx = 0 if os.environ.get("GAI_SINGLE_DEVICE") == "1" else local
        torch.cuda.set_device(dev_idx)
        ctx.device = torch.device("cuda", dev_idx)
    if world > 1:
        if not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            kw = dict(backend=backend, timeout=datetime.timedelta(seconds=timeout_s))
            if backend == "nccl" and os.environ.get("GAI_SINGLE_DEVICE") != "1":
                kw["device_id"] = ctx.device
            dist.init_process_group(**kw)
        assert world % tp_size == 0, "world size must be a multiple of tp_size"
        ctx.tp_size, ctx.dp_size = tp_size, world // tp_size
        ctx.world_group = dist.group.WORLD
        # every rank must create every group in the same order
        # RCCL runs the TP group's collectives on a high-priority stream, so an all-reduce issued
        # asynchronously beside a GEMM (tp_linear_all_reduce) is scheduled ahead of the compute kernels
        tp_opts = None
        if backend == "nccl":
            try:
                tp_opts = dist.ProcessGroupNCCL.Options()
                tp_opts.is_high_priority_stream = True
            except (AttributeError, RuntimeError):
                tp_opts = None
        for d in range(ctx.dp_size):
            ranks = list(range(d * tp_size, (d + 1) * tp_size))
            g = (dist.new_group(ranks, pg_options=tp_opts) if tp_opts is not None else dist.new_group(ranks)) \
                if tp_size > 1 else None
            if rank in ranks:
                ctx.tp_group = g
        for t in range(tp_size):
            ranks = list(range(t, world, tp_size))
            g = dist.new_group(ranks) if ctx.dp_size > 1 else None
            if rank in ranks:
                ctx.dp_group = g
        want_car = os.environ.get("GAI_CUSTOM_AR", "1" if backend == "nccl" else "0") == "1"
        if tp_size > 1 and use_gpu and want_car:
            from .custom_ar import maybe_create

            ctx.custom_ar = maybe_create(ctx.tp_group, tp_size, ctx.device)
    _CTX = ctx
    return ctx


def shutdown():
    global _CTX
    if _CTX is not None and _CTX.custom_ar is not None:
        _CTX.custom_ar.close()
        _CTX.custom_ar = None
    if dist.is_initialized():
        dist.destroy_process_group()
    _CTX = None
