"""Autograd-aware tensor-parallel collectives (Megatron f / g operators) for training over RCCL."""
from __future__ import annotations

import torch
import torch.distributed as dist


class _CopyToTP(torch.autograd.Function):
    """Column-parallel input: identity forward, all-reduce of the input gradient backward."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return x

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        dist.all_reduce(g, group=ctx.group)
        return g, None


class _ReduceFromTP(torch.autograd.Function):
    """Row-parallel output: all-reduce of the partial sums forward, identity backward."""

    @staticmethod
    def forward(ctx, x, group):
        x = x.contiguous()
        dist.all_reduce(x, group=group)
        return x

    @staticmethod
    def backward(ctx, g):
        return g, None


class _GatherLast(torch.autograd.Function):
    """Vocab-parallel logits: all-gather along the last dim forward, keep the local slice backward."""

    @staticmethod
    def forward(ctx, x, group, rank, world):
        ctx.rank, ctx.n = rank, x.shape[-1]
        parts = [torch.empty_like(x) for _ in range(world)]
        dist.all_gather(parts, x.contiguous(), group=group)
        return torch.cat(parts, -1)

    @staticmethod
    def backward(ctx, g):
        return g[..., ctx.rank * ctx.n:(ctx.rank + 1) * ctx.n].contiguous(), None, None, None


def copy_to_tp(x, ctx):
    return _CopyToTP.apply(x, ctx.tp_group) if ctx.tp_size > 1 else x


def reduce_from_tp(x, ctx):
    return _ReduceFromTP.apply(x, ctx.tp_group) if ctx.tp_size > 1 else x


def gather_last(x, ctx):
    return _GatherLast.apply(x, ctx.tp_group, ctx.tp_rank, ctx.tp_size) if ctx.tp_size > 1 else x
