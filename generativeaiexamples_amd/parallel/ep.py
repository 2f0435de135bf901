"""Expert parallelism with all-to-all token exchange (§5.8 "All-to-all ... direct peer
writes over the 7 xGMI links").

For data-parallel attention + expert-parallel MoE: each rank owns E/W experts and its own tokens.
``dispatch`` sends every (token, expert) pair to the rank owning the expert (one count exchange,
then one variable-split ``all_to_all_single`` of the rows, expert ids and routing weights - RCCL
runs all-to-all as direct peer transfers, one xGMI link per peer); the owner runs its grouped
GEMMs on the received rows; ``combine`` returns the expert outputs with the reverse all-to-all and
reduces them with the routing weights into the token order.

``dispatch_padded`` / ``local_experts_padded`` / ``combine_padded`` are the decode-time variant: every
rank sends each peer a fixed-capacity slab (``capacity`` rows, default T*k = dropless), positions
inside a slab are computed on the device (scatter / cumsum, no ``bincount`` / ``.tolist()``), padding
rows carry the sentinel expert id ``e_local`` that the grouped GEMM skips, and both exchanges are
equal-split ``all_to_all_single`` calls - no host synchronisation anywhere, so a whole MoE decode step
(routing, dispatch, grouped GEMMs, combine) can be captured in one HIP graph. The price is bandwidth:
W x capacity rows per exchange instead of the exact counts, which at decode batch sizes (tens of tokens)
is a few MB over xGMI and far cheaper than a host round trip.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List

import torch
import torch.distributed as dist


@dataclass
class EPPlan:
    order: torch.Tensor           # pair indices sorted by destination rank
    send_counts: List[int]
    recv_counts: List[int]
    num_tokens: int
    top_k: int


def _host_plane(x: torch.Tensor, group) -> bool:
    """Device tensors over a gloo group (one-GPU multi-rank rehearsal): exchange through host memory."""
    return x.is_cuda and dist.get_backend(group) == "gloo"


def _a2a(x: torch.Tensor, send: List[int], recv: List[int], group) -> torch.Tensor:
    if _host_plane(x, group):
        return _a2a(x.cpu(), send, recv, group).to(x.device)
    out = torch.empty(sum(recv), *x.shape[1:], dtype=x.dtype, device=x.device)
    if x.is_cuda or x.dtype in (torch.float32, torch.int64, torch.int32):
        dist.all_to_all_single(out, x.contiguous(), recv, send, group=group)
        return out
    # gloo on CPU: move reduced-precision payloads as fp32
    o32 = torch.empty(out.shape, dtype=torch.float32)
    dist.all_to_all_single(o32, x.float().contiguous(), recv, send, group=group)
    return o32.to(x.dtype)


def dispatch(x: torch.Tensor, ids: torch.Tensor, weights: torch.Tensor, num_experts: int, group=None):
    """-> (rows [R, D], local expert ids [R] int32, plan). Rows arrive grouped by source rank."""
    world = dist.get_world_size(group)
    e_local = num_experts // world
    T, k = ids.shape
    flat = ids.reshape(-1).long()
    dest = flat // e_local
    order = torch.argsort(dest, stable=True)
    send_counts = torch.bincount(dest, minlength=world)
    recv_counts = torch.empty_like(send_counts)
    if _host_plane(send_counts, group):
        rc = torch.empty(world, dtype=send_counts.dtype)
        dist.all_to_all_single(rc, send_counts.cpu(), group=group)
        recv_counts = rc
    else:
        dist.all_to_all_single(recv_counts, send_counts, group=group)
    sc, rc = send_counts.tolist(), recv_counts.tolist()
    rows = x[(order // k)]
    eid = (flat[order] % e_local).to(torch.int32)
    recv_rows = _a2a(rows, sc, rc, group)
    recv_eid = _a2a(eid, sc, rc, group)
    return recv_rows, recv_eid, EPPlan(order, sc, rc, T, k)


def combine(y: torch.Tensor, weights: torch.Tensor, plan: EPPlan, group=None) -> torch.Tensor:
    """y: expert outputs for the received rows (same order as dispatch delivered them)."""
    back = _a2a(y, plan.recv_counts, plan.send_counts, group)  # pairs in `order` order
    pair_out = torch.empty_like(back)
    pair_out[plan.order] = back
    w = weights.reshape(-1, 1).to(torch.float32)
    out = (pair_out.float() * w).view(plan.num_tokens, plan.top_k, -1).sum(1)
    return out.to(y.dtype)


def local_experts(rows: torch.Tensor, eid: torch.Tensor, w13: torch.Tensor, w2: torch.Tensor) -> torch.Tensor:
    """Run the received rows through the local experts with the grouped GEMM kernels."""
    from .. import ops

    e_local = w13.shape[0]
    R = rows.shape[0]
    if R == 0:
        return rows.new_zeros(0, w2.shape[1])
    order = torch.argsort(eid.long(), stable=True)
    counts = torch.bincount(eid.long(), minlength=e_local)
    offs = torch.zeros(e_local + 1, dtype=torch.int32, device=rows.device)
    offs[1:] = counts.cumsum(0).to(torch.int32)
    h1 = ops.moe_gemm(rows, order.to(torch.int32), w13, offs, R, True)
    y_sorted = ops.moe_gemm(h1, None, w2, offs, R, False)
    y = torch.empty_like(y_sorted)
    y[order] = y_sorted
    return y


def _a2a_equal(x: torch.Tensor, group, xchg=None) -> torch.Tensor:
    """Equal-split all-to-all: the peer-memory one-shot kernel when the group has one (``xchg``, a
    CustomAllReduce of the EP group: direct xGMI writes, one hop, capturable even over a gloo control plane),
    else RCCL's ``all_to_all_single`` (gloo on CPU)."""
    if xchg is not None and xchg.eligible_a2a(x):
        return xchg.all_to_all(x.contiguous())
    if _host_plane(x, group):
        return _a2a_equal(x.cpu(), group).to(x.device)
    out = torch.empty_like(x)
    if x.is_cuda or x.dtype in (torch.float32, torch.int64, torch.int32):
        dist.all_to_all_single(out, x.contiguous(), group=group)
        return out
    o32 = torch.empty(x.shape, dtype=torch.float32)
    dist.all_to_all_single(o32, x.float().contiguous(), group=group)
    return o32.to(x.dtype)


@dataclass
class EPPaddedPlan:
    ids: torch.Tensor   # [T, k] global expert ids of the pairs
    pos: torch.Tensor   # [T, k] rank of each pair in its destination's (token, choice)-ordered run
    offs: torch.Tensor  # [W + 1] start of every destination's run
    capacity: int
    e_local: int


def dispatch_padded(x: torch.Tensor, ids: torch.Tensor, num_experts: int, capacity: int | None = None, group=None,
                    xchg=None):
    """-> (rows [W*C, D], local expert ids [W*C] int32 (e_local = padding), plan). Sync-free, capturable.
    Pairs beyond ``capacity`` for one destination are dropped (capacity = T*k never drops). The plan is one
    counting-sort kernel over the destinations (ops.ep_dispatch_plan) and the slabs one gather kernel
    (ops.ep_pack); the rows and their expert ids travel in ONE exchange (ids packed as two bf16 lanes)."""
    from .. import ops

    world = dist.get_world_size(group)
    e_local = num_experts // world
    T, k = ids.shape
    C = T * k if capacity is None else capacity
    offs, pos, a_pairs = ops.ep_dispatch_plan(ids, world, e_local)
    if xchg is not None:  # one exchange: the expert id rides in each slab row's 16-B tail
        D = x.shape[1]
        slab, _ = ops.ep_pack(x, ids, offs, a_pairs, world, C, e_local, ids_in_rows=True)
        got = _a2a_equal(slab, group, xchg)
        rows = got[:, :D].contiguous()
        eid = got[:, D:D + 2].contiguous().view(torch.int32).view(-1)
    else:
        send, send_eid = ops.ep_pack(x, ids, offs, a_pairs, world, C, e_local)
        rows = _a2a_equal(send, group)
        eid = _a2a_equal(send_eid, group)
    return rows, eid, EPPaddedPlan(ids, pos, offs, C, e_local)


def local_experts_padded(rows: torch.Tensor, eid: torch.Tensor, w13: torch.Tensor, w2: torch.Tensor) -> torch.Tensor:
    """Grouped expert GEMMs over a padded slab: the device-side dispatch plan sorts the sentinel rows
    last and the grouped GEMM's tile walk stops at offs[e_local], so padding costs no FLOPs."""
    from .. import ops

    e_local = w13.shape[0]
    R = rows.shape[0]
    a_rows, offs, pos = ops.moe_dispatch(eid.view(-1, 1), e_local + 1)
    h1 = ops.moe_gemm(rows, a_rows, w13, offs, R, True)
    y_sorted = ops.moe_gemm(h1, None, w2, offs, R, False)
    return y_sorted[pos.view(-1).long()]


def combine_padded(y: torch.Tensor, weights: torch.Tensor, plan: EPPaddedPlan, group=None, xchg=None,
                   residual: torch.Tensor | None = None) -> torch.Tensor:
    """Return the expert outputs to their ranks and reduce them with the routing weights (+ residual) in one
    kernel (ops.ep_combine); dropped pairs contribute nothing."""
    from .. import ops

    back = _a2a_equal(y.contiguous(), group, xchg)
    return ops.ep_combine(back, plan.ids, plan.pos, plan.offs, weights, residual, plan.e_local, plan.capacity)
