"""Expert parallelism with all-to-all token exchange (§5.8 "All-to-all ... direct peer
writes over the 7 xGMI links").

For data-parallel attention + expert-parallel MoE: each rank owns E/W experts and its own tokens.
``dispatch`` sends every (token, expert) pair to the rank owning the expert (one count exchange,
then one variable-split ``all_to_all_single`` of the rows, expert ids and routing weights - RCCL
runs all-to-all as direct peer transfers, one xGMI link per peer); the owner runs its grouped
GEMMs on the received rows; ``combine`` returns the expert outputs with the reverse all-to-all and
reduces them with the routing weights into the token order.
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


def _a2a(x: torch.Tensor, send: List[int], recv: List[int], group) -> torch.Tensor:
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
