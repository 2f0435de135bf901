"""Expert parallelism with all-to-all token exchange (§5.8 "All-to-all ... direct peer
writes over the 7 xGMI links").

For data-parallel attention + expert-parallel MoE: each rank owns E/W experts and its own tokens. Every step,
prefill or decode, exchanges fixed-capacity slabs and never synchronises the host:

* ``dispatch_padded``: the (token, choice) pairs are counting-sorted by destination rank on the device
  (ops.ep_dispatch_plan), packed into W slabs of ``capacity`` rows (ops.ep_pack; padding rows carry the sentinel
  expert id ``e_local``, which the grouped GEMM skips) and exchanged with one equal-split all-to-all;
* ``local_experts_padded``: the owner runs its grouped GEMMs on the received rows;
* ``combine_padded``: the expert outputs go back with the reverse all-to-all and are reduced with the routing
  weights (+ residual) into the token order in one kernel (ops.ep_combine).

The capacity is the step's largest per-rank token count times top-k (agreed by the engine's EP lockstep), so no
pair is ever dropped. Decode steps (tens of tokens) move whole slabs - a few MB - and capture in one HIP graph.
Prefill steps (``exact_counts=True``) exchange the per-destination pair counts first, ON THE DEVICE (a 16-byte
peer-memory all-to-all), and the slab exchange then moves only each segment's valid rows over xGMI
(CustomAllReduce.all_to_all send_rows / recv_rows); rows past a peer's count are marked padding on the receiver.
So prefill moves the exact bytes of the old count-then-variable-split exchange without its host round trip
(round 4 copied the bincount of the destinations to the host: one device sync per MoE layer). Over
RCCL (slabs beyond the peer buffers, or no peer exchange) the equal-split ``all_to_all_single`` moves whole
slabs, also sync-free.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


def _host_plane(x: torch.Tensor, group) -> bool:
    """Device tensors over a gloo group (one-GPU multi-rank rehearsal): exchange through host memory."""
    return x.is_cuda and dist.get_backend(group) == "gloo"


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
    send_rows: Optional[torch.Tensor] = None  # [W] int32 valid rows sent to each peer (exact-count exchange)
    recv_rows: Optional[torch.Tensor] = None  # [W] int32 valid rows received from each peer


def exchange_counts(send_rows: torch.Tensor, group=None, xchg=None) -> torch.Tensor:
    """[W] int32 per-destination counts -> [W] counts received from each peer, without leaving the device: one
    16-byte-segment peer-memory all-to-all (or RCCL's equal-split all_to_all_single)."""
    W = send_rows.numel()
    if xchg is not None:
        buf = torch.zeros(W, 4, dtype=torch.int32, device=send_rows.device)
        buf[:, 0] = send_rows
        return xchg.all_to_all(buf)[:, 0].contiguous()
    return _a2a_equal(send_rows.contiguous(), group)


def dispatch_padded(x: torch.Tensor, ids: torch.Tensor, num_experts: int, capacity: int | None = None, group=None,
                    xchg=None, exact_counts: bool = False):
    """-> (rows [W*C, D], local expert ids [W*C] int32 (e_local = padding), plan). Sync-free, capturable.
    Pairs beyond ``capacity`` for one destination are dropped (capacity = T*k never drops). The plan is one
    counting-sort kernel over the destinations (ops.ep_dispatch_plan) and the slabs one gather kernel
    (ops.ep_pack); the rows and their expert ids travel in ONE exchange (ids packed as two bf16 lanes).
    exact_counts (prefill-sized steps on the peer-memory exchange): only the valid rows of each slab move."""
    from .. import ops

    world = dist.get_world_size(group)
    e_local = num_experts // world
    T, k = ids.shape
    C = T * k if capacity is None else capacity
    offs, pos, a_pairs = ops.ep_dispatch_plan(ids, world, e_local)
    send_n = recv_n = None
    if xchg is not None and x.is_cuda and x.dtype == torch.bfloat16:  # one exchange: the expert id rides in each
        # slab row's 16-B tail (two bf16 lanes)
        D = x.shape[1]
        slab, _ = ops.ep_pack(x, ids, offs, a_pairs, world, C, e_local, ids_in_rows=True)
        if exact_counts and xchg.eligible_a2a(slab):
            send_n = (offs[1:] - offs[:-1]).clamp(max=C).to(torch.int32)
            recv_n = exchange_counts(send_n, group, xchg)
            got = xchg.all_to_all(slab, send_rows=send_n, recv_rows=recv_n)
        else:
            got = _a2a_equal(slab, group, xchg)
        rows = got[:, :D].contiguous()
        eid = got[:, D:D + 2].contiguous().view(torch.int32).view(-1)
        if recv_n is not None:  # rows past a peer's count were never written: padding
            r = torch.arange(world * C, device=eid.device)
            eid = torch.where(r % C < recv_n.long()[r // C], eid, torch.full_like(eid, e_local))
    else:
        send, send_eid = ops.ep_pack(x, ids, offs, a_pairs, world, C, e_local)
        rows = _a2a_equal(send, group)
        eid = _a2a_equal(send_eid, group)
    return rows, eid, EPPaddedPlan(ids, pos, offs, C, e_local, send_n, recv_n)


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

    y = y.contiguous()
    if plan.send_rows is not None and xchg is not None and xchg.eligible_a2a(y):
        # only the rows this rank received go back (the peers read nothing else)
        back = xchg.all_to_all(y, send_rows=plan.recv_rows, recv_rows=plan.send_rows)
    else:
        back = _a2a_equal(y, group, xchg)
    return ops.ep_combine(back, plan.ids, plan.pos, plan.offs, weights, residual, plan.e_local, plan.capacity)
