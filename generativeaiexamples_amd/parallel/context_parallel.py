"""Context parallelism: ring attention over a CP process group.

The reference has no long-context mechanism (it scales knowledge by retrieval + truncation, SURVEY
§5.7); this is the optional MI355X design for prompts beyond one GPU's comfort: the sequence is
sharded over ``cp`` ranks and the K/V shards rotate around a ring over xGMI point-to-point links
(each step moves one neighbour's shard over one link, overlapped with the attention of the shard
already held), so no rank ever materialises the full K/V.

Sharding is *zigzag* for causal attention: the sequence is cut into ``2 * cp`` equal chunks and
rank r holds chunks r and 2cp-1-r, so every rank has the same amount of causal work. For a
(query chunk a, key chunk b) pair: b < a attends fully, b == a is the causal diagonal, b > a is
skipped. Partial results carry their natural-log softmax normalisers (LSE) and are merged exactly:
``o = sum_i exp(lse_i - lse) o_i``, ``lse = logsumexp_i lse_i``.

Per-pair attention runs in the gfx950 flash-attention kernel (``attn_prefill``, which writes the
LSE) on GPU, and in the fp32 PyTorch reference on CPU (gloo test tier).
"""
from __future__ import annotations

import math
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist

from .. import ops


# ------------------------------------------------------------------------------------------------
# zigzag sharding
# ------------------------------------------------------------------------------------------------
def zigzag_chunks(rank: int, cp: int) -> Tuple[int, int]:
    return rank, 2 * cp - 1 - rank


def zigzag_shard(x: torch.Tensor, rank: int, cp: int, dim: int = 0) -> torch.Tensor:
    """This rank's two chunks of ``x`` (length divisible by 2*cp along ``dim``), concatenated."""
    parts = x.chunk(2 * cp, dim=dim)
    a, b = zigzag_chunks(rank, cp)
    return torch.cat([parts[a], parts[b]], dim=dim)


def zigzag_unshard(shards: List[torch.Tensor], dim: int = 0) -> torch.Tensor:
    """Inverse of zigzag_shard given every rank's shard in rank order."""
    cp = len(shards)
    chunks: List[Optional[torch.Tensor]] = [None] * (2 * cp)
    for r, s in enumerate(shards):
        a, b = zigzag_chunks(r, cp)
        chunks[a], chunks[b] = s.chunk(2, dim=dim)
    return torch.cat(chunks, dim=dim)  # type: ignore[arg-type]


def zigzag_positions(seq_len: int, rank: int, cp: int, device=None) -> torch.Tensor:
    """Absolute token positions of this rank's shard (for RoPE)."""
    return zigzag_shard(torch.arange(seq_len, device=device), rank, cp)


# ------------------------------------------------------------------------------------------------
# one (query block, key block) pair
# ------------------------------------------------------------------------------------------------
def _to_pages(k: torch.Tensor, v: torch.Tensor):
    """Contiguous K/V [T, Hkv, D] -> the paged cache layout of the kernels (16-token pages:
    K [n, Hkv, 16, D], V^T [n, Hkv, D, 16]) with an identity block table."""
    T, H, D = k.shape
    n = (T + 15) // 16
    if n * 16 != T:
        pad = n * 16 - T
        k = torch.cat([k, k.new_zeros(pad, H, D)])
        v = torch.cat([v, v.new_zeros(pad, H, D)])
    kp = k.view(n, 16, H, D).permute(0, 2, 1, 3).contiguous()
    vp = v.view(n, 16, H, D).permute(0, 2, 3, 1).contiguous()
    bt = torch.arange(n, dtype=torch.int32, device=k.device).view(1, n)
    return kp, vp, bt


def block_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, scale: float,
                    causal: bool) -> Tuple[torch.Tensor, torch.Tensor]:
    """q [Tq, Hq, D], k/v [Tk, Hkv, D] (GQA allowed) -> (out [Tq, Hq, D] in q.dtype, lse fp32 [Tq, Hq]).
    ``causal`` masks with the queries aligned to the END of the keys (diagonal block when Tq == Tk)."""
    Tq, Hq, _ = q.shape
    kp, vp, bt = _to_pages(k, v)
    dev = q.device
    cu = torch.tensor([0, Tq], dtype=torch.int32, device=dev)
    ctx = torch.tensor([k.shape[0]], dtype=torch.int32, device=dev)
    lse = torch.empty(Tq, Hq, dtype=torch.float32, device=dev)
    out = ops.attention_prefill(q.contiguous(), kp, vp, bt, cu, ctx, scale, causal, q_lens=[Tq], lse=lse)
    return out, lse


def merge_partial(o_acc: Optional[torch.Tensor], lse_acc: Optional[torch.Tensor], o: torch.Tensor,
                  lse: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Exact merge of two softmax-attention partials over disjoint key sets (fp32 accumulator)."""
    o = o.float()
    if o_acc is None:
        return o, lse
    new = torch.logaddexp(lse_acc, lse)
    a = torch.exp(lse_acc - new).unsqueeze(-1)
    b = torch.exp(lse - new).unsqueeze(-1)
    return o_acc * a + o * b, new


# ------------------------------------------------------------------------------------------------
# ring
# ------------------------------------------------------------------------------------------------
class _Ring:
    """Send the held K/V shard to rank+1 and receive rank-1's, asynchronously (RCCL P2P over one
    xGMI link; gloo on the CPU tier, staging CUDA tensors through host memory)."""

    def __init__(self, group):
        self.group = group
        self.cp = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.cpu_stage = dist.get_backend(group) == "gloo"
        g = (lambda r: dist.get_global_rank(group, r)) if group is not None else (lambda r: r)
        self.nxt, self.prv = g((self.rank + 1) % self.cp), g((self.rank - 1) % self.cp)

    def start(self, t: torch.Tensor):
        src = t.cpu() if (self.cpu_stage and t.is_cuda) else t
        recv = torch.empty_like(src)
        # even ranks send first, odd ranks receive first: no cycle of blocking sends on gloo
        ops_ = [dist.P2POp(dist.isend, src, self.nxt, self.group), dist.P2POp(dist.irecv, recv, self.prv, self.group)]
        if self.rank % 2:
            ops_.reverse()
        reqs = dist.batch_isend_irecv(ops_)
        return reqs, recv, t.device

    @staticmethod
    def finish(handle) -> torch.Tensor:
        reqs, recv, dev = handle
        for r in reqs:
            r.wait()
        return recv.to(dev)


def ring_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, group=None, scale: Optional[float] = None,
                   causal: bool = True) -> torch.Tensor:
    """Attention of this rank's zigzag query shard against the whole (sharded) sequence.

    q [2c, Hq, D], k/v [2c, Hkv, D]: this rank's two zigzag chunks (``zigzag_shard``) of a sequence of
    length ``2 * cp * c``. Returns out [2c, Hq, D] (q.dtype) for the same rows. ``causal=False`` is
    bidirectional (encoders). One ring pass of ``cp - 1`` K/V transfers, each overlapped with the
    attention of the shard already held.
    """
    cp = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    scale = scale if scale is not None else 1.0 / math.sqrt(q.shape[-1])
    c = q.shape[0] // 2
    assert q.shape[0] == 2 * c and k.shape[0] == 2 * c, "zigzag shards hold two equal chunks"
    qa = zigzag_chunks(rank, cp)
    q_parts = (q[:c], q[c:])
    acc: List[Tuple[Optional[torch.Tensor], Optional[torch.Tensor]]] = [(None, None), (None, None)]
    kv = torch.stack([k, v])
    ring = _Ring(group) if cp > 1 else None
    for step in range(cp):
        handle = ring.start(kv) if ring is not None and step < cp - 1 else None
        src = (rank - step) % cp
        kb = zigzag_chunks(src, cp)
        for i, a in enumerate(qa):
            for j, b in enumerate(kb):
                if causal and b > a:
                    continue
                kk, vv = kv[0, j * c:(j + 1) * c], kv[1, j * c:(j + 1) * c]
                o, l = block_attention(q_parts[i], kk, vv, scale, causal=causal and a == b)
                acc[i] = merge_partial(acc[i][0], acc[i][1], o, l)
        if handle is not None:
            kv = _Ring.finish(handle)
    return torch.cat([acc[0][0], acc[1][0]]).to(q.dtype)  # type: ignore[list-item]
