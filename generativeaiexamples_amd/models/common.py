"""Shared model-side plumbing: the per-step ForwardBatch and weight initialisation helpers."""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import torch


@dataclass
class ForwardBatch:
    """Device-side description of one engine step (prefill tokens first, then decode tokens).

    Produced by the engine from the native scheduler's StepBatch.
    """
    token_ids: torch.Tensor          # [T] int32
    positions: torch.Tensor          # [T] int32
    slots: torch.Tensor              # [T] int32 (KV slot = block*16 + offset)
    num_prefill_tokens: int = 0
    # prefill part (varlen, chunked over cached prefixes)
    cu_q: Optional[torch.Tensor] = None            # [P+1] int32
    prefill_ctx: Optional[torch.Tensor] = None     # [P] int32
    prefill_block_tables: Optional[torch.Tensor] = None  # [P, maxb] int32
    prefill_tiles: Optional[torch.Tensor] = None   # attention tiles (host-built)
    prefill_qlen: List[int] = field(default_factory=list)
    prefill_ctx_host: List[int] = field(default_factory=list)  # host copy of prefill_ctx (state-slot models)
    # decode part
    decode_ctx: Optional[torch.Tensor] = None      # [Dn] int32
    decode_block_tables: Optional[torch.Tensor] = None  # [Dn, maxb] int32
    max_decode_ctx: int = 0
    # rows of the flat token dim whose logits are needed (in output order)
    sample_rows: Optional[torch.Tensor] = None     # [S] int64
    # host-side sequence ids of the rows (prefill sequences, then decode sequences) and model-specific
    # per-step inputs built by the model's prepare_batch hook (e.g. cross-attention tables)
    seq_ids: Optional[list] = None
    extra: Optional[dict] = None
    lora_slots: Optional[torch.Tensor] = None  # [T] int32 adapter slot per token (multi-LoRA), None = none
    # TP models: return this rank's vocab shard of the logits (no all-gather); the caller samples with
    # ops.sample_tp
    tp_local_logits: bool = False

    @property
    def num_tokens(self) -> int:
        return int(self.token_ids.shape[0])

    @property
    def num_decode(self) -> int:
        return self.num_tokens - self.num_prefill_tokens


def init_linear_(w: torch.Tensor, gen: torch.Generator, fan_in: int) -> torch.Tensor:
    """Deterministic scaled-normal init done in fp32 on the CPU generator, then cast (random-init weights)."""
    std = 1.0 / math.sqrt(fan_in)
    tmp = torch.empty(w.shape, dtype=torch.float32)
    tmp.normal_(0.0, std, generator=gen)
    w.copy_(tmp)
    return w


def randn_like_(w: torch.Tensor, seed: int, std: float) -> torch.Tensor:
    """Fast on-device random init (for multi-GB benchmark models)."""
    g = torch.Generator(device=w.device)
    g.manual_seed(seed)
    if w.is_floating_point():
        w.normal_(0.0, std, generator=g)
    return w


def quantize_linear_weights_fp8(w: dict, keys) -> int:
    """Replace the 2-D linear weights ``w[k]`` (k in keys) by per-output-channel e4m3fn
    :class:`~generativeaiexamples_amd.ops.Fp8Weight` in place; ops.linear then runs them on the fp8
    MFMA GEMM (BASELINE config 4). Returns the bytes saved."""
    from ..ops import Fp8Weight
    saved = 0
    for k in keys:
        t = w[k]
        if isinstance(t, Fp8Weight) or t.dim() != 2 or t.shape[1] % 128:
            continue
        w[k] = Fp8Weight.quantize(t)
        saved += t.numel() * (t.element_size() - 1)
        del t
    return saved


class PackedAttention:
    """Self- (or cross-) attention over a packed varlen batch for encoders (BERT/E5, CLIP, ViT).

    The paged flash-attention kernels read K/V from a paged cache, so an encoder forward allocates
    one *transient* cache for the whole batch (sequence b owns blocks [off_b, off_b + ceil(n_b/16)));
    every layer scatters its K/V into it with the RoPE/KV kernel (rotation off) and runs the
    bidirectional (or causal) prefill kernel. All index tensors are built once per forward.
    ``kv_lens`` (cross-attention) gives the key length per sequence when it differs from the query.
    """

    def __init__(self, q_lens: Sequence[int], num_heads: int, head_dim: int, device, dtype=torch.bfloat16,
                 causal: bool = False, num_kv_heads: Optional[int] = None, kv_lens: Optional[Sequence[int]] = None,
                 cos_sin: Optional[torch.Tensor] = None):
        from .. import ops
        self.H, self.Hkv, self.hd = num_heads, num_kv_heads or num_heads, head_dim
        self.causal, self.dtype, self.device = causal, dtype, torch.device(device)
        q_lens = [int(n) for n in q_lens]
        kv_lens = [int(n) for n in (kv_lens if kv_lens is not None else q_lens)]
        self.q_lens, self.kv_lens = q_lens, kv_lens
        self.T = sum(q_lens)
        B, BS = len(q_lens), ops.BLOCK
        nbs = [(n + BS - 1) // BS for n in kv_lens]
        offs = [0]
        for n in nbs:
            offs.append(offs[-1] + n)
        bt = torch.zeros(B, max(nbs + [1]), dtype=torch.int32)
        kv_slots = torch.empty(sum(kv_lens), dtype=torch.int32)
        t0 = 0
        for b, n in enumerate(kv_lens):
            bt[b, : nbs[b]] = torch.arange(offs[b], offs[b] + nbs[b], dtype=torch.int32)
            kv_slots[t0:t0 + n] = offs[b] * BS + torch.arange(n, dtype=torch.int32)
            t0 += n
        cu = [0]
        for n in q_lens:
            cu.append(cu[-1] + n)
        dev = self.device
        self.positions = torch.cat([torch.arange(n, dtype=torch.int32) for n in q_lens] or
                                   [torch.zeros(0, dtype=torch.int32)]).to(dev, non_blocking=True)
        self.block_tables = bt.to(dev, non_blocking=True)
        self.slots = kv_slots.to(dev, non_blocking=True)
        self.cu_q = torch.tensor(cu, dtype=torch.int32).to(dev, non_blocking=True)
        self.ctx = torch.tensor(kv_lens, dtype=torch.int32).to(dev, non_blocking=True)
        self.tiles = (ops.build_prefill_tiles(q_lens, self.H, self.Hkv, dev, head_dim=head_dim) if dev.type == "cuda"
                      else None)
        # self-attention without RoPE (BERT / E5 / CLIP / ViT encoders): every page's K / V^T image is packed straight
        # from the QKV rows by one kernel (ops.kv_pack) and the attention reads q from those rows - no q copy, no
        # per-(token, head) scatter
        self.pack = None
        if cos_sin is None and kv_lens == q_lens and dtype == torch.bfloat16:
            blk_tok, blk_n = [], []
            for b, n in enumerate(kv_lens):
                for i in range(nbs[b]):
                    blk_tok.append(cu[b] + BS * i)
                    blk_n.append(min(BS, n - BS * i))
            self.pack = (torch.tensor(blk_tok, dtype=torch.int32).to(dev, non_blocking=True),
                         torch.tensor(blk_n, dtype=torch.int32).to(dev, non_blocking=True))
        self.k_cache = torch.zeros(offs[-1] + 1, self.Hkv, BS, head_dim, device=dev, dtype=dtype)
        self.v_cache = torch.zeros(offs[-1] + 1, self.Hkv, head_dim, BS, device=dev, dtype=dtype)
        self.q = torch.empty(self.T, self.H, head_dim, device=dev, dtype=dtype)
        # RoPE table [max_pos, hd] (decoder-based encoders, e.g. the Mistral reranker) or none
        self.rope = cos_sin is not None
        self.cs = cos_sin if self.rope else torch.zeros(1, head_dim, dtype=torch.float32, device=dev)

    def __call__(self, qkv: torch.Tensor, scale: float, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """qkv [T, (H + 2 Hkv) * hd] -> attention output [T, H * hd]."""
        from .. import ops
        if self.pack is not None:
            ops.kv_pack(qkv, self.pack[0], self.pack[1], self.k_cache, self.v_cache, self.H, self.Hkv, self.hd)
            q = qkv.view(self.T, self.H + 2 * self.Hkv, self.hd)[:, : self.H]
        else:
            ops.rope_kv_write(qkv, self.positions, self.cs, self.slots, self.q, self.k_cache, self.v_cache, self.H,
                              self.Hkv, self.hd, rope=self.rope)
            q = self.q
        o = torch.empty_like(self.q) if out is None else out.view(self.T, self.H, self.hd)
        ops.attention_prefill(q, self.k_cache, self.v_cache, self.block_tables, self.cu_q, self.ctx, scale,
                              causal=self.causal, tiles=self.tiles, q_lens=self.q_lens, out=o)
        return o.view(self.T, self.H * self.hd)
