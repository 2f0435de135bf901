"""Differentiable forward of a :class:`~..models.llama.LlamaModel` (frozen bf16 base + LoRA) for SFT.

Same math and weight layout as the inference path (fused QKV with RoPE, GQA, interleaved gate/up
SwiGLU, residual stream), expressed with autograd ops: RMSNorm in fp32, hipBLASLt GEMMs, PyTorch
SDPA for causal attention. Tensor parallel follows the inference sharding (column-parallel QKV /
gate-up, row-parallel O / down, vocab-parallel LM head) with the autograd-aware collectives of
:mod:`.tp`. Loss: token cross-entropy on the response tokens only (mask), mean over those tokens.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .. import ops
from .lora import LoRAAdapter
from .tp import copy_to_tp, gather_last, reduce_from_tp


def _rms(x, g, eps):
    xf = x.float()
    return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * g.float()).to(x.dtype)


def _norm(model, x, name):
    c, w = model.cfg, model.w
    if c.norm == "layernorm":
        return F.layer_norm(x.float(), (x.shape[-1],), w[name].float(), w[name + "_b"].float(), c.rms_eps).to(x.dtype)
    return _rms(x, w[name], c.rms_eps)


def _lin(x, w, lora: LoRAAdapter | None, layer: int, target: str, bias=None):
    # a frozen base weight may be stored in the fragment-ordered inference layout (an engine serves the same model):
    # read its row-major values (FullTrainer, which updates the weights, refuses such models)
    y = x @ ops.natural_weight(w).t()
    if bias is not None:
        y = y + bias
    if lora is not None:
        a = lora.params.get(f"l{layer}.{target}.A")
        if a is not None:
            b = lora.params[f"l{layer}.{target}.B"]
            xa = x.float()
            if lora.cfg.dropout > 0:
                xa = F.dropout(xa, lora.cfg.dropout, training=True)
            y = y + ((xa @ a.t()) @ b.t() * lora.cfg.scale).to(y.dtype)
    return y


def lm_loss(model, lora: LoRAAdapter | None, ids: torch.Tensor, labels: torch.Tensor,
            checkpoint: bool = False) -> torch.Tensor:
    """ids / labels [B, S] (labels = -100 where not trained). Returns the mean token loss."""
    c, w, ctx = model.cfg, model.w, model.ctx
    B, S = ids.shape
    hd, hq, hkv = c.head_dim, model.hq, model.hkv
    # vocab-parallel embedding: rows outside the local shard are zero, then summed over TP
    local = ids - model.vstart
    inside = (local >= 0) & (local < model.vocab_local)
    x = F.embedding(local.clamp(0, model.vocab_local - 1), w["embed"]) * inside[..., None].to(w["embed"].dtype)
    x = reduce_from_tp(x, ctx)
    if c.embed_scale:
        x = x * model.embed_multiplier
    cs = model.cos_sin[:S].to(x.device)
    rank0 = ctx.tp_rank == 0
    cos, sin = cs[:, : hd // 2], cs[:, hd // 2:]

    def rope(t):  # [B, S, h, hd]
        a, b = t[..., : hd // 2].float(), t[..., hd // 2:].float()
        cc, ss = cos[None, :, None], sin[None, :, None]
        return torch.cat([a * cc - b * ss, b * cc + a * ss], -1).to(t.dtype)

    def block(x, i):
        p = f"l{i}."
        h = copy_to_tp(_norm(model, x, p + "attn_norm"), ctx)
        qkv = _lin(h, w[p + "qkv"], lora, i, "qkv", w.get(p + "qkv_b"))
        q, k, v = qkv.split([hq * hd, hkv * hd, hkv * hd], -1)
        q, k = q.view(B, S, hq, hd), k.view(B, S, hkv, hd)
        if c.qk_norm:
            q, k = _rms(q, w[p + "q_norm"], c.rms_eps), _rms(k, w[p + "k_norm"], c.rms_eps)
        q, k = rope(q), rope(k)
        v = v.view(B, S, hkv, hd)
        a = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2),
                                           is_causal=True, enable_gqa=hq != hkv)
        o = _lin(a.transpose(1, 2).reshape(B, S, hq * hd), w[p + "o"], lora, i, "o",
                 w.get(p + "o_b") if rank0 else None)
        x = x + reduce_from_tp(o, ctx)
        h = copy_to_tp(_norm(model, x, p + "mlp_norm"), ctx)
        if c.mlp == "gelu_tanh":
            m = F.gelu(_lin(h, w[p + "fc"], lora, i, "fc", w.get(p + "fc_b")).float(), approximate="tanh").to(x.dtype)
        else:
            gu = _lin(h, w[p + "gate_up"], lora, i, "gate_up")
            gu = gu.view(B, S, -1, 2, 16)
            g = F.silu(gu[..., 0, :].float()) if c.mlp == "swiglu" else F.gelu(gu[..., 0, :].float(), approximate="tanh")
            m = (g * gu[..., 1, :].float()).to(x.dtype).reshape(B, S, -1)
        return x + reduce_from_tp(_lin(m, w[p + "down"], lora, i, "down", w.get(p + "down_b") if rank0 else None), ctx)

    for i in range(c.num_layers):
        if checkpoint:
            x = torch.utils.checkpoint.checkpoint(block, x, i, use_reentrant=False)
        else:
            x = block(x, i)
    h = copy_to_tp(_norm(model, x, "norm"), ctx)
    logits = gather_last(h @ ops.natural_weight(w["lm_head"]).t(), ctx)[..., : c.vocab_size].float()
    if not bool((labels[:, 1:] != -100).any()):  # nothing to learn in this micro-batch
        return logits.sum() * 0.0
    return F.cross_entropy(logits[:, :-1].reshape(-1, logits.shape[-1]), labels[:, 1:].reshape(-1), ignore_index=-100)
