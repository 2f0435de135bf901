"""OPT decoder (BASELINE config 1, the CPU plumbing generator: OPT-125m; SURVEY S12 HF local LLM).

Learned absolute positions (offset 2), pre-LayerNorm blocks with biases, ReLU MLP, tied LM head.
Runs through the same paged-KV engine as Llama: the RoPE/KV kernel with rotation disabled writes
K/V, attention is the same paged flash kernels, GEMMs use the bias / bias+ReLU / bias+residual
fused epilogues.
"""
from __future__ import annotations

import json
import math
import os
from dataclasses import dataclass
from typing import Dict

import torch

from .. import ops
from ..parallel.dist import DistContext, get_context
from .common import ForwardBatch, randn_like_


@dataclass
class OPTConfig:
    vocab_size: int = 50272
    hidden_size: int = 768
    intermediate_size: int = 3072
    num_layers: int = 12
    num_heads: int = 12
    max_position: int = 2048
    ln_eps: float = 1e-5
    bos_token_id: int = 2
    eos_token_ids: tuple = (2,)
    name: str = "facebook/opt-125m"

    @property
    def head_dim(self) -> int:
        return self.hidden_size // self.num_heads

    @property
    def num_kv_heads(self) -> int:
        return self.num_heads

    @staticmethod
    def opt_125m(**kw):
        return OPTConfig(**kw)

    @staticmethod
    def from_hf(path: str) -> "OPTConfig":
        with open(os.path.join(path, "config.json")) as f:
            c = json.load(f)
        return OPTConfig(vocab_size=c["vocab_size"], hidden_size=c["hidden_size"], intermediate_size=c["ffn_dim"],
                         num_layers=c["num_hidden_layers"], num_heads=c["num_attention_heads"],
                         max_position=c.get("max_position_embeddings", 2048), name=os.path.basename(path.rstrip("/")))


class OPTModel:
    def __init__(self, cfg: OPTConfig, device=None, dtype=torch.bfloat16, dist_ctx: DistContext | None = None):
        self.cfg, self.ctx = cfg, dist_ctx or get_context()
        assert self.ctx.tp_size == 1, "OPT plumbing model is TP=1"
        self.device = torch.device(device) if device is not None else self.ctx.device
        self.dtype = dtype
        self.hq = self.hkv = cfg.num_heads
        self.scale = 1.0 / math.sqrt(cfg.head_dim)
        D, F, V = cfg.hidden_size, cfg.intermediate_size, cfg.vocab_size
        e = lambda *s: torch.empty(*s, device=self.device, dtype=dtype)  # noqa: E731
        self.w: Dict[str, torch.Tensor] = {"embed": e(V, D), "pos": e(cfg.max_position + 2, D),
                                           "final_ln_w": e(D), "final_ln_b": e(D)}
        for i in range(cfg.num_layers):
            p = f"l{i}."
            for n, s in (("ln1_w", (D,)), ("ln1_b", (D,)), ("qkv", (3 * D, D)), ("qkv_b", (3 * D,)), ("o", (D, D)),
                         ("o_b", (D,)), ("ln2_w", (D,)), ("ln2_b", (D,)), ("fc1", (F, D)), ("fc1_b", (F,)),
                         ("fc2", (D, F)), ("fc2_b", (D,))):
                self.w[p + n] = e(*s)
        self._cs = torch.zeros(1, cfg.head_dim, dtype=torch.float32, device=self.device)

    def random_init(self, seed: int = 0):
        s = seed * 1000
        for k, t in self.w.items():
            if k.endswith("_w") and "ln" in k:
                t.fill_(1.0)
            elif k.endswith("_b"):
                t.zero_()
            elif k in ("embed", "pos"):
                randn_like_(t, s, 0.02)
            else:
                randn_like_(t, s, 1.0 / math.sqrt(t.shape[1]))
            s += 1
        return self

    def load_hf_state(self, sd):
        c = self.cfg
        pre = "model.decoder."

        def put(n, t):
            self.w[n].copy_(t.to(self.dtype))

        put("embed", sd[pre + "embed_tokens.weight"])
        put("pos", sd[pre + "embed_positions.weight"])
        put("final_ln_w", sd[pre + "final_layer_norm.weight"])
        put("final_ln_b", sd[pre + "final_layer_norm.bias"])
        for i in range(c.num_layers):
            p, h = f"l{i}.", f"{pre}layers.{i}."
            put(p + "ln1_w", sd[h + "self_attn_layer_norm.weight"])
            put(p + "ln1_b", sd[h + "self_attn_layer_norm.bias"])
            put(p + "qkv", torch.cat([sd[h + f"self_attn.{n}_proj.weight"] for n in "qkv"]))
            put(p + "qkv_b", torch.cat([sd[h + f"self_attn.{n}_proj.bias"] for n in "qkv"]))
            put(p + "o", sd[h + "self_attn.out_proj.weight"])
            put(p + "o_b", sd[h + "self_attn.out_proj.bias"])
            put(p + "ln2_w", sd[h + "final_layer_norm.weight"])
            put(p + "ln2_b", sd[h + "final_layer_norm.bias"])
            put(p + "fc1", sd[h + "fc1.weight"])
            put(p + "fc1_b", sd[h + "fc1.bias"])
            put(p + "fc2", sd[h + "fc2.weight"])
            put(p + "fc2_b", sd[h + "fc2.bias"])
        return self

    def num_params(self) -> int:
        return sum(t.numel() for t in self.w.values())

    def forward(self, fb: ForwardBatch, kv, decode_ws=None) -> torch.Tensor:
        c, w = self.cfg, self.w
        T, P, hd = fb.num_tokens, fb.num_prefill_tokens, c.head_dim
        h = ops.embedding(fb.token_ids, w["embed"])
        h = h + w["pos"][(fb.positions + 2).long()]
        q = torch.empty(T, self.hq, hd, device=h.device, dtype=self.dtype)
        attn = torch.empty_like(q)
        for i in range(c.num_layers):
            p = f"l{i}."
            x = ops.layer_norm(h, w[p + "ln1_w"], w[p + "ln1_b"], c.ln_eps)
            qkv = ops.linear(x, w[p + "qkv"], bias=w[p + "qkv_b"])
            kc, vc = kv.layer(i)
            ops.rope_kv_write(qkv, fb.positions, self._cs, fb.slots, q, kc, vc, self.hq, self.hkv, hd, rope=False)
            if P > 0:
                ops.attention_prefill(q[:P], kc, vc, fb.prefill_block_tables, fb.cu_q, fb.prefill_ctx, self.scale,
                                      True, tiles=fb.prefill_tiles, q_lens=fb.prefill_qlen, out=attn[:P])
            if T > P:
                ops.attention_decode(q[P:], kc, vc, fb.decode_block_tables, fb.decode_ctx, self.scale, ws=decode_ws,
                                     max_ctx=fb.max_decode_ctx, out=attn[P:])
            h = ops.linear(attn.view(T, -1), w[p + "o"], bias=w[p + "o_b"], residual=h)
            x = ops.layer_norm(h, w[p + "ln2_w"], w[p + "ln2_b"], c.ln_eps)
            f = ops.linear(x, w[p + "fc1"], bias=w[p + "fc1_b"], act="relu")
            h = ops.linear(f, w[p + "fc2"], bias=w[p + "fc2_b"], residual=h)
        if fb.sample_rows is not None:
            h = h.index_select(0, fb.sample_rows)
        x = ops.layer_norm(h, w["final_ln_w"], w["final_ln_b"], c.ln_eps)
        return ops.linear(x, w["embed"], out_dtype=torch.float32)
