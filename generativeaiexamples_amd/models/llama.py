"""Llama-3 family decoder (Llama-3-8B / 70B / 3.1 / 3.2 text, Mistral-style GQA) on the gfx950 kernels.

Replaces the reference's NIM-LLM container (``nvcr.io/nim/meta/llama3-8b-instruct``,
API default ``meta/llama3-70b-instruct``, RAG/examples/local_deploy/docker-compose-nim-ms.yaml:2-28).

Per layer, 7 launches: RMSNorm -> QKV GEMM -> fused RoPE + paged-KV write -> attention
(prefill tokens: paged flash-attention; decode tokens: split-KV flash-decoding) -> O-proj GEMM
with the residual add fused in its epilogue -> RMSNorm -> gate/up GEMM with SwiGLU fused in its
epilogue (interleaved weights) -> down GEMM with fused residual add.

Tensor parallel: QKV and gate/up are column-parallel (heads / intermediate split),
O and down are row-parallel followed by one all-reduce each (the residual is added on TP rank 0
only, so it is counted once), embedding and LM head are vocab-parallel (all-gather of logits).
"""
from __future__ import annotations

import json
import math
import os
from dataclasses import asdict, dataclass
from typing import Dict, Optional

import torch

from .. import ops
from ..parallel.dist import DistContext, get_context
from .common import ForwardBatch, randn_like_


@dataclass
class LlamaConfig:
    vocab_size: int = 128256
    hidden_size: int = 4096
    intermediate_size: int = 14336
    num_layers: int = 32
    num_heads: int = 32
    num_kv_heads: int = 8
    head_dim: int = 128
    rope_theta: float = 500000.0
    rope_scaling: Optional[dict] = None
    rms_eps: float = 1e-5
    max_position: int = 8192
    tie_embeddings: bool = False
    bos_token_id: int = 128000
    eos_token_ids: tuple = (128001, 128009)
    name: str = "llama"

    @staticmethod
    def llama3_8b(**kw):
        return LlamaConfig(name="meta/llama3-8b-instruct", **kw)

    @staticmethod
    def llama3_70b(**kw):
        return LlamaConfig(name="meta/llama3-70b-instruct", hidden_size=8192, intermediate_size=28672,
                           num_layers=80, num_heads=64, num_kv_heads=8, **kw)

    @staticmethod
    def llama31_8b(**kw):
        return LlamaConfig(name="meta/llama-3.1-8b-instruct", max_position=131072,
                           rope_scaling={"factor": 8.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
                                         "original_max_position_embeddings": 8192}, **kw)

    @staticmethod
    def mistral_7b(**kw):
        return LlamaConfig(name="mistralai/mistral-7b-instruct", vocab_size=32768, rope_theta=1e6,
                           max_position=32768, bos_token_id=1, eos_token_ids=(2,), **kw)

    @staticmethod
    def tiny(**kw):
        base = dict(vocab_size=512, hidden_size=256, intermediate_size=512, num_layers=2, num_heads=4,
                    num_kv_heads=2, head_dim=64, max_position=2048, bos_token_id=1, eos_token_ids=(2,),
                    name="tiny-llama")
        base.update(kw)
        return LlamaConfig(**base)

    @staticmethod
    def from_hf(path: str) -> "LlamaConfig":
        with open(os.path.join(path, "config.json")) as f:
            c = json.load(f)
        eos = c.get("eos_token_id", 2)
        return LlamaConfig(
            vocab_size=c["vocab_size"], hidden_size=c["hidden_size"], intermediate_size=c["intermediate_size"],
            num_layers=c["num_hidden_layers"], num_heads=c["num_attention_heads"],
            num_kv_heads=c.get("num_key_value_heads", c["num_attention_heads"]),
            head_dim=c.get("head_dim") or c["hidden_size"] // c["num_attention_heads"],
            rope_theta=c.get("rope_theta", 10000.0), rope_scaling=c.get("rope_scaling"),
            rms_eps=c.get("rms_norm_eps", 1e-5), max_position=c.get("max_position_embeddings", 8192),
            tie_embeddings=c.get("tie_word_embeddings", False), bos_token_id=c.get("bos_token_id", 1),
            eos_token_ids=tuple(eos) if isinstance(eos, list) else (eos,), name=os.path.basename(path.rstrip("/")))


class LlamaModel:
    """Weights + forward. Weights are plain tensors (no nn.Module): the engine owns execution."""

    def __init__(self, cfg: LlamaConfig, device=None, dtype=torch.bfloat16, dist_ctx: DistContext | None = None):
        self.cfg = cfg
        self.ctx = dist_ctx or get_context()
        self.device = torch.device(device) if device is not None else self.ctx.device
        self.dtype = dtype
        tp = self.ctx.tp_size
        assert cfg.num_heads % tp == 0 and cfg.num_kv_heads % tp == 0 and cfg.intermediate_size % (16 * tp) == 0
        self.hq = cfg.num_heads // tp
        self.hkv = cfg.num_kv_heads // tp
        self.inter = cfg.intermediate_size // tp
        self.vocab_local = (cfg.vocab_size + tp - 1) // tp
        self.vstart = self.ctx.tp_rank * self.vocab_local
        self.scale = 1.0 / math.sqrt(cfg.head_dim)
        self.w: Dict[str, torch.Tensor] = {}
        self.lora_names: list = []          # slot s (1-based) -> adapter name; slot 0 = base model
        self.lora_w: Dict[tuple, tuple] = {}  # (slot, layer, target) -> (A [r, in] bf16, B [out, r] bf16, scale)
        self.cos_sin = ops.rope_cos_sin(cfg.max_position, cfg.head_dim, cfg.rope_theta, cfg.rope_scaling,
                                        device=self.device)
        self._alloc()

    # ------------------------------------------------------------------ weights
    def _alloc(self):
        c, d, dt = self.cfg, self.device, self.dtype
        D, hd = c.hidden_size, c.head_dim
        e = lambda *s: torch.empty(*s, device=d, dtype=dt)  # noqa: E731
        self.w["embed"] = e(self.vocab_local, D)
        for i in range(c.num_layers):
            p = f"l{i}."
            self.w[p + "attn_norm"] = e(D)
            self.w[p + "qkv"] = e((self.hq + 2 * self.hkv) * hd, D)
            self.w[p + "o"] = e(D, self.hq * hd)
            self.w[p + "mlp_norm"] = e(D)
            self.w[p + "gate_up"] = e(2 * self.inter, D)  # interleaved per 16 rows
            self.w[p + "down"] = e(D, self.inter)
        self.w["norm"] = e(D)
        self.w["lm_head"] = self.w["embed"] if c.tie_embeddings else e(self.vocab_local, D)

    def random_init(self, seed: int = 0):
        """Random-init weights of the real architecture (benchmarks have no checkpoints offline)."""
        c = self.cfg
        s = seed * 1000 + self.ctx.tp_rank
        for k, t in self.w.items():
            if k.endswith("norm"):
                t.fill_(1.0)
            elif k == "lm_head" and c.tie_embeddings:
                continue
            else:
                fan_in = t.shape[1]
                randn_like_(t, s, 1.0 / math.sqrt(fan_in) if k not in ("embed",) else 0.02)
            s += 1
        return self

    def load_hf_state(self, sd: Dict[str, torch.Tensor]):
        """Load a HF Llama state dict (full weights; each TP rank keeps its shard)."""
        c, tp, r = self.cfg, self.ctx.tp_size, self.ctx.tp_rank
        hd = c.head_dim

        def shard_rows(t, n):  # column-parallel (output dim)
            return t.reshape(tp, n // tp, *t.shape[1:])[r] if tp > 1 else t

        def put(name, t):
            self.w[name].copy_(t.to(self.dtype))

        emb = sd["model.embed_tokens.weight"]
        pad = self.vocab_local * tp - emb.shape[0]
        if pad:
            emb = torch.cat([emb, emb.new_zeros(pad, emb.shape[1])])
        put("embed", shard_rows(emb, emb.shape[0]))
        for i in range(c.num_layers):
            p, h = f"l{i}.", f"model.layers.{i}."
            put(p + "attn_norm", sd[h + "input_layernorm.weight"])
            put(p + "mlp_norm", sd[h + "post_attention_layernorm.weight"])
            q = shard_rows(sd[h + "self_attn.q_proj.weight"], c.num_heads * hd)
            k = shard_rows(sd[h + "self_attn.k_proj.weight"], c.num_kv_heads * hd)
            v = shard_rows(sd[h + "self_attn.v_proj.weight"], c.num_kv_heads * hd)
            put(p + "qkv", torch.cat([q, k, v]))
            o = sd[h + "self_attn.o_proj.weight"]
            put(p + "o", o.reshape(o.shape[0], tp, -1)[:, r] if tp > 1 else o)
            self._load_mlp(sd, i)
        put("norm", sd["model.norm.weight"])
        if not c.tie_embeddings:
            lm = sd["lm_head.weight"]
            if pad:
                lm = torch.cat([lm, lm.new_zeros(pad, lm.shape[1])])
            put("lm_head", shard_rows(lm, lm.shape[0]))
        return self

    def _load_mlp(self, sd: Dict[str, torch.Tensor], i: int):
        c, tp, r = self.cfg, self.ctx.tp_size, self.ctx.tp_rank
        p, h = f"l{i}.", f"model.layers.{i}."

        def shard_rows(t, n):
            return t.reshape(tp, n // tp, *t.shape[1:])[r] if tp > 1 else t

        g = shard_rows(sd[h + "mlp.gate_proj.weight"], c.intermediate_size)
        u = shard_rows(sd[h + "mlp.up_proj.weight"], c.intermediate_size)
        self.w[p + "gate_up"].copy_(ops.interleave_gate_up(g, u).to(self.dtype))
        dn = sd[h + "mlp.down_proj.weight"]
        self.w[p + "down"].copy_((dn.reshape(dn.shape[0], tp, -1)[:, r] if tp > 1 else dn).to(self.dtype))

    def export_hf_state(self) -> Dict[str, torch.Tensor]:
        """Inverse of load_hf_state for a TP=1 model (checkpoint export, TP-reshard tests)."""
        assert self.ctx.tp_size == 1
        c, hd, w = self.cfg, self.cfg.head_dim, self.w
        sd = {"model.embed_tokens.weight": w["embed"].clone(), "model.norm.weight": w["norm"].clone()}
        if not c.tie_embeddings:
            sd["lm_head.weight"] = w["lm_head"].clone()
        nq, nk = c.num_heads * hd, c.num_kv_heads * hd
        for i in range(c.num_layers):
            p, h = f"l{i}.", f"model.layers.{i}."
            qkv = w[p + "qkv"]
            sd[h + "self_attn.q_proj.weight"] = qkv[:nq].clone()
            sd[h + "self_attn.k_proj.weight"] = qkv[nq:nq + nk].clone()
            sd[h + "self_attn.v_proj.weight"] = qkv[nq + nk:].clone()
            sd[h + "self_attn.o_proj.weight"] = w[p + "o"].clone()
            gu = w[p + "gate_up"].reshape(-1, 2, 16, c.hidden_size)
            sd[h + "mlp.gate_proj.weight"] = gu[:, 0].reshape(-1, c.hidden_size).clone()
            sd[h + "mlp.up_proj.weight"] = gu[:, 1].reshape(-1, c.hidden_size).clone()
            sd[h + "mlp.down_proj.weight"] = w[p + "down"].clone()
            sd[h + "input_layernorm.weight"] = w[p + "attn_norm"].clone()
            sd[h + "post_attention_layernorm.weight"] = w[p + "mlp_norm"].clone()
        return sd

    def load_safetensors_dir(self, path: str):
        from safetensors.torch import load_file

        sd = {}
        for f in sorted(os.listdir(path)):
            if f.endswith(".safetensors"):
                sd.update(load_file(os.path.join(path, f)))
        return self.load_hf_state(sd)

    def num_params(self) -> int:
        seen, n = set(), 0
        for t in self.w.values():
            if t.data_ptr() not in seen:
                seen.add(t.data_ptr())
                n += t.numel()
        return n

    # ------------------------------------------------------------------ multi-LoRA serving
    def add_lora(self, name: str, adapter) -> int:
        """Register a trained :class:`~..training.lora.LoRAAdapter` (or a path to one) under ``name``;
        requests select it per sequence (``lora`` argument / the OpenAI ``model`` field). Adapters are
        applied unmerged: y += mask_slot * ((x A^T) B^T) * scale for every adapted projection, so
        requests for different adapters (and the base model) share one batch and one HIP graph."""
        if isinstance(adapter, str):
            from ..training.lora import LoRAAdapter
            adapter = LoRAAdapter.load(adapter, self, device=self.device)
        if name in self.lora_names:
            slot = self.lora_names.index(name) + 1
        else:
            self.lora_names.append(name)
            slot = len(self.lora_names)
        for key, a in adapter.params.items():
            if not key.endswith(".A"):
                continue
            base = key[:-2]
            li, t = base.split(".", 1)
            b = adapter.params[base + ".B"]
            self.lora_w[(slot, int(li[1:]), t)] = (a.detach().to(self.device, self.dtype).contiguous(),
                                                   b.detach().to(self.device, self.dtype).contiguous(),
                                                   float(adapter.cfg.scale))
        return slot

    def lora_slot(self, name: Optional[str]) -> int:
        if not name:
            return 0
        if name not in self.lora_names:
            raise KeyError(f"unknown LoRA adapter '{name}'")
        return self.lora_names.index(name) + 1

    def _lora(self, y: torch.Tensor, x: torch.Tensor, layer: int, target: str, fb: ForwardBatch) -> torch.Tensor:
        slots = getattr(fb, "lora_slots", None)
        if not self.lora_names or slots is None:
            return y
        for s in range(1, len(self.lora_names) + 1):
            ab = self.lora_w.get((s, layer, target))
            if ab is None:
                continue
            a, b, scale = ab
            m = (slots == s).to(x.dtype)[:, None]
            y += ((x * m) @ a.t() @ b.t()) * scale
        return y

    # ------------------------------------------------------------------ forward
    def kv_shape(self, num_blocks: int):
        return (num_blocks, self.hkv, ops.BLOCK, self.cfg.head_dim), (num_blocks, self.hkv, self.cfg.head_dim, ops.BLOCK)

    def forward(self, fb: ForwardBatch, kv, decode_ws=None) -> torch.Tensor:
        """Returns fp32 logits [len(sample_rows), vocab] (gathered over TP)."""
        c, w, ctx = self.cfg, self.w, self.ctx
        T, P = fb.num_tokens, fb.num_prefill_tokens
        hd = c.head_dim
        # residual stream `res` is updated in place by the fused add+RMSNorm kernel, so the O and down
        # projections are plain GEMMs (row-parallel partial sums all-reduced before the add)
        res = ops.embedding(fb.token_ids, w["embed"], self.vstart, self.vstart + self.vocab_local)
        ctx.tp_all_reduce(res)
        q = torch.empty(T, self.hq, hd, device=res.device, dtype=self.dtype)
        attn = torch.empty_like(q)
        h = None
        for i in range(c.num_layers):
            p = f"l{i}."
            x = ops.rms_norm(res, w[p + "attn_norm"], c.rms_eps) if h is None else \
                ops.rms_norm(h, w[p + "attn_norm"], c.rms_eps, residual=res)
            qkv = self._lora(ops.linear(x, w[p + "qkv"]), x, i, "qkv", fb)
            kc, vc = kv.layer(i)
            ops.rope_kv_write(qkv, fb.positions, self.cos_sin, fb.slots, q, kc, vc, self.hq, self.hkv, hd, True)
            if P > 0:
                ops.attention_prefill(q[:P], kc, vc, fb.prefill_block_tables, fb.cu_q, fb.prefill_ctx, self.scale,
                                      True, tiles=fb.prefill_tiles, q_lens=fb.prefill_qlen, out=attn[:P])
            if T > P:
                ops.attention_decode(q[P:], kc, vc, fb.decode_block_tables, fb.decode_ctx, self.scale, ws=decode_ws,
                                     max_ctx=fb.max_decode_ctx, out=attn[P:])
            h = self._lora(ops.linear(attn.view(T, -1), w[p + "o"]), attn.view(T, -1), i, "o", fb)
            ctx.tp_all_reduce(h)
            x = ops.rms_norm(h, w[p + "mlp_norm"], c.rms_eps, residual=res)
            g = ops.linear(x, w[p + "gate_up"], act="swiglu")
            h = ops.linear(g, w[p + "down"])
            ctx.tp_all_reduce(h)
        if fb.sample_rows is not None:
            h = h.index_select(0, fb.sample_rows)
            res = res.index_select(0, fb.sample_rows)
        x = ops.rms_norm(h, w["norm"], c.rms_eps, residual=res)
        logits = ops.linear(x, w["lm_head"], out_dtype=torch.float32)
        logits = ctx.tp_all_gather_last(logits)
        return logits[:, : c.vocab_size]

    # ------------------------------------------------------------------ reference
    @torch.no_grad()
    def reference_forward(self, token_ids: torch.Tensor) -> torch.Tensor:
        """Dense full-sequence fp32 forward with no cache (test oracle; TP=1 only)."""
        c, w = self.cfg, {k: v.float().cpu() for k, v in self.w.items()}
        T = token_ids.numel()
        hd = c.head_dim
        h = w["embed"][token_ids.long().cpu()]
        cs = self.cos_sin.cpu()[:T]
        cos, sin = cs[:, None, : hd // 2], cs[:, None, hd // 2:]

        def rope(t):
            a, b = t[..., : hd // 2], t[..., hd // 2:]
            return torch.cat([a * cos - b * sin, b * cos + a * sin], -1)

        def rms(x, g):
            return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + c.rms_eps) * g

        for i in range(c.num_layers):
            p = f"l{i}."
            x = rms(h, w[p + "attn_norm"])
            qkv = (x @ w[p + "qkv"].t()).view(T, self.hq + 2 * self.hkv, hd)
            q, k, v = qkv[:, : self.hq], qkv[:, self.hq: self.hq + self.hkv], qkv[:, self.hq + self.hkv:]
            q, k = rope(q), rope(k)
            rep = self.hq // self.hkv
            k, v = k.repeat_interleave(rep, 1), v.repeat_interleave(rep, 1)
            att = torch.einsum("qhd,khd->hqk", q, k) * self.scale
            att = att.masked_fill(torch.ones(T, T, dtype=torch.bool).triu(1)[None], float("-inf"))
            o = torch.einsum("hqk,khd->qhd", att.softmax(-1), v).reshape(T, -1)
            h = h + o @ w[p + "o"].t()
            x = rms(h, w[p + "mlp_norm"])
            gu = (x @ w[p + "gate_up"].t()).reshape(T, -1, 2, 16)
            g = (torch.nn.functional.silu(gu[:, :, 0]) * gu[:, :, 1]).reshape(T, -1)
            h = h + g @ w[p + "down"].t()
        return rms(h, w["norm"]) @ w["lm_head"].t()

    def config_dict(self):
        return asdict(self.cfg)
