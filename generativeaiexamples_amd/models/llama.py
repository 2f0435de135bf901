"""Llama-3 family decoder (Llama-3-8B / 70B / 3.1 / 3.2 text, Mistral-style GQA) on the gfx950 kernels.

Replaces the reference's NIM-LLM container (``nvcr.io/nim/meta/llama3-8b-instruct``,
API default ``meta/llama3-70b-instruct``, RAG/examples/local_deploy/docker-compose-nim-ms.yaml:2-28).

Per layer, 7 launches: RMSNorm -> QKV GEMM -> fused RoPE + paged-KV write -> attention
(prefill tokens: paged flash-attention; decode tokens: split-KV flash-decoding) -> O-proj GEMM
with the residual add fused in its epilogue -> RMSNorm -> gate/up GEMM with SwiGLU fused in its
epilogue (interleaved weights) -> down GEMM with fused residual add.

The same decoder serves the other dense families the reference fine-tunes or serves through NIM
 via architecture flags on :class:`LlamaConfig`:
  * Gemma / CodeGemma (finetuning/Gemma, finetuning/Codegemma): RMSNorm with (1 + w) weights
    (folded at load), GeGLU MLP (tanh-GELU gate), embeddings scaled by sqrt(hidden), tied LM head,
    head_dim 256 (MHA 7B, MQA 2B);
  * StarCoder2 (finetuning/StarCoder2): LayerNorm with bias, non-gated tanh-GELU MLP (c_fc / c_proj)
    with biases, biased QKV / O projections, GQA;
  * Qwen2 / 2.5 (QKV bias) and Qwen3 (per-head q/k RMSNorm before RoPE);
  * Mistral (no flags).

Tensor parallel: QKV and gate/up are column-parallel (heads / intermediate split),
O and down are row-parallel followed by one all-reduce each (the residual is added on TP rank 0
only, so it is counted once), embedding and LM head are vocab-parallel (all-gather of logits).
"""
from __future__ import annotations

import json
import math
import os
from dataclasses import asdict, dataclass
from typing import Dict, List, Optional

import torch

from .. import ops
from ..parallel.dist import DistContext, get_context
from .common import ForwardBatch, randn_like_

_GEMV_B1 = os.environ.get("GAI_GEMV_B1", "0") == "1"


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
    # architecture flags (defaults = Llama)
    arch: str = "llama"        # llama | mistral | gemma | starcoder2 | qwen2 | qwen3
    norm: str = "rms"          # rms | layernorm (weight + bias)
    mlp: str = "swiglu"        # swiglu | geglu (interleaved gate/up) | gelu_tanh (non-gated fc -> down)
    qkv_bias: bool = False
    o_bias: bool = False
    mlp_bias: bool = False
    embed_scale: bool = False  # h = embed * sqrt(hidden) (Gemma)
    qk_norm: bool = False      # per-head RMSNorm of q and k before RoPE (Qwen3)

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
    def gemma_7b(**kw):
        return LlamaConfig(name="google/gemma-7b", arch="gemma", vocab_size=256000, hidden_size=3072,
                           intermediate_size=24576, num_layers=28, num_heads=16, num_kv_heads=16, head_dim=256,
                           rope_theta=10000.0, rms_eps=1e-6, tie_embeddings=True, mlp="geglu", embed_scale=True,
                           bos_token_id=2, eos_token_ids=(1, 107), **kw)

    @staticmethod
    def gemma_2b(**kw):
        return LlamaConfig(name="google/gemma-2b", arch="gemma", vocab_size=256000, hidden_size=2048,
                           intermediate_size=16384, num_layers=18, num_heads=8, num_kv_heads=1, head_dim=256,
                           rope_theta=10000.0, rms_eps=1e-6, tie_embeddings=True, mlp="geglu", embed_scale=True,
                           bos_token_id=2, eos_token_ids=(1, 107), **kw)

    @staticmethod
    def codegemma_7b(**kw):
        return LlamaConfig.gemma_7b(**{**dict(name="google/codegemma-7b"), **kw})

    @staticmethod
    def starcoder2_15b(**kw):
        return LlamaConfig(name="bigcode/starcoder2-15b", arch="starcoder2", vocab_size=49152, hidden_size=6144,
                           intermediate_size=24576, num_layers=40, num_heads=48, num_kv_heads=4, head_dim=128,
                           rope_theta=100000.0, rms_eps=1e-5, max_position=16384, norm="layernorm",
                           mlp="gelu_tanh", qkv_bias=True, o_bias=True, mlp_bias=True, bos_token_id=0,
                           eos_token_ids=(0,), **kw)

    @staticmethod
    def starcoder2_7b(**kw):
        return LlamaConfig.starcoder2_15b(**{**dict(name="bigcode/starcoder2-7b", hidden_size=4608,
                                                    intermediate_size=18432, num_layers=32, num_heads=36,
                                                    num_kv_heads=4, rope_theta=1000000.0), **kw})

    @staticmethod
    def qwen25_7b(**kw):
        return LlamaConfig(name="qwen/qwen2.5-7b-instruct", arch="qwen2", vocab_size=152064, hidden_size=3584,
                           intermediate_size=18944, num_layers=28, num_heads=28, num_kv_heads=4, head_dim=128,
                           rope_theta=1000000.0, rms_eps=1e-6, max_position=32768, qkv_bias=True,
                           bos_token_id=151643, eos_token_ids=(151645, 151643), **kw)

    @staticmethod
    def qwen3_8b(**kw):
        return LlamaConfig(name="qwen/qwen3-8b", arch="qwen3", vocab_size=151936, hidden_size=4096,
                           intermediate_size=12288, num_layers=36, num_heads=32, num_kv_heads=8, head_dim=128,
                           rope_theta=1000000.0, rms_eps=1e-6, max_position=40960, qk_norm=True,
                           bos_token_id=151643, eos_token_ids=(151645, 151643), **kw)

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
        return LlamaConfig(**LlamaConfig.hf_fields(c, os.path.basename(path.rstrip("/"))))

    @staticmethod
    def hf_fields(c: dict, name: str) -> dict:
        """LlamaConfig keyword arguments of a HF decoder config.json (llama / mistral / mixtral / gemma /
        starcoder2 / qwen2 / qwen3; transformers 4 and 5 rope layouts)."""
        eos = c.get("eos_token_id", 2)
        mt = c.get("model_type", "llama")
        flags = {}
        if mt == "gemma":
            flags = dict(arch="gemma", mlp="geglu", embed_scale=True)
            c.setdefault("tie_word_embeddings", True)
        elif mt == "starcoder2":
            flags = dict(arch="starcoder2", norm="layernorm", mlp="gelu_tanh", qkv_bias=c.get("use_bias", True),
                         o_bias=c.get("use_bias", True), mlp_bias=c.get("use_bias", True))
            c.setdefault("rms_norm_eps", c.get("norm_epsilon", 1e-5))
        elif mt == "qwen2":
            flags = dict(arch="qwen2", qkv_bias=True)
        elif mt == "qwen3":
            flags = dict(arch="qwen3", qk_norm=True, qkv_bias=bool(c.get("attention_bias", False)))
        elif mt in ("mistral", "mixtral"):
            flags = dict(arch="mistral")
        theta, scaling = hf_rope(c)
        return dict(**flags,
            vocab_size=c["vocab_size"], hidden_size=c["hidden_size"], intermediate_size=c["intermediate_size"],
            num_layers=c["num_hidden_layers"], num_heads=c["num_attention_heads"],
            num_kv_heads=c.get("num_key_value_heads") or c["num_attention_heads"],
            head_dim=c.get("head_dim") or c["hidden_size"] // c["num_attention_heads"],
            rope_theta=theta, rope_scaling=scaling,
            rms_eps=c.get("rms_norm_eps", 1e-5), max_position=c.get("max_position_embeddings", 8192),
            tie_embeddings=c.get("tie_word_embeddings", False), bos_token_id=c.get("bos_token_id", 1),
            eos_token_ids=tuple(eos) if isinstance(eos, list) else (eos,), name=name)


def hf_rope(c: dict) -> tuple:
    """(rope_theta, llama3 scaling dict or None) of a HF config: transformers 4 keeps ``rope_theta`` and
    ``rope_scaling`` at the top level (the published Llama-3.x checkpoints), transformers 5 writes one
    ``rope_parameters`` dict. Only the default and ``llama3`` rope types exist in this framework."""
    rp = c.get("rope_parameters") or {}
    theta = float(c.get("rope_theta") or rp.get("rope_theta") or 10000.0)
    sc = c.get("rope_scaling") or rp
    kind = (sc or {}).get("rope_type", (sc or {}).get("type", "default"))
    if kind in ("default", None) or not sc:
        return theta, None
    if kind != "llama3":
        raise ValueError(f"rope_type {kind!r} is not supported (default and llama3 are)")
    return theta, {k: sc[k] for k in ("factor", "low_freq_factor", "high_freq_factor",
                                      "original_max_position_embeddings") if k in sc}


class LlamaModel:
    """Weights + forward. Weights are plain tensors (no nn.Module): the engine owns execution."""

    supports_fp8_kv = True  # the attention path passes the KV cache's per-layer scales (EngineConfig.kv_cache_dtype)

    supports_tp_sampling = True  # forward honours ForwardBatch.tp_local_logits (engine: ops.sample_tp)

    def __init__(self, cfg: LlamaConfig, device=None, dtype=torch.bfloat16, dist_ctx: DistContext | None = None):
        self.cfg = cfg
        self.ctx = dist_ctx or get_context()
        self.device = torch.device(device) if device is not None else self.ctx.device
        self.dtype = dtype
        tp = self.ctx.tp_size
        assert cfg.num_heads % tp == 0 and cfg.num_kv_heads % tp == 0 and cfg.intermediate_size % (16 * tp) == 0
        assert cfg.norm in ("rms", "layernorm") and cfg.mlp in ("swiglu", "geglu", "gelu_tanh"), cfg
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
        ln = c.norm == "layernorm"
        self.w["embed"] = e(self.vocab_local, D)
        for i in range(c.num_layers):
            p = f"l{i}."
            self.w[p + "attn_norm"] = e(D)
            self.w[p + "qkv"] = e((self.hq + 2 * self.hkv) * hd, D)
            self.w[p + "o"] = e(D, self.hq * hd)
            self.w[p + "mlp_norm"] = e(D)
            if c.mlp == "gelu_tanh":
                self.w[p + "fc"] = e(self.inter, D)
            else:
                self.w[p + "gate_up"] = e(2 * self.inter, D)  # interleaved per 16 rows
            self.w[p + "down"] = e(D, self.inter)
            if ln:
                self.w[p + "attn_norm_b"] = e(D)
                self.w[p + "mlp_norm_b"] = e(D)
            if c.qkv_bias:
                self.w[p + "qkv_b"] = e((self.hq + 2 * self.hkv) * hd)
            if c.o_bias:
                self.w[p + "o_b"] = e(D)
            if c.mlp_bias:
                self.w[p + ("fc_b" if c.mlp == "gelu_tanh" else "gate_up_b")] = e(
                    self.inter if c.mlp == "gelu_tanh" else 2 * self.inter)
                self.w[p + "down_b"] = e(D)
            if c.qk_norm:
                self.w[p + "q_norm"] = e(hd)
                self.w[p + "k_norm"] = e(hd)
        self.w["norm"] = e(D)
        if ln:
            self.w["norm_b"] = e(D)
        self.w["lm_head"] = self.w["embed"] if c.tie_embeddings else e(self.vocab_local, D)

    # Projections that keep a fragment-shuffled decode copy (ops.preshuffle_weight, EngineConfig.decode_preshuffle,
    # on by default): HBM-cold at M = 64 (profiles/r3/psw_ab/dec_hbm.jsonl) gate_up + SwiGLU 56.1 -> 44.3 us,
    # down 36.0 -> 29.3, LM head 238 -> 208, QKV 23.8 -> 21.4, O 17.2 -> 16.4 us.
    DECODE_PROJECTIONS = ("qkv", "o", "gate_up", "down", "proj", "lm_head")

    # decode-GEMM gain of the fragment-shuffled copy per projection kind (profiles/r3/psw_ab, B = 64): the budget
    # goes to whole kinds in this order
    PSW_PRIORITY = ("gate_up", "down", "lm_head", "qkv", "proj", "o")

    def preshuffle_decode_weights(self, budget_bytes: Optional[int] = None, in_place: bool = False) -> int:
        """Fragment-ordered decode weights for the per-layer projections; returns the bytes added. Call after the
        weights are final.

        ``in_place`` (the engine's default, EngineConfig.weight_layout = "fragment"): each qualifying bf16 projection
        is rewritten in place into MFMA fragment order (ops.to_fragment_layout_) - ONE layout, read by the prefill
        GEMMs, the decode GEMMs and the batch <= 4 GEMV alike, no copy (17 GB less than the two-copy layout for
        Llama-3-8B). Weights that do not qualify (fp8, >= 2 GiB, a LM head tied to the embedding table) fall back to
        a copy under the budget.

        Otherwise (two layouts) fragment-shuffled copies are attached (ops.preshuffle_weight). With ``budget_bytes``
        whole projection kinds are copied in PSW_PRIORITY order while they fit (gate_up +26 %, down +23 %,
        lm_head +14 %, qkv +11 %, o +5 % decode GEMM speed): a 70B model on ONE GPU keeps most of its HBM for
        the KV cache and still gets the down / LM head / QKV copies (53 of 57 GB at a 20 % budget)."""
        tied = {id(v) for k, v in self.w.items() if k.rsplit(".", 1)[-1] not in self.DECODE_PROJECTIONS}
        kinds: dict = {}
        for k, v in self.w.items():
            kind = k.rsplit(".", 1)[-1]
            done = v.dec is not None if isinstance(v, ops.Fp8Weight) else ops.decode_operand(v) is not None
            if kind in self.DECODE_PROJECTIONS and isinstance(v, (torch.Tensor, ops.Fp8Weight)) and not done:
                if in_place and id(v) not in tied and ops.to_fragment_layout_(v):
                    continue
                kinds.setdefault(kind, {})[id(v)] = v  # tied weights count once
        added, left = 0, budget_bytes
        for kind in self.PSW_PRIORITY:
            ws = [v for v in kinds.get(kind, {}).values() if ops.psw_qualifies(v)]
            need = sum(ops.psw_bytes(v) for v in ws)
            if not ws or (left is not None and need > left):
                continue
            for v in ws:
                ops.preshuffle_weight(v)
            added += need
            if left is not None:
                left -= need
        return added

    def random_init(self, seed: int = 0):
        """Random-init weights of the real architecture (benchmarks have no checkpoints offline)."""
        c = self.cfg
        s = seed * 1000 + self.ctx.tp_rank
        for k, t in self.w.items():
            if k.endswith("norm"):
                t.fill_(1.0)
            elif k.endswith("_b"):
                t.zero_() if k.endswith("norm_b") else randn_like_(t, s, 0.02)
            elif k == "lm_head" and c.tie_embeddings:
                continue
            else:
                fan_in = t.shape[1]
                randn_like_(t, s, 1.0 / math.sqrt(fan_in) if k not in ("embed",) else 0.02)
            s += 1
        return self

    def _put(self, name: str, t: torch.Tensor) -> None:
        """Copy a row-major weight in; a weight an engine already rewrote into the one (fragment-ordered) layout
        (ops.to_fragment_layout_) is stored fragment-ordered again."""
        dst = self.w[name]
        dst.copy_(t.to(self.dtype))
        if ops.is_frag(dst):
            ops.shuffle_fragments_(dst)

    def load_hf_state(self, sd: Dict[str, torch.Tensor]):
        """Load a HF Llama state dict (full weights; each TP rank keeps its shard)."""
        c, tp, r = self.cfg, self.ctx.tp_size, self.ctx.tp_rank
        hd = c.head_dim

        def shard_rows(t, n):  # column-parallel (output dim)
            return t.reshape(tp, n // tp, *t.shape[1:])[r] if tp > 1 else t

        put = self._put

        def norm_w(t):  # Gemma stores RMSNorm weights as w with y = x_hat * (1 + w): fold the 1 in
            return t.float() + 1.0 if c.arch == "gemma" else t

        emb = sd["model.embed_tokens.weight"]
        pad = self.vocab_local * tp - emb.shape[0]
        if pad:
            emb = torch.cat([emb, emb.new_zeros(pad, emb.shape[1])])
        put("embed", shard_rows(emb, emb.shape[0]))
        for i in range(c.num_layers):
            p, h = f"l{i}.", f"model.layers.{i}."
            put(p + "attn_norm", norm_w(sd[h + "input_layernorm.weight"]))
            put(p + "mlp_norm", norm_w(sd[h + "post_attention_layernorm.weight"]))
            if c.norm == "layernorm":
                put(p + "attn_norm_b", sd[h + "input_layernorm.bias"])
                put(p + "mlp_norm_b", sd[h + "post_attention_layernorm.bias"])
            q = shard_rows(sd[h + "self_attn.q_proj.weight"], c.num_heads * hd)
            k = shard_rows(sd[h + "self_attn.k_proj.weight"], c.num_kv_heads * hd)
            v = shard_rows(sd[h + "self_attn.v_proj.weight"], c.num_kv_heads * hd)
            put(p + "qkv", torch.cat([q, k, v]))
            if c.qkv_bias:
                put(p + "qkv_b", torch.cat([shard_rows(sd[h + "self_attn.q_proj.bias"], c.num_heads * hd),
                                            shard_rows(sd[h + "self_attn.k_proj.bias"], c.num_kv_heads * hd),
                                            shard_rows(sd[h + "self_attn.v_proj.bias"], c.num_kv_heads * hd)]))
            if c.qk_norm:
                put(p + "q_norm", sd[h + "self_attn.q_norm.weight"])
                put(p + "k_norm", sd[h + "self_attn.k_norm.weight"])
            o = sd[h + "self_attn.o_proj.weight"]
            put(p + "o", o.reshape(o.shape[0], tp, -1)[:, r] if tp > 1 else o)
            if c.o_bias:
                put(p + "o_b", sd[h + "self_attn.o_proj.bias"])
            self._load_mlp(sd, i)
        put("norm", norm_w(sd["model.norm.weight"]))
        if c.norm == "layernorm":
            put("norm_b", sd["model.norm.bias"])
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

        if c.mlp == "gelu_tanh":  # StarCoder2: c_fc -> gelu -> c_proj
            self._put(p + "fc", shard_rows(sd[h + "mlp.c_fc.weight"], c.intermediate_size))
            dn = sd[h + "mlp.c_proj.weight"]
            if c.mlp_bias:
                self.w[p + "fc_b"].copy_(shard_rows(sd[h + "mlp.c_fc.bias"], c.intermediate_size).to(self.dtype))
                self.w[p + "down_b"].copy_(sd[h + "mlp.c_proj.bias"].to(self.dtype))
        else:
            g = shard_rows(sd[h + "mlp.gate_proj.weight"], c.intermediate_size)
            u = shard_rows(sd[h + "mlp.up_proj.weight"], c.intermediate_size)
            self._put(p + "gate_up", ops.interleave_gate_up(g, u))
            dn = sd[h + "mlp.down_proj.weight"]
        self._put(p + "down", dn.reshape(dn.shape[0], tp, -1)[:, r] if tp > 1 else dn)

    def export_hf_state(self) -> Dict[str, torch.Tensor]:
        """Inverse of load_hf_state for a TP=1 model (checkpoint export, TP-reshard tests)."""
        assert self.ctx.tp_size == 1
        c, hd = self.cfg, self.cfg.head_dim
        w = {k: ops.natural_weight(v) for k, v in self.w.items()}  # row-major whatever the resident layout

        def norm_w(t):
            return (t.float() - 1.0).to(t.dtype) if c.arch == "gemma" else t.clone()

        sd = {"model.embed_tokens.weight": w["embed"].clone(), "model.norm.weight": norm_w(w["norm"])}
        if c.norm == "layernorm":
            sd["model.norm.bias"] = w["norm_b"].clone()
        if not c.tie_embeddings:
            sd["lm_head.weight"] = w["lm_head"].clone()
        nq, nk = c.num_heads * hd, c.num_kv_heads * hd
        for i in range(c.num_layers):
            p, h = f"l{i}.", f"model.layers.{i}."
            qkv = w[p + "qkv"]
            sd[h + "self_attn.q_proj.weight"] = qkv[:nq].clone()
            sd[h + "self_attn.k_proj.weight"] = qkv[nq:nq + nk].clone()
            sd[h + "self_attn.v_proj.weight"] = qkv[nq + nk:].clone()
            if c.qkv_bias:
                b = w[p + "qkv_b"]
                sd[h + "self_attn.q_proj.bias"] = b[:nq].clone()
                sd[h + "self_attn.k_proj.bias"] = b[nq:nq + nk].clone()
                sd[h + "self_attn.v_proj.bias"] = b[nq + nk:].clone()
            if c.qk_norm:
                sd[h + "self_attn.q_norm.weight"] = w[p + "q_norm"].clone()
                sd[h + "self_attn.k_norm.weight"] = w[p + "k_norm"].clone()
            sd[h + "self_attn.o_proj.weight"] = w[p + "o"].clone()
            if c.o_bias:
                sd[h + "self_attn.o_proj.bias"] = w[p + "o_b"].clone()
            if c.mlp == "gelu_tanh":
                sd[h + "mlp.c_fc.weight"] = w[p + "fc"].clone()
                sd[h + "mlp.c_proj.weight"] = w[p + "down"].clone()
                if c.mlp_bias:
                    sd[h + "mlp.c_fc.bias"] = w[p + "fc_b"].clone()
                    sd[h + "mlp.c_proj.bias"] = w[p + "down_b"].clone()
            else:
                gu = w[p + "gate_up"].reshape(-1, 2, 16, c.hidden_size)
                sd[h + "mlp.gate_proj.weight"] = gu[:, 0].reshape(-1, c.hidden_size).clone()
                sd[h + "mlp.up_proj.weight"] = gu[:, 1].reshape(-1, c.hidden_size).clone()
                sd[h + "mlp.down_proj.weight"] = w[p + "down"].clone()
            sd[h + "input_layernorm.weight"] = norm_w(w[p + "attn_norm"])
            sd[h + "post_attention_layernorm.weight"] = norm_w(w[p + "mlp_norm"])
            if c.norm == "layernorm":
                sd[h + "input_layernorm.bias"] = w[p + "attn_norm_b"].clone()
                sd[h + "post_attention_layernorm.bias"] = w[p + "mlp_norm_b"].clone()
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
        if slots.shape[0] < x.shape[0]:  # sequence-parallel padding rows use the base model
            slots = torch.cat([slots, slots.new_zeros(x.shape[0] - slots.shape[0])])
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

    def _norm(self, x, name: str, residual=None):
        c = self.cfg
        if c.norm == "layernorm":
            return ops.layer_norm(x, self.w[name], self.w[name + "_b"], c.rms_eps, residual=residual)
        return ops.rms_norm(x, self.w[name], c.rms_eps, residual=residual)

    def _row_bias(self, name: str):
        """Bias of a row-parallel projection: added once (TP rank 0) before the all-reduce."""
        return self.w.get(name) if self.ctx.tp_rank == 0 else None

    @property
    def embed_multiplier(self) -> float:
        # Gemma scales embeddings by sqrt(hidden) rounded to the activation dtype (HF `normalizer`)
        return float(torch.tensor(self.cfg.hidden_size ** 0.5, dtype=self.dtype))

    def _qk_norm(self, qkv: torch.Tensor, p: str):
        T, hd, hq, hkv = qkv.shape[0], self.cfg.head_dim, self.hq, self.hkv
        q3 = qkv.view(T, hq + 2 * hkv, hd)
        for sl, key in ((slice(0, hq), "q_norm"), (slice(hq, hq + hkv), "k_norm")):
            part = q3[:, sl].reshape(-1, hd)
            q3[:, sl] = ops.rms_norm(part, self.w[p + key], self.cfg.rms_eps).view(T, -1, hd)

    def _gemv_ok(self, fb: ForwardBatch, kv) -> bool:
        """Batch <= 4 pure decode on the small-batch GEMV path (gemv.hip): five launches per layer, the norms
        staged into the consumer projections, no split-K slabs or tail kernels."""
        c, w = self.cfg, self.w
        T = fb.num_tokens
        if not (fb.token_ids.is_cuda and fb.num_prefill_tokens == 0 and 1 <= T <= 4 and self.ctx.tp_size == 1):
            return False
        if (c.norm != "rms" or c.mlp != "swiglu" or c.qk_norm or c.head_dim != 128 or self.lora_names
                or c.qkv_bias or c.o_bias or c.mlp_bias or os.environ.get("GAI_GEMV", "1") != "1"):
            return False
        if kv.layer(0)[0].dtype != torch.bfloat16 or not isinstance(w["l0.qkv"], torch.Tensor):
            return False
        D, I = c.hidden_size, self.inter
        return (ops.gemv_ok(T, w["l0.qkv"].shape[0], D, True) and ops.gemv_ok(T, D, self.hq * c.head_dim)
                and ops.gemv_ok(T, 2 * I, D, True) and ops.gemv_ok(T, D, I) and ops.gemv_ok(T, w["lm_head"].shape[0], D, True))

    def _forward_gemv(self, fb: ForwardBatch, kv, decode_ws=None) -> torch.Tensor:
        c, w = self.cfg, self.w
        T, hd = fb.num_tokens, c.head_dim
        res = ops.embedding(fb.token_ids, w["embed"], self.vstart, self.vstart + self.vocab_local)
        if c.embed_scale:
            res.mul_(self.embed_multiplier)
        q = torch.empty(T, self.hq, hd, device=res.device, dtype=self.dtype)
        attn = torch.empty_like(q)
        # batch 1, opt-in (GAI_GEMV_B1=1): the launches rebalanced onto more workgroups - QKV as 2 K parts whose
        # fp32 slabs the attention launch folds (sum, RoPE, KV write), gate_up as an fp32 GEMV of one 16-row column
        # per workgroup (1792 for Llama-3-8B) with the SwiGLU applied while the down projection stages its input.
        # Measured slower (graph replay 3.197 vs 3.135 ms, profiles/r6/decode_b1): gate_up was already streaming
        # at 5.8 TB/s (40.8 vs 41.1 us), the fp32 staging costs down ~1.7 us, the fold costs attention ~1.1 us
        b1 = T == 1 and _GEMV_B1 and ops.is_frag(w["l0.gate_up"]) and ops.is_frag(w["l0.down"])
        slabs = gu = None
        if b1:
            slabs = torch.empty(2, T, w["l0.qkv"].shape[0], device=res.device, dtype=torch.float32)
            gu = torch.empty(T, w["l0.gate_up"].shape[0], device=res.device, dtype=torch.float32)
        for i in range(c.num_layers):
            p = f"l{i}."
            kc, vc = kv.layer(i)
            ks, vs = kv.scales(i)
            fold = None
            if b1:
                fold = ops.gemv_qkv_partials(res, w[p + "qkv"], w[p + "attn_norm"], c.rms_eps, kc, hd, decode_ws, ks,
                                             vs, out=slabs)
            if fold is None:
                ops.gemv_rope_kv(res, w[p + "qkv"], w[p + "attn_norm"], c.rms_eps, fb.positions, self.cos_sin,
                                 fb.slots, q, kc, vc, self.hq, self.hkv)
            else:
                fold = fold + (fb.positions, self.cos_sin, fb.slots)
            ops.attention_decode(q, kc, vc, fb.decode_block_tables, fb.decode_ctx, self.scale, ws=decode_ws,
                                 max_ctx=fb.max_decode_ctx, out=attn, k_scale=ks, v_scale=vs, qkv_fold=fold)
            ops.gemv(attn.view(T, -1), w[p + "o"], epi="residual", res=res)
            if b1:
                ops.gemv(res, w[p + "gate_up"], gamma=w[p + "mlp_norm"], eps=c.rms_eps, epi="f32", out=gu)
                ops.gemv(None, w[p + "down"], epi="residual", res=res, swi=gu)
            else:
                g = ops.gemv(res, w[p + "gate_up"], gamma=w[p + "mlp_norm"], eps=c.rms_eps, epi="swiglu")
                ops.gemv(g, w[p + "down"], epi="residual", res=res)
        if fb.sample_rows is not None:
            res = res.index_select(0, fb.sample_rows)
        logits = ops.gemv(res, w["lm_head"], gamma=w["norm"], eps=c.rms_eps, epi="f32")
        return logits[:, : c.vocab_size]

    def forward(self, fb: ForwardBatch, kv, decode_ws=None) -> torch.Tensor:
        """Returns fp32 logits [len(sample_rows), vocab] (gathered over TP)."""
        if self.ctx.tp_size > 1 and self.ctx.sequence_parallel and fb.num_prefill_tokens > 0:
            return self._forward_sp(fb, kv, decode_ws)
        if self._gemv_ok(fb, kv):
            return self._forward_gemv(fb, kv, decode_ws)
        c, w, ctx = self.cfg, self.w, self.ctx
        T, P = fb.num_tokens, fb.num_prefill_tokens
        hd = c.head_dim
        # residual stream `res` is updated in place by the fused add+norm kernel, so the O and down
        # projections are plain GEMMs (row-parallel partial sums all-reduced before the add)
        res = ops.embedding(fb.token_ids, w["embed"], self.vstart, self.vstart + self.vocab_local)
        ctx.tp_all_reduce(res)
        if c.embed_scale:
            res.mul_(self.embed_multiplier)
        q = torch.empty(T, self.hq, hd, device=res.device, dtype=self.dtype)
        attn = torch.empty_like(q)
        h = None
        # TP = 1 decode: fold each row-parallel projection's split-K reduce, the residual add and the next
        # RMSNorm into one kernel (ops.linear_add_rmsnorm); xn carries the normalised input forward
        fuse = (res.is_cuda and ctx.tp_size == 1 and c.norm != "layernorm" and not self.lora_names and T <= 64
                and os.environ.get("GAI_FUSE_NORM", "1") == "1")
        xn = None
        # decode (T <= 64): split-K partials -> RoPE -> q / paged KV in one kernel; prefill (T >= 1024): the
        # same in the 256x256 GEMM's epilogue (ops.linear_rope_kv falls back where the kernels do not apply)
        fuse_qkv = (res.is_cuda and (T <= 64 or T >= 1024) and not self.lora_names and not c.qk_norm
                    and os.environ.get("GAI_FUSE_ROPE", "1") == "1")
        # TP prefill: row-parallel projections pipelined with their all-reduce (DistContext.tp_linear_all_reduce)
        overlap = (ctx.tp_size > 1 and not self.lora_names and os.environ.get("GAI_TP_OVERLAP", "1") == "1"
                   and T >= 2 * int(os.environ.get("GAI_TP_OVERLAP_CHUNK_ROWS", "1024")))
        # TP: the all-reduce of each row-parallel projection carries the residual add and the next RMSNorm
        tp_norm = (ctx.tp_size > 1 and c.norm != "layernorm" and os.environ.get("GAI_FUSE_NORM", "1") == "1")
        # TP = 1 prefill: the O / down GEMMs' residual epilogue writes bf16(bf16(h) + residual) into the residual
        # stream in place - the rounding the residual-adding norm kernel applies - and the norms then only read it:
        # one fewer [T, d] read and write per norm (a 16K-token chunk: 134 MB each)
        res_epi = (res.is_cuda and ctx.tp_size == 1 and not fuse and not self.lora_names
                   and os.environ.get("GAI_RES_EPI", "1") == "1")
        for i in range(c.num_layers):
            p = f"l{i}."
            if xn is not None:
                x, xn = xn, None
            else:
                x = self._norm(res, p + "attn_norm") if h is None else self._norm(h, p + "attn_norm", residual=res)
            kc, vc = kv.layer(i)
            ks, vs = kv.scales(i)
            # pure decode: the QKV RoPE / KV-write tail runs inside the decode-attention launch (ops.qkv_fold_partials)
            fold = (ops.qkv_fold_partials(x, w[p + "qkv"], w.get(p + "qkv_b"), kc, hd, decode_ws, ks, vs)
                    if fuse_qkv and P == 0 and T <= 64 else None)
            if fold is not None:
                fold = (fold[0], fold[1], fb.positions, self.cos_sin, fb.slots)
            elif fuse_qkv:
                ops.linear_rope_kv(x, w[p + "qkv"], w.get(p + "qkv_b"), fb.positions, self.cos_sin, fb.slots, q, kc,
                                   vc, self.hq, self.hkv, hd, ks, vs)
            else:
                qkv = self._lora(ops.linear(x, w[p + "qkv"], bias=w.get(p + "qkv_b")), x, i, "qkv", fb)
                if c.qk_norm:
                    self._qk_norm(qkv, p)
                ops.rope_kv_write(qkv, fb.positions, self.cos_sin, fb.slots, q, kc, vc, self.hq, self.hkv, hd, True,
                                  ks, vs)
            if P > 0:
                ops.attention_prefill(q[:P], kc, vc, fb.prefill_block_tables, fb.cu_q, fb.prefill_ctx, self.scale,
                                      True, tiles=fb.prefill_tiles, q_lens=fb.prefill_qlen, out=attn[:P], k_scale=ks,
                                      v_scale=vs)
            if T > P:
                ops.attention_decode(q[P:], kc, vc, fb.decode_block_tables, fb.decode_ctx, self.scale, ws=decode_ws,
                                     max_ctx=fb.max_decode_ctx, out=attn[P:], k_scale=ks, v_scale=vs, qkv_fold=fold)
            a2 = attn.view(T, -1)
            if fuse:
                x = ops.linear_add_rmsnorm(a2, w[p + "o"], res, w[p + "mlp_norm"], c.rms_eps, bias=w.get(p + "o_b"))
            elif overlap:  # TP prefill: each row chunk's all-reduce overlaps the next chunk's GEMM
                h = ctx.tp_linear_all_reduce(a2, w[p + "o"], self._row_bias(p + "o_b"))
                x = self._norm(h, p + "mlp_norm", residual=res)
            elif res_epi:
                ops.linear(a2, w[p + "o"], bias=w.get(p + "o_b"), residual=res, out=res)
                x = self._norm(res, p + "mlp_norm")
            else:
                h = self._lora(ops.linear(a2, w[p + "o"], bias=self._row_bias(p + "o_b")), a2, i, "o", fb)
                if tp_norm:  # all-reduce + residual add + RMSNorm in one peer-memory kernel
                    x = ctx.tp_all_reduce_rmsnorm(h, res, w[p + "mlp_norm"], c.rms_eps)
                else:
                    ctx.tp_all_reduce(h)
                    x = self._norm(h, p + "mlp_norm", residual=res)
            if c.mlp == "gelu_tanh":
                g = self._lora(ops.linear(x, w[p + "fc"], bias=w.get(p + "fc_b"), act="gelu_tanh"), x, i, "fc", fb)
            else:
                g = ops.linear(x, w[p + "gate_up"], act=c.mlp)
            last = i + 1 == c.num_layers
            if fuse and not (last and fb.sample_rows is not None):
                nxt = "norm" if last else f"l{i + 1}.attn_norm"
                xn = ops.linear_add_rmsnorm(g, w[p + "down"], res, w[nxt], c.rms_eps, bias=w.get(p + "down_b"))
                h = None
            elif overlap:
                h = ctx.tp_linear_all_reduce(g, w[p + "down"], self._row_bias(p + "down_b"))
            elif res_epi:  # the next layer's norm (or the final one) reads the updated residual stream
                ops.linear(g, w[p + "down"], bias=w.get(p + "down_b"), residual=res, out=res)
                h = None
            else:
                h = ops.linear(g, w[p + "down"], bias=self._row_bias(p + "down_b"))
                if tp_norm and not (last and fb.sample_rows is not None):
                    nxt = "norm" if last else f"l{i + 1}.attn_norm"
                    xn = ctx.tp_all_reduce_rmsnorm(h, res, w[nxt], c.rms_eps)
                    h = None
                else:
                    ctx.tp_all_reduce(h)
        if xn is not None:  # the final norm already ran inside the last layer's down projection
            logits = ops.linear(xn, w["lm_head"], out_dtype=torch.float32)
            if fb.tp_local_logits and ctx.tp_size > 1:
                return logits
            return ctx.tp_all_gather_last(logits)[:, : c.vocab_size]
        if fb.sample_rows is not None:
            h = h.index_select(0, fb.sample_rows) if h is not None else None
            res = res.index_select(0, fb.sample_rows)
        x = self._norm(res, "norm") if h is None else self._norm(h, "norm", residual=res)
        logits = ops.linear(x, w["lm_head"], out_dtype=torch.float32)
        if fb.tp_local_logits and ctx.tp_size > 1:
            return logits
        logits = ctx.tp_all_gather_last(logits)
        return logits[:, : c.vocab_size]

    def _forward_sp(self, fb: ForwardBatch, kv, decode_ws=None) -> torch.Tensor:
        """Tensor + sequence parallel forward for prefill / mixed steps: the residual stream
        and the norms live on T/tp token rows per rank; every row-parallel output is reduce-scattered
        and every column-parallel input all-gathered (tokens padded to a multiple of tp)."""
        c, w, ctx = self.cfg, self.w, self.ctx
        tp = ctx.tp_size
        T, P = fb.num_tokens, fb.num_prefill_tokens
        Tp = -(-T // tp) * tp
        hd = c.head_dim
        ids = fb.token_ids
        if Tp > T:
            ids = torch.cat([ids, ids.new_zeros(Tp - T)])
        res = ctx.tp_reduce_scatter_rows(ops.embedding(ids, w["embed"], self.vstart, self.vstart + self.vocab_local))
        if c.embed_scale:
            res.mul_(self.embed_multiplier)
        q = torch.empty(Tp, self.hq, hd, device=res.device, dtype=self.dtype)
        attn = torch.zeros_like(q)
        h = None
        for i in range(c.num_layers):
            p = f"l{i}."
            x = self._norm(res, p + "attn_norm") if h is None else self._norm(h, p + "attn_norm", residual=res)
            x = ctx.tp_all_gather_rows(x)
            qkv = self._lora(ops.linear(x, w[p + "qkv"], bias=w.get(p + "qkv_b")), x, i, "qkv", fb)
            if c.qk_norm:
                self._qk_norm(qkv, p)
            kc, vc = kv.layer(i)
            ks, vs = kv.scales(i)
            ops.rope_kv_write(qkv[:T], fb.positions, self.cos_sin, fb.slots, q[:T], kc, vc, self.hq, self.hkv, hd,
                              True, ks, vs)
            ops.attention_prefill(q[:P], kc, vc, fb.prefill_block_tables, fb.cu_q, fb.prefill_ctx, self.scale,
                                  True, tiles=fb.prefill_tiles, q_lens=fb.prefill_qlen, out=attn[:P], k_scale=ks,
                                  v_scale=vs)
            if T > P:
                ops.attention_decode(q[P:T], kc, vc, fb.decode_block_tables, fb.decode_ctx, self.scale, ws=decode_ws,
                                     max_ctx=fb.max_decode_ctx, out=attn[P:T], k_scale=ks, v_scale=vs)
            a2 = attn.view(Tp, -1)
            h = ctx.tp_reduce_scatter_rows(
                self._lora(ops.linear(a2, w[p + "o"], bias=self._row_bias(p + "o_b")), a2, i, "o", fb))
            x = ctx.tp_all_gather_rows(self._norm(h, p + "mlp_norm", residual=res))
            if c.mlp == "gelu_tanh":
                g = self._lora(ops.linear(x, w[p + "fc"], bias=w.get(p + "fc_b"), act="gelu_tanh"), x, i, "fc", fb)
            else:
                g = ops.linear(x, w[p + "gate_up"], act=c.mlp)
            h = ctx.tp_reduce_scatter_rows(ops.linear(g, w[p + "down"], bias=self._row_bias(p + "down_b")))
        x = ctx.tp_all_gather_rows(self._norm(h, "norm", residual=res))[:T]
        if fb.sample_rows is not None:
            x = x.index_select(0, fb.sample_rows)
        logits = ctx.tp_all_gather_last(ops.linear(x, w["lm_head"], out_dtype=torch.float32))
        return logits[:, : c.vocab_size]

    # ------------------------------------------------------------------ reference
    @torch.no_grad()
    def reference_forward(self, token_ids: torch.Tensor) -> torch.Tensor:
        """Dense full-sequence fp32 forward with no cache (test oracle; TP=1 only)."""
        c, w = self.cfg, {k: ops.natural_weight(v).float().cpu() for k, v in self.w.items()}
        T = token_ids.numel()
        hd = c.head_dim
        h = w["embed"][token_ids.long().cpu()]
        if c.embed_scale:
            h = h * self.embed_multiplier
        cs = self.cos_sin.cpu()[:T]
        cos, sin = cs[:, None, : hd // 2], cs[:, None, hd // 2:]

        def rope(t):
            a, b = t[..., : hd // 2], t[..., hd // 2:]
            return torch.cat([a * cos - b * sin, b * cos + a * sin], -1)

        def rms(x, g):
            return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + c.rms_eps) * g

        def norm(x, name):
            if c.norm == "layernorm":
                return torch.nn.functional.layer_norm(x, (x.shape[-1],), w[name], w[name + "_b"], c.rms_eps)
            return rms(x, w[name])

        def bias(name):
            return w.get(name, 0.0)

        for i in range(c.num_layers):
            p = f"l{i}."
            x = norm(h, p + "attn_norm")
            qkv = (x @ w[p + "qkv"].t() + bias(p + "qkv_b")).view(T, self.hq + 2 * self.hkv, hd)
            q, k, v = qkv[:, : self.hq], qkv[:, self.hq: self.hq + self.hkv], qkv[:, self.hq + self.hkv:]
            if c.qk_norm:
                q, k = rms(q, w[p + "q_norm"]), rms(k, w[p + "k_norm"])
            q, k = rope(q), rope(k)
            rep = self.hq // self.hkv
            k, v = k.repeat_interleave(rep, 1), v.repeat_interleave(rep, 1)
            att = torch.einsum("qhd,khd->hqk", q, k) * self.scale
            att = att.masked_fill(torch.ones(T, T, dtype=torch.bool).triu(1)[None], float("-inf"))
            o = torch.einsum("hqk,khd->qhd", att.softmax(-1), v).reshape(T, -1)
            h = h + o @ w[p + "o"].t() + bias(p + "o_b")
            x = norm(h, p + "mlp_norm")
            if c.mlp == "gelu_tanh":
                g = torch.nn.functional.gelu(x @ w[p + "fc"].t() + bias(p + "fc_b"), approximate="tanh")
            else:
                gu = (x @ w[p + "gate_up"].t()).reshape(T, -1, 2, 16)
                act = torch.nn.functional.silu(gu[:, :, 0]) if c.mlp == "swiglu" else \
                    torch.nn.functional.gelu(gu[:, :, 0], approximate="tanh")
                g = (act * gu[:, :, 1]).reshape(T, -1)
            h = h + g @ w[p + "down"].t() + bias(p + "down_b")
        return norm(h, "norm") @ w["lm_head"].t()

    @torch.no_grad()
    def reference_logits_at(self, token_ids: torch.Tensor, rows: List[int], device="cuda",
                            q_chunk: int = 256) -> torch.Tensor:
        """fp32 logits [len(rows), vocab] of a long sequence at the given positions, in plain PyTorch on ``device``
        (the long-context oracle: reference_forward's [T, T] score matrix would be 128 GB at T = 32K). RMSNorm /
        SwiGLU Llama layout, TP = 1. Causal attention runs in query chunks of ``q_chunk`` rows against the keys so
        far; the last layer computes queries, attention and the MLP for ``rows`` only."""
        c, dev = self.cfg, torch.device(device)
        assert c.norm == "rms" and c.mlp == "swiglu" and not c.qk_norm and self.ctx.tp_size == 1
        T, hd, hq, hkv = token_ids.numel(), c.head_dim, self.hq, self.hkv
        rep = hq // hkv

        def W(name):
            return ops.natural_weight(self.w[name]).to(dev, torch.float32)

        def rms(x, g):
            return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + c.rms_eps) * g

        cs = self.cos_sin[:T].to(dev)
        cos, sin = cs[:, None, : hd // 2], cs[:, None, hd // 2:]

        def rope(t, idx):
            a, b = t[..., : hd // 2], t[..., hd // 2:]
            return torch.cat([a * cos[idx] - b * sin[idx], b * cos[idx] + a * sin[idx]], -1)

        h = W("embed")[token_ids.long().to(dev)]
        if c.embed_scale:
            h = h * self.embed_multiplier
        sel = torch.tensor(rows, dtype=torch.long, device=dev)
        all_rows = torch.arange(T, device=dev)
        for i in range(c.num_layers):
            p = f"l{i}."
            last = i + 1 == c.num_layers
            wqkv, wo, wgu, wd = W(p + "qkv"), W(p + "o"), W(p + "gate_up"), W(p + "down")
            x = rms(h, W(p + "attn_norm"))
            kv = (x @ wqkv[hq * hd:].t()).view(T, 2 * hkv, hd)
            k, v = rope(kv[:, :hkv], all_rows), kv[:, hkv:]
            qrows = sel if last else all_rows
            out = torch.empty(qrows.numel(), hq * hd, device=dev)
            for s in range(0, qrows.numel(), q_chunk):
                r = qrows[s:s + q_chunk]
                q = rope((x[r] @ wqkv[: hq * hd].t()).view(-1, hq, hd), r)
                kmax = int(r.max()) + 1
                kk = k[:kmax].repeat_interleave(rep, 1)
                vv = v[:kmax].repeat_interleave(rep, 1)
                att = torch.einsum("qhd,khd->hqk", q, kk) * self.scale
                att = att.masked_fill(torch.arange(kmax, device=dev)[None, None, :] > r[None, :, None], float("-inf"))
                out[s:s + r.numel()] = torch.einsum("hqk,khd->qhd", att.softmax(-1), vv).reshape(r.numel(), -1)
                del att, kk, vv
            hr = h[qrows] + out @ wo.t()
            xm = rms(hr, W(p + "mlp_norm"))
            gu = (xm @ wgu.t()).reshape(hr.shape[0], -1, 2, 16)
            g = (torch.nn.functional.silu(gu[:, :, 0]) * gu[:, :, 1]).reshape(hr.shape[0], -1)
            h = hr + g @ wd.t()
            del wqkv, wo, wgu, wd
        return (rms(h, W("norm")) @ W("lm_head").t()).float().cpu()

    def config_dict(self):
        return asdict(self.cfg)
