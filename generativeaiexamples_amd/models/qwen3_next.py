"""Qwen3-Next (hybrid linear-attention MoE decoder; SURVEY W13, the model of the reference's
``oss_tutorials/Building_a_Simple_AI_Agent_with_Qwen3_Next_powered_by_NVIDIA_NIM.ipynb``, served here
through the same ``/v1/chat/completions`` + tools API instead of a hosted NIM).

Architecture (checked against the HF ``qwen3_next`` implementation by tests/test_qwen3_next_cpu.py):
  * layers cycle ``full_attention_interval - 1`` Gated-DeltaNet (linear attention) layers and one
    gated full-attention layer;
  * full attention: GQA, head_dim 256, per-head zero-centred q/k RMSNorm, partial RoPE (25 % of the
    head dims), output gated by ``sigmoid(x W_gate)`` before o_proj;
  * Gated DeltaNet: fused in-projection -> causal depthwise conv (kernel 4, SiLU) over q|k|v ->
    l2-normalised q, k; per-head decay ``g = -exp(A_log) softplus(a + dt_bias)`` and write strength
    ``beta = sigmoid(b)``; recurrent state ``S <- exp(g) S + k (beta (v - (exp(g) S)^T k))^T``,
    ``o = S^T q``; gated RMSNorm ``norm(o) * silu(z)``; out-projection;
  * MoE MLP: softmax router top-k (renormalised), SwiGLU experts, plus a shared SwiGLU expert scaled by
    ``sigmoid(x w_shared_gate)``; zero-centred RMSNorms ``x * (1 + w)`` everywhere else.

MI355X mapping:
  * 80B-A3B in bf16 is 160 GB: it fits ONE 288 GB MI355X, so TP = 1 (no collectives on the token path);
  * full-attention layers use the paged KV cache and the gfx950 prefill / decode attention kernels (head
    dim 256); partial RoPE runs in the fused rope_kv kernel by permuting the q/k head dims at load time
    so HF's rotate-half pairs (i, i + r/2) become the kernel's (i, i + D/2) pairs, with identity
    rotation (cos 1, sin 0) on the pass-through dims;
  * linear-attention layers keep per-sequence fp32 states (conv window + [Hv, dk, dv] recurrent state)
    in a slot pool; decode steps update them in place with the ``gdn_decode`` HIP kernel (graph
    capturable: slot vector is a static graph input); prefill chunks run the chunked (WY-form) gated
    delta rule as batched fp32 GEMMs, resuming from the slot state across chunked-prefill steps;
  * MoE reuses the Mixtral route / dispatch / grouped-GEMM / combine kernels; the shared-expert gate
    is one extra row of the router GEMM.
"""
from __future__ import annotations

import json
import math
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn.functional as F

from .. import ops
from ..parallel.dist import DistContext, get_context
from .common import ForwardBatch, randn_like_


@dataclass
class Qwen3NextConfig:
    name: str = "qwen/qwen3-next-80b-a3b-instruct"
    vocab_size: int = 151936
    hidden_size: int = 2048
    intermediate_size: int = 5120  # dense MLP of mlp_only layers
    num_layers: int = 48
    num_heads: int = 16
    num_kv_heads: int = 2
    head_dim: int = 256
    partial_rotary_factor: float = 0.25
    rope_theta: float = 10000000.0
    linear_num_key_heads: int = 16
    linear_num_value_heads: int = 32
    linear_key_head_dim: int = 128
    linear_value_head_dim: int = 128
    linear_conv_kernel_dim: int = 4
    num_experts: int = 512
    top_k: int = 10
    norm_topk_prob: bool = True
    moe_intermediate_size: int = 512
    shared_expert_intermediate_size: int = 512
    decoder_sparse_step: int = 1
    mlp_only_layers: Tuple[int, ...] = ()
    full_attention_interval: int = 4
    layer_types: Tuple[str, ...] = field(default_factory=tuple)
    rms_eps: float = 1e-6
    max_position: int = 262144
    bos_token_id: int = 151643
    eos_token_ids: Tuple[int, ...] = (151645, 151643)
    tie_word_embeddings: bool = False

    def __post_init__(self):
        if not self.layer_types:
            n = self.full_attention_interval
            self.layer_types = tuple("full_attention" if (i + 1) % n == 0 else "linear_attention"
                                     for i in range(self.num_layers))

    def is_moe(self, i: int) -> bool:
        return i not in self.mlp_only_layers and self.num_experts > 0 and (i + 1) % self.decoder_sparse_step == 0

    @property
    def rotary_dim(self) -> int:
        return int(self.head_dim * self.partial_rotary_factor)

    @staticmethod
    def qwen3_next_80b_a3b(**kw):
        return Qwen3NextConfig(**kw)

    @staticmethod
    def tiny(**kw):
        base = dict(name="tiny-qwen3-next", vocab_size=512, hidden_size=256, intermediate_size=256, num_layers=4,
                    num_heads=4, num_kv_heads=2, head_dim=64, linear_num_key_heads=2, linear_num_value_heads=4,
                    linear_key_head_dim=64, linear_value_head_dim=64, num_experts=8, top_k=2,
                    moe_intermediate_size=128, shared_expert_intermediate_size=128, max_position=2048,
                    bos_token_id=1, eos_token_ids=(2,), rope_theta=10000.0)
        base.update(kw)
        return Qwen3NextConfig(**base)

    @staticmethod
    def from_hf(path_or_dict) -> "Qwen3NextConfig":
        if isinstance(path_or_dict, dict):
            c = path_or_dict
        else:
            with open(os.path.join(path_or_dict, "config.json")) as f:
                c = json.load(f)
        eos = c.get("eos_token_id", 151645)
        return Qwen3NextConfig(
            name=c.get("_name_or_path", "qwen3-next"), vocab_size=c["vocab_size"], hidden_size=c["hidden_size"],
            intermediate_size=c.get("intermediate_size", 5120), num_layers=c["num_hidden_layers"],
            num_heads=c["num_attention_heads"], num_kv_heads=c["num_key_value_heads"],
            head_dim=c.get("head_dim", 256), partial_rotary_factor=c.get("partial_rotary_factor", 0.25),
            rope_theta=c.get("rope_theta", (c.get("rope_parameters") or {}).get("rope_theta", 1e7)),
            linear_num_key_heads=c["linear_num_key_heads"], linear_num_value_heads=c["linear_num_value_heads"],
            linear_key_head_dim=c["linear_key_head_dim"], linear_value_head_dim=c["linear_value_head_dim"],
            linear_conv_kernel_dim=c.get("linear_conv_kernel_dim", 4), num_experts=c.get("num_experts", 0),
            top_k=c.get("num_experts_per_tok", 10), norm_topk_prob=c.get("norm_topk_prob", True),
            moe_intermediate_size=c.get("moe_intermediate_size", 512),
            shared_expert_intermediate_size=c.get("shared_expert_intermediate_size", 512),
            decoder_sparse_step=c.get("decoder_sparse_step", 1), mlp_only_layers=tuple(c.get("mlp_only_layers", ())),
            full_attention_interval=c.get("full_attention_interval", 4),
            layer_types=tuple(c.get("layer_types") or ()), rms_eps=c.get("rms_norm_eps", 1e-6),
            max_position=c.get("max_position_embeddings", 262144), bos_token_id=c.get("bos_token_id", 151643),
            eos_token_ids=tuple(eos) if isinstance(eos, list) else (eos,),
            tie_word_embeddings=c.get("tie_word_embeddings", False))


# ------------------------------------------------------------------------------------------------
# gated delta rule (fp32 reference math; the decode step has a HIP kernel)
# ------------------------------------------------------------------------------------------------
def gdn_chunk_prefill(q, k, v, g, beta, S0, chunk: int = 64):
    """Chunked gated delta rule over one sequence. q, k [L, H, dk] (l2-normalised, q scaled), v [L, H, dv],
    g / beta [L, H], S0 [H, dk, dv]; all fp32. Returns (o [L, H, dv], S_L).

    Inside a chunk with cumulative log-decay G_t, the delta-rule writes u_s satisfy the unit lower
    triangular system (I + diag(beta) A) U = diag(beta) (V - diag(e^G) K S0) with
    A[s, r] = e^(G_s - G_r) (k_s . k_r) for r < s; then O = diag(e^G) Q S0 + M U with
    M[t, s] = e^(G_t - G_s) (q_t . k_s) for s <= t, and S_C = e^(G_C) S0 + K^T diag(e^(G_C - G)) U.
    """
    L = q.shape[0]
    S = S0
    outs = []
    for c0 in range(0, L, chunk):
        qc, kc, vc = (x[c0:c0 + chunk].transpose(0, 1) for x in (q, k, v))  # [H, C, d]
        gc, bc = g[c0:c0 + chunk].t(), beta[c0:c0 + chunk].t()  # [H, C]
        C = qc.shape[1]
        G = gc.cumsum(-1)
        Gd = G[:, :, None] - G[:, None, :]
        ar = torch.arange(C, device=q.device)
        strict = ar[None, :] < ar[:, None]
        incl = ar[None, :] <= ar[:, None]
        A = torch.exp(Gd.masked_fill(~strict, float("-inf"))) * (kc @ kc.transpose(-1, -2))
        T = torch.eye(C, device=q.device, dtype=q.dtype) + bc[:, :, None] * A
        eG = torch.exp(G)[:, :, None]
        rhs = bc[:, :, None] * (vc - eG * (kc @ S))
        U = torch.linalg.solve_triangular(T, rhs, upper=False, unitriangular=True)
        M = torch.exp(Gd.masked_fill(~incl, float("-inf"))) * (qc @ kc.transpose(-1, -2))
        outs.append((eG * (qc @ S) + M @ U).transpose(0, 1))
        wlast = torch.exp(G[:, -1:] - G)[:, :, None]
        S = torch.exp(G[:, -1])[:, None, None] * S + kc.transpose(-1, -2) @ (wlast * U)
    return torch.cat(outs), S


def gdn_recurrent_step(q, k, v, g, beta, S):
    """One token for a batch: q, k [B, H, dk], v [B, H, dv], g / beta [B, H], S [B, H, dk, dv] -> (o, S)."""
    S = S * torch.exp(g)[..., None, None]
    m = (S * k[..., None]).sum(-2)
    d = (v - m) * beta[..., None]
    S = S + k[..., None] * d[..., None, :]
    return (S * q[..., None]).sum(-2), S


def _l2n(x, eps=1e-6):
    return x * torch.rsqrt((x * x).sum(-1, keepdim=True) + eps)


class Qwen3NextModel:
    """Weights (plain tensors) + forward for the serving engine (same hooks as LlamaModel / Mllama)."""

    def __init__(self, cfg: Qwen3NextConfig, device=None, dtype=torch.bfloat16, dist_ctx: DistContext | None = None,
                 state_slots: Optional[int] = None):
        self.cfg = cfg
        self.ctx = dist_ctx or get_context()
        assert self.ctx.tp_size == 1, "Qwen3-Next runs TP=1 (80B-A3B bf16 = 160 GB fits one 288 GB MI355X)"
        self.device = torch.device(device) if device is not None else self.ctx.device
        self.dtype = dtype
        c = cfg
        self.hq, self.hkv = c.num_heads, c.num_kv_heads
        self.scale = 1.0 / math.sqrt(c.head_dim)
        self.full_layers = [i for i, t in enumerate(c.layer_types) if t == "full_attention"]
        self.kv_index = {layer: j for j, layer in enumerate(self.full_layers)}
        self.lin_layers = [i for i, t in enumerate(c.layer_types) if t == "linear_attention"]
        self.lin_index = {layer: j for j, layer in enumerate(self.lin_layers)}
        self.num_kv_layers = len(self.full_layers)
        self.kd = c.linear_num_key_heads * c.linear_key_head_dim
        self.vd = c.linear_num_value_heads * c.linear_value_head_dim
        self.conv_dim = 2 * self.kd + self.vd
        self.vocab_local, self.vstart = c.vocab_size, 0
        self.lora_names: list = []
        self.perm = self._rope_perm(c.head_dim, c.rotary_dim)
        self.cos_sin = self._rope_table(c, self.device)
        self.w: Dict[str, torch.Tensor] = {}
        self._alloc()
        # linear-attention state pool (allocated on first use): slot -> conv window + recurrent state
        self.n_slots = state_slots or int(os.environ.get("GAI_LINEAR_STATE_SLOTS", "64"))
        self.conv_state: Optional[torch.Tensor] = None  # [Ll, slots + 1, K - 1, conv_dim] fp32
        self.ssm_state: Optional[torch.Tensor] = None   # [Ll, slots + 1, Hv, dk, dv] fp32 (last slot = pad)
        self.slot_of: Dict[int, int] = {}
        self.free_slots: List[int] = []

    # ------------------------------------------------------------------ rope (partial, permuted)
    @staticmethod
    def _rope_perm(D: int, rd: int) -> torch.Tensor:
        """new head dim index -> HF head dim index, so HF pairs (i, i + rd/2) sit at (i, i + D/2)."""
        h, r = D // 2, rd // 2
        rest = list(range(rd, D))
        idx = list(range(r)) + rest[:h - r] + list(range(r, rd)) + rest[h - r:]
        return torch.tensor(idx, dtype=torch.long)

    @staticmethod
    def _rope_table(c: Qwen3NextConfig, device) -> torch.Tensor:
        D, rd = c.head_dim, c.rotary_dim
        inv = 1.0 / (c.rope_theta ** (torch.arange(0, rd, 2, dtype=torch.float64) / rd))
        freqs = torch.zeros(D // 2, dtype=torch.float64)
        freqs[: rd // 2] = inv
        f = torch.outer(torch.arange(c.max_position, dtype=torch.float64), freqs)
        return torch.cat([f.cos(), f.sin()], -1).float().to(device)

    # ------------------------------------------------------------------ weights
    def _alloc(self):
        c, d, dt = self.cfg, self.device, self.dtype
        D, hd = c.hidden_size, c.head_dim
        e = lambda *s, dtype=dt: torch.empty(*s, device=d, dtype=dtype)  # noqa: E731
        self.w["embed"] = e(c.vocab_size, D)
        self.w["lm_head"] = self.w["embed"] if c.tie_word_embeddings else e(c.vocab_size, D)
        self.w["norm"] = e(D)
        Hv, dv = c.linear_num_value_heads, c.linear_value_head_dim
        for i in range(c.num_layers):
            p = f"l{i}."
            self.w[p + "attn_norm"], self.w[p + "mlp_norm"] = e(D), e(D)
            if c.layer_types[i] == "full_attention":
                self.w[p + "qkv"] = e((self.hq + 2 * self.hkv) * hd, D)
                self.w[p + "gate"] = e(self.hq * hd, D)
                self.w[p + "q_norm"], self.w[p + "k_norm"] = e(hd), e(hd)
                self.w[p + "o"] = e(D, self.hq * hd)
            else:
                self.w[p + "in_proj"] = e(2 * self.kd + 2 * self.vd + 2 * Hv, D)
                self.w[p + "conv"] = e(self.conv_dim, c.linear_conv_kernel_dim, dtype=torch.float32)
                self.w[p + "A_log"] = e(Hv, dtype=torch.float32)
                self.w[p + "dt_bias"] = e(Hv, dtype=torch.float32)
                self.w[p + "gnorm"] = e(dv)
                self.w[p + "out"] = e(D, self.vd)
            if c.is_moe(i):
                E, I, Is = c.num_experts, c.moe_intermediate_size, c.shared_expert_intermediate_size
                self.w[p + "router"] = e(E + 1, D)  # last row: shared-expert gate
                self.w[p + "w13"] = e(E, 2 * I, D)  # gate/up interleaved per 16
                self.w[p + "w2"] = e(E, D, I)
                self.w[p + "sh_gate_up"] = e(2 * Is, D)
                self.w[p + "sh_down"] = e(D, Is)
            else:
                self.w[p + "gate_up"] = e(2 * c.intermediate_size, D)
                self.w[p + "down"] = e(D, c.intermediate_size)

    def random_init(self, seed: int = 0):
        s = seed * 1000
        c = self.cfg
        for k, t in self.w.items():
            name = k.rsplit(".", 1)[-1]
            if name in ("attn_norm", "mlp_norm", "norm", "q_norm", "k_norm", "gnorm"):
                t.fill_(1.0)
            elif name == "A_log":
                t.copy_(torch.log(torch.linspace(1.0, 16.0, t.numel())))
            elif name == "dt_bias":
                t.fill_(1.0)
            elif name == "conv":
                randn_like_(t, s, 1.0 / math.sqrt(c.linear_conv_kernel_dim))
            elif k == "embed":
                randn_like_(t, s, 0.02)
            else:
                randn_like_(t, s, 1.0 / math.sqrt(t.shape[-1]))
            s += 1
        return self

    def load_hf_state(self, sd: Dict[str, torch.Tensor]):
        """HF ``Qwen3NextForCausalLM`` state dict -> our fused / permuted / folded layout."""
        c, dt = self.cfg, self.dtype
        hd, H, Hkv = c.head_dim, self.hq, self.hkv
        Hk, Hv, dk, dv = c.linear_num_key_heads, c.linear_num_value_heads, c.linear_key_head_dim, c.linear_value_head_dim
        r = Hv // Hk
        P = self.perm
        fold = lambda t: (1.0 + t.float())  # noqa: E731  zero-centred RMSNorm weight
        put = lambda k, t: self.w[k].copy_(t.to(self.w[k].dtype))  # noqa: E731
        put("embed", sd["model.embed_tokens.weight"])
        if not c.tie_word_embeddings:
            put("lm_head", sd["lm_head.weight"])
        put("norm", fold(sd["model.norm.weight"]))
        for i in range(c.num_layers):
            p, h = f"l{i}.", f"model.layers.{i}."
            put(p + "attn_norm", fold(sd[h + "input_layernorm.weight"]))
            put(p + "mlp_norm", fold(sd[h + "post_attention_layernorm.weight"]))
            if c.layer_types[i] == "full_attention":
                a = h + "self_attn."
                qg = sd[a + "q_proj.weight"].view(H, 2, hd, -1)
                q = qg[:, 0][:, P].reshape(H * hd, -1)
                k = sd[a + "k_proj.weight"].view(Hkv, hd, -1)[:, P].reshape(Hkv * hd, -1)
                put(p + "qkv", torch.cat([q, k, sd[a + "v_proj.weight"]]))
                put(p + "gate", qg[:, 1].reshape(H * hd, -1))
                put(p + "q_norm", fold(sd[a + "q_norm.weight"])[P])
                put(p + "k_norm", fold(sd[a + "k_norm.weight"])[P])
                put(p + "o", sd[a + "o_proj.weight"])
            else:
                a = h + "linear_attn."
                qkvz = sd[a + "in_proj_qkvz.weight"].view(Hk, 2 * dk + 2 * r * dv, -1)
                qw, kw, vw, zw = torch.split(qkvz, [dk, dk, r * dv, r * dv], dim=1)
                ba = sd[a + "in_proj_ba.weight"].view(Hk, 2 * r, -1)
                bw, aw = torch.split(ba, [r, r], dim=1)
                flat = lambda t: t.reshape(-1, t.shape[-1])  # noqa: E731
                put(p + "in_proj", torch.cat([flat(qw), flat(kw), flat(vw), flat(zw), flat(bw), flat(aw)]))
                put(p + "conv", sd[a + "conv1d.weight"].squeeze(1))
                put(p + "A_log", sd[a + "A_log"])
                put(p + "dt_bias", sd[a + "dt_bias"])
                put(p + "gnorm", sd[a + "norm.weight"])
                put(p + "out", sd[a + "out_proj.weight"])
            if c.is_moe(i):
                m = h + "mlp."
                put(p + "router", torch.cat([sd[m + "gate.weight"], sd[m + "shared_expert_gate.weight"]]))
                I = c.moe_intermediate_size
                if m + "experts.gate_up_proj" in sd:  # fused 3-D expert tensors
                    gu, dn = sd[m + "experts.gate_up_proj"], sd[m + "experts.down_proj"]
                    for e_ in range(c.num_experts):
                        self.w[p + "w13"][e_].copy_(ops.interleave_gate_up(gu[e_, :I], gu[e_, I:]).to(dt))
                        self.w[p + "w2"][e_].copy_(dn[e_].to(dt))
                else:  # per-expert checkpoints
                    for e_ in range(c.num_experts):
                        x = m + f"experts.{e_}."
                        self.w[p + "w13"][e_].copy_(ops.interleave_gate_up(sd[x + "gate_proj.weight"],
                                                                           sd[x + "up_proj.weight"]).to(dt))
                        self.w[p + "w2"][e_].copy_(sd[x + "down_proj.weight"].to(dt))
                s_ = m + "shared_expert."
                put(p + "sh_gate_up", ops.interleave_gate_up(sd[s_ + "gate_proj.weight"], sd[s_ + "up_proj.weight"]))
                put(p + "sh_down", sd[s_ + "down_proj.weight"])
            else:
                m = h + "mlp."
                put(p + "gate_up", ops.interleave_gate_up(sd[m + "gate_proj.weight"], sd[m + "up_proj.weight"]))
                put(p + "down", sd[m + "down_proj.weight"])
        return self

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

    # ------------------------------------------------------------------ linear-attention state slots
    def _ensure_pool(self):
        if self.ssm_state is not None:
            return
        c, Ll, n = self.cfg, len(self.lin_layers), self.n_slots + 1
        self.conv_state = torch.zeros(Ll, n, c.linear_conv_kernel_dim - 1, self.conv_dim, device=self.device)
        self.ssm_state = torch.zeros(Ll, n, c.linear_num_value_heads, c.linear_key_head_dim,
                                     c.linear_value_head_dim, device=self.device)
        self.free_slots = list(range(self.n_slots))[::-1]

    @property
    def pad_slot(self) -> int:
        return self.n_slots

    def _slot(self, sid: int, fresh: bool) -> int:
        s = self.slot_of.get(sid)
        if s is None:
            if not self.free_slots:
                raise RuntimeError("Qwen3-Next state pool exhausted: raise GAI_LINEAR_STATE_SLOTS or lower "
                                   "max_num_seqs")
            s = self.slot_of[sid] = self.free_slots.pop()
            fresh = True
        if fresh:
            self.conv_state[:, s].zero_()
            self.ssm_state[:, s].zero_()
        return s

    def release_request(self, sid: int):
        s = self.slot_of.pop(sid, None)
        if s is not None:
            self.free_slots.append(s)

    def prepare_batch(self, fb: ForwardBatch):
        """Engine hook: map the step's sequences to state slots (fresh prompts start from zero state)."""
        self._ensure_pool()
        P = len(fb.prefill_qlen)
        ctx = fb.prefill_ctx_host or []
        pre = [self._slot(sid, ctx[i] == fb.prefill_qlen[i]) for i, sid in enumerate(fb.seq_ids[:P])]
        dec = [self._slot(sid, False) for sid in fb.seq_ids[P:]]
        fb.extra = dict(prefill_slots=pre,
                        decode_slots=torch.tensor(dec, dtype=torch.int32).to(self.device, non_blocking=True))

    def graph_static_inputs(self, bs: int) -> dict:
        self._ensure_pool()
        return dict(prefill_slots=[], decode_slots=torch.full((bs,), self.pad_slot, dtype=torch.int32,
                                                              device=self.device))

    def fill_graph_inputs(self, extra: dict, seq_ids, n: int):
        ids = torch.tensor([self._slot(s, False) for s in seq_ids], dtype=torch.int32)
        extra["decode_slots"][:n].copy_(ids, non_blocking=True)
        extra["decode_slots"][n:].fill_(self.pad_slot)

    # ------------------------------------------------------------------ blocks
    def _full_attention(self, x, i, fb, kv, decode_ws, T, P):
        c, w, p = self.cfg, self.w, f"l{i}."
        hd = c.head_dim
        qkv = ops.linear(x, w[p + "qkv"])
        gate = ops.linear(x, w[p + "gate"])
        q3 = qkv.view(T, self.hq + 2 * self.hkv, hd)
        for sl, key in ((slice(0, self.hq), "q_norm"), (slice(self.hq, self.hq + self.hkv), "k_norm")):
            q3[:, sl] = ops.rms_norm(q3[:, sl].reshape(-1, hd), w[p + key], c.rms_eps).view(T, -1, hd)
        q = torch.empty(T, self.hq, hd, device=x.device, dtype=self.dtype)
        attn = torch.empty_like(q)
        kc, vc = kv.layer(self.kv_index[i])
        ops.rope_kv_write(qkv, fb.positions, self.cos_sin, fb.slots, q, kc, vc, self.hq, self.hkv, hd, True)
        if P > 0:
            ops.attention_prefill(q[:P], kc, vc, fb.prefill_block_tables, fb.cu_q, fb.prefill_ctx, self.scale, True,
                                  tiles=fb.prefill_tiles, q_lens=fb.prefill_qlen, out=attn[:P])
        if T > P:
            ops.attention_decode(q[P:], kc, vc, fb.decode_block_tables, fb.decode_ctx, self.scale, ws=decode_ws,
                                 max_ctx=fb.max_decode_ctx, out=attn[P:])
        a = attn.view(T, -1) * torch.sigmoid(gate)
        return ops.linear(a, w[p + "o"])

    def _linear_attention(self, x, i, fb, T, P):
        c, w, p = self.cfg, self.w, f"l{i}."
        Hk, Hv, dk, dv = c.linear_num_key_heads, c.linear_num_value_heads, c.linear_key_head_dim, c.linear_value_head_dim
        Kc, li = c.linear_conv_kernel_dim, self.lin_index[i]
        proj = ops.linear(x, w[p + "in_proj"])
        cd, vd = self.conv_dim, self.vd
        mixed = proj[:, :cd].float()
        z = proj[:, cd:cd + vd]
        b = proj[:, cd + vd:cd + vd + Hv].float()
        a = proj[:, cd + vd + Hv:].float()
        cw = w[p + "conv"]  # [cd, Kc]
        conv = torch.empty(T, cd, device=x.device)
        extra = fb.extra or {}
        cs = self.conv_state[li]
        # prefill sequences: window = [state (Kc-1) | chunk]
        off = 0
        for s_i, L in enumerate(fb.prefill_qlen):
            slot = extra["prefill_slots"][s_i]
            xs = torch.cat([cs[slot], mixed[off:off + L]])
            conv[off:off + L] = (xs.unfold(0, Kc, 1) * cw).sum(-1)
            cs[slot] = xs[-(Kc - 1):]
            off += L
        if T > P:
            ds = extra["decode_slots"][: T - P].long()
            win = torch.cat([cs.index_select(0, ds), mixed[P:, None]], 1)  # [Dn, Kc, cd]
            conv[P:] = (win * cw.t()).sum(1)
            cs.index_copy_(0, ds, win[:, 1:])
        conv = F.silu(conv)
        q = _l2n(conv[:, :self.kd].view(T, Hk, dk)) * (dk ** -0.5)
        k = _l2n(conv[:, self.kd:2 * self.kd].view(T, Hk, dk))
        v = conv[:, 2 * self.kd:].reshape(T, Hv, dv)
        if Hv != Hk:
            q, k = q.repeat_interleave(Hv // Hk, 1), k.repeat_interleave(Hv // Hk, 1)
        beta = torch.sigmoid(b)
        g = -torch.exp(w[p + "A_log"]) * F.softplus(a + w[p + "dt_bias"])
        core = torch.empty(T, Hv, dv, device=x.device)
        ss = self.ssm_state[li]
        off = 0
        for s_i, L in enumerate(fb.prefill_qlen):
            slot = extra["prefill_slots"][s_i]
            o, S = gdn_chunk_prefill(q[off:off + L], k[off:off + L], v[off:off + L], g[off:off + L],
                                     beta[off:off + L], ss[slot])
            core[off:off + L] = o
            ss[slot] = S
            off += L
        if T > P:
            ds = extra["decode_slots"][: T - P]
            if x.is_cuda:
                ops.native().gdn_decode(q[P:].contiguous(), k[P:].contiguous(), v[P:].contiguous(),
                                        g[P:].contiguous(), beta[P:].contiguous(), ss, ds, core[P:])
            else:
                dl = ds.long()
                o, S = gdn_recurrent_step(q[P:], k[P:], v[P:], g[P:], beta[P:], ss.index_select(0, dl))
                core[P:] = o
                ss.index_copy_(0, dl, S)
        # gated RMSNorm per value head: w * norm(o) (rounded like the HF module) * silu(z)
        y = core * torch.rsqrt(core.pow(2).mean(-1, keepdim=True) + c.rms_eps)
        y = w[p + "gnorm"] * y.to(self.dtype)
        y = (y.float() * F.silu(z.view(T, Hv, dv).float())).to(self.dtype)
        return ops.linear(y.view(T, vd), w[p + "out"])

    def _mlp(self, x, i):
        c, w, p = self.cfg, self.w, f"l{i}."
        if not c.is_moe(i):
            return ops.linear(ops.linear(x, w[p + "gate_up"], act="swiglu"), w[p + "down"])
        T, E, k = x.shape[0], c.num_experts, c.top_k
        logits = ops.linear(x, w[p + "router"], out_dtype=torch.float32)
        ids, wts = ops.moe_route(logits[:, :E].contiguous(), k, c.norm_topk_prob)
        a_rows, offs, pos = ops.moe_dispatch(ids, E)
        h1 = ops.moe_gemm(x, a_rows, w[p + "w13"], offs, T * k, swiglu=True)
        y = ops.moe_gemm(h1, None, w[p + "w2"], offs, T * k, swiglu=False)
        moe = ops.moe_combine(y, pos, wts, None)
        sh = ops.linear(ops.linear(x, w[p + "sh_gate_up"], act="swiglu"), w[p + "sh_down"])
        return (moe.float() + torch.sigmoid(logits[:, E:E + 1]) * sh.float()).to(self.dtype)

    def forward(self, fb: ForwardBatch, kv, decode_ws=None) -> torch.Tensor:
        """Returns fp32 logits [len(sample_rows), vocab]."""
        c, w = self.cfg, self.w
        T, P = fb.num_tokens, fb.num_prefill_tokens
        if self.ssm_state is None:
            self._ensure_pool()
        if fb.extra is None:  # direct forward without the engine hook
            self.prepare_batch(fb)
        res = ops.embedding(fb.token_ids, w["embed"], 0, c.vocab_size)
        h = None
        for i in range(c.num_layers):
            p = f"l{i}."
            x = ops.rms_norm(res, w[p + "attn_norm"], c.rms_eps) if h is None else \
                ops.rms_norm(h, w[p + "attn_norm"], c.rms_eps, residual=res)
            if c.layer_types[i] == "full_attention":
                h = self._full_attention(x, i, fb, kv, decode_ws, T, P)
            else:
                h = self._linear_attention(x, i, fb, T, P)
            x = ops.rms_norm(h, w[p + "mlp_norm"], c.rms_eps, residual=res)
            h = self._mlp(x, i)
        if fb.sample_rows is not None:
            h = h.index_select(0, fb.sample_rows)
            res = res.index_select(0, fb.sample_rows)
        x = ops.rms_norm(h, w["norm"], c.rms_eps, residual=res)
        return ops.linear(x, w["lm_head"], out_dtype=torch.float32)[:, : c.vocab_size]
