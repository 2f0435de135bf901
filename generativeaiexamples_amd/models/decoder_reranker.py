"""Decoder-based cross-encoder reranker: the NV-RerankQA-Mistral-4B-v3 class (the
``ranking-ms`` service of RAG/examples/local_deploy/docker-compose-nim-ms.yaml:58-82, BASELINE config 3
"NV-Rerank-QA cross-encoder").

Geometry: a Mistral-7B decoder truncated to its first 16 layers (hidden 4096, 32 query / 8 KV heads,
SwiGLU 14336), run with *bidirectional* attention over the packed (query, passage) pair prompt
``"question:{q} \\n \\n passage:{p}"``, mean-pooled over the pair's tokens, then a linear head -> one
relevance logit. ~3.5B parameters.

Forward (packed varlen, no padding): embedding kernel -> per layer: fused add+RMSNorm -> QKV GEMM
-> RoPE + K/V scatter into a transient paged cache -> bidirectional GQA flash attention (prefill
kernel, causal off) -> O GEMM -> fused add+RMSNorm -> gate/up GEMM with fused SwiGLU -> down GEMM
-> final RMSNorm -> masked mean-pool kernel -> score GEMV.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List

import torch

from .. import ops
from .common import PackedAttention, randn_like_
from .llama import LlamaConfig


@dataclass
class DecoderRerankerConfig(LlamaConfig):
    max_length: int = 512
    pooling: str = "mean"

    @staticmethod
    def nv_rerankqa_mistral_4b(**kw):
        return DecoderRerankerConfig(name="nvidia/nv-rerankqa-mistral-4b-v3", vocab_size=32000, num_layers=16,
                                     rope_theta=1e6, max_position=4096, bos_token_id=1, eos_token_ids=(2,), **kw)

    @staticmethod
    def tiny(**kw):
        base = dict(vocab_size=512, hidden_size=256, intermediate_size=512, num_layers=2, num_heads=4,
                    num_kv_heads=2, head_dim=64, max_position=1024, bos_token_id=1, eos_token_ids=(2,),
                    name="tiny-decoder-reranker")
        base.update(kw)
        return DecoderRerankerConfig(**base)


class DecoderRerankerModel:
    def __init__(self, cfg: DecoderRerankerConfig, device=None, dtype=torch.bfloat16):
        self.cfg = cfg
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        self.dtype = dtype
        c, d = cfg, self.device
        D, hd = c.hidden_size, c.head_dim
        e = lambda *s: torch.empty(*s, device=d, dtype=dtype)  # noqa: E731
        self.w: Dict[str, torch.Tensor] = {"embed": e(c.vocab_size, D), "norm": e(D)}
        for i in range(c.num_layers):
            p = f"l{i}."
            self.w[p + "attn_norm"] = e(D)
            self.w[p + "qkv"] = e((c.num_heads + 2 * c.num_kv_heads) * hd, D)
            self.w[p + "o"] = e(D, c.num_heads * hd)
            self.w[p + "mlp_norm"] = e(D)
            self.w[p + "gate_up"] = e(2 * c.intermediate_size, D)
            self.w[p + "down"] = e(D, c.intermediate_size)
        # score head padded to 16 rows so it runs on the MFMA GEMM; row 0 is the logit
        self.w["score"] = e(16, D)
        self.scale = 1.0 / math.sqrt(hd)
        self.cos_sin = ops.rope_cos_sin(c.max_position, hd, c.rope_theta, c.rope_scaling, device=d)

    def random_init(self, seed: int = 0):
        s = seed * 1000
        for k, t in self.w.items():
            if k.endswith("norm"):
                t.fill_(1.0)
            else:
                randn_like_(t, s, 0.02 if k == "embed" else 1.0 / math.sqrt(t.shape[1]))
            s += 1
        return self

    def load_hf_state(self, sd: Dict[str, torch.Tensor]):
        c = self.cfg
        pre = "model." if any(k.startswith("model.") for k in sd) else ""

        def put(name, t):
            self.w[name].copy_(t.to(self.dtype))

        put("embed", sd[pre + "embed_tokens.weight"])
        put("norm", sd[pre + "norm.weight"])
        for i in range(c.num_layers):
            p, h = f"l{i}.", f"{pre}layers.{i}."
            put(p + "attn_norm", sd[h + "input_layernorm.weight"])
            put(p + "mlp_norm", sd[h + "post_attention_layernorm.weight"])
            put(p + "qkv", torch.cat([sd[h + f"self_attn.{n}_proj.weight"] for n in "qkv"]))
            put(p + "o", sd[h + "self_attn.o_proj.weight"])
            self.w[p + "gate_up"].copy_(ops.interleave_gate_up(sd[h + "mlp.gate_proj.weight"],
                                                               sd[h + "mlp.up_proj.weight"]).to(self.dtype))
            put(p + "down", sd[h + "mlp.down_proj.weight"])
        head = next(v for k, v in sd.items() if k.endswith("score.weight") or k.endswith("classifier.weight"))
        self.w["score"].zero_()
        self.w["score"][: head.shape[0]].copy_(head.to(self.dtype))
        return self

    @torch.no_grad()
    def score(self, ids: torch.Tensor, cu_seqlens: torch.Tensor, seq_lens: List[int]) -> torch.Tensor:
        """Packed pair tokens [T] -> relevance logits [B] fp32."""
        c, w = self.cfg, self.w
        attn = PackedAttention(seq_lens, c.num_heads, c.head_dim, ids.device, self.dtype,
                               num_kv_heads=c.num_kv_heads, cos_sin=self.cos_sin)
        res = ops.embedding(ids, w["embed"])
        h = None
        for i in range(c.num_layers):
            p = f"l{i}."
            x = ops.rms_norm(res, w[p + "attn_norm"], c.rms_eps) if h is None else \
                ops.rms_norm(h, w[p + "attn_norm"], c.rms_eps, residual=res)
            a = attn(ops.linear(x, w[p + "qkv"]), self.scale)
            h = ops.linear(a, w[p + "o"])
            x = ops.rms_norm(h, w[p + "mlp_norm"], c.rms_eps, residual=res)
            h = ops.linear(ops.linear(x, w[p + "gate_up"], act="swiglu"), w[p + "down"])
        x = ops.rms_norm(h, w["norm"], c.rms_eps, residual=res)
        pooled = ops.pool(x, cu_seqlens, c.pooling, normalize=False)  # fp32 [B, D]
        return ops.linear(pooled.to(self.dtype), w["score"], out_dtype=torch.float32)[:, 0]

    @torch.no_grad()
    def reference_score(self, ids: torch.Tensor, seq_lens: List[int]) -> torch.Tensor:
        """Dense fp32 reference (bidirectional attention, mean pool) for tests."""
        import torch.nn.functional as F
        c = self.cfg
        wf = {k: v.float().cpu() for k, v in self.w.items()}
        hd, H, Hkv = c.head_dim, c.num_heads, c.num_kv_heads
        out, o = [], 0
        cs = self.cos_sin.float().cpu()

        def rms(v, g):
            return v * torch.rsqrt(v.pow(2).mean(-1, keepdim=True) + c.rms_eps) * g

        for n in seq_lens:
            t = ids[o:o + n].long().cpu()
            o += n
            x = wf["embed"][t]
            cos, sin = cs[:n, : hd // 2], cs[:n, hd // 2:]

            def rope(v):
                a, b = v[..., : hd // 2], v[..., hd // 2:]
                return torch.cat([a * cos[:, None] - b * sin[:, None], b * cos[:, None] + a * sin[:, None]], -1)

            for i in range(c.num_layers):
                p = f"l{i}."
                q, k, v = (rms(x, wf[p + "attn_norm"]) @ wf[p + "qkv"].t()).split([H * hd, Hkv * hd, Hkv * hd], -1)
                q, k, v = rope(q.view(n, H, hd)), rope(k.view(n, Hkv, hd)), v.view(n, Hkv, hd)
                k, v = k.repeat_interleave(H // Hkv, 1), v.repeat_interleave(H // Hkv, 1)
                a = F.scaled_dot_product_attention(q.transpose(0, 1), k.transpose(0, 1), v.transpose(0, 1))
                x = x + a.transpose(0, 1).reshape(n, -1) @ wf[p + "o"].t()
                y = ops.reference.linear(rms(x, wf[p + "mlp_norm"]), wf[p + "gate_up"], act="swiglu",
                                         out_dtype=torch.float32)
                x = x + y @ wf[p + "down"].t()
            out.append((rms(x, wf["norm"]).mean(0) @ wf["score"].t())[0])
        return torch.stack(out)
