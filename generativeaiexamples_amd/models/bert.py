"""BERT-family bidirectional encoders on the gfx950 kernels: E5 embedders and cross-encoder rerankers.

Replaces the embedding NIM (``nv-embedqa-e5-v5``, 1024-d E5-large-class encoder),
the HF sentence-transformers embedder (S11, ``utils.py:406-444``) and the Triton MiniLM service
(S8), plus BERT-style cross-encoder rerankers (S3 analogue).

Forward over a varlen batch (no padding): word+position+type embedding -> LayerNorm, then per
layer: QKV GEMM(+bias) -> K/V scattered into a transient paged cache by the RoPE/KV kernel with
rotation disabled -> bidirectional paged flash attention -> O GEMM with bias+residual fused ->
LayerNorm (post-LN) -> FFN-up GEMM with bias+GELU fused -> FFN-down GEMM with bias+residual fused
-> LayerNorm. Pooling (mean / CLS) + L2-normalise in one kernel.
"""
from __future__ import annotations

import json
import math
import os
from dataclasses import dataclass
from typing import Dict, List, Optional

import torch

from .. import ops
from .common import PackedAttention, randn_like_


@dataclass
class BertConfig:
    vocab_size: int = 30522
    hidden_size: int = 1024
    intermediate_size: int = 4096
    num_layers: int = 24
    num_heads: int = 16
    max_position: int = 512
    type_vocab_size: int = 2
    ln_eps: float = 1e-12
    pooling: str = "mean"          # E5: average pool
    normalize: bool = True
    num_labels: int = 0            # >0: cross-encoder classification head on CLS
    name: str = "bert"

    @property
    def head_dim(self) -> int:
        return self.hidden_size // self.num_heads

    @property
    def head_dim_padded(self) -> int:
        """Attention kernels run D = 64 / 128: smaller heads (MiniLM: 32) are zero-padded inside the
        QKV / O weights (padded q/k dims add 0 to the scores, padded v dims feed zero O columns)."""
        return 64 if self.head_dim <= 64 else 128

    @staticmethod
    def e5_large_v2(**kw):
        return BertConfig(name="intfloat/e5-large-v2", **kw)

    @staticmethod
    def e5_base_v2(**kw):
        return BertConfig(name="intfloat/e5-base-v2", hidden_size=768, intermediate_size=3072, num_layers=12,
                          num_heads=12, **kw)

    @staticmethod
    def minilm_l6_v2(**kw):
        # sentence-transformers/all-MiniLM-L6-v2: the reference's Triton streaming-ingest embedder (S8)
        return BertConfig(name="sentence-transformers/all-MiniLM-L6-v2", hidden_size=384, intermediate_size=1536,
                          num_layers=6, num_heads=12, **kw)

    @staticmethod
    def bge_reranker_large(**kw):
        # XLM-R-large-class cross-encoder geometry; CLS -> 1 logit
        return BertConfig(name="bge-reranker-large", num_labels=1, pooling="cls", normalize=False, **kw)

    @staticmethod
    def tiny(**kw):
        base = dict(vocab_size=2048, hidden_size=256, intermediate_size=512, num_layers=2, num_heads=4,
                    max_position=512, name="tiny-bert")
        base.update(kw)
        return BertConfig(**base)

    @staticmethod
    def from_hf(path: str) -> "BertConfig":
        with open(os.path.join(path, "config.json")) as f:
            c = json.load(f)
        return BertConfig(vocab_size=c["vocab_size"], hidden_size=c["hidden_size"],
                          intermediate_size=c["intermediate_size"], num_layers=c["num_hidden_layers"],
                          num_heads=c["num_attention_heads"], max_position=c.get("max_position_embeddings", 512),
                          type_vocab_size=c.get("type_vocab_size", 2), ln_eps=c.get("layer_norm_eps", 1e-12),
                          num_labels=len(c.get("id2label", {})) if "ForSequenceClassification" in str(c.get("architectures")) else 0,
                          name=os.path.basename(path.rstrip("/")))


class BertModel:
    def __init__(self, cfg: BertConfig, device=None, dtype=torch.bfloat16):
        self.cfg = cfg
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        self.dtype = dtype
        self.scale = 1.0 / math.sqrt(cfg.head_dim)
        self.w: Dict[str, torch.Tensor] = {}
        c, d, dt = cfg, self.device, dtype
        D = c.hidden_size
        e = lambda *s: torch.empty(*s, device=d, dtype=dt)  # noqa: E731
        self.w["word"] = e(c.vocab_size, D)
        self.w["pos"] = e(c.max_position, D)
        self.w["type"] = e(c.type_vocab_size, D)
        self.w["emb_ln_w"], self.w["emb_ln_b"] = e(D), e(D)
        for i in range(c.num_layers):
            p = f"l{i}."
            HP = c.num_heads * c.head_dim_padded
            self.w[p + "qkv"], self.w[p + "qkv_b"] = e(3 * HP, D), e(3 * HP)
            self.w[p + "o"], self.w[p + "o_b"] = e(D, HP), e(D)
            self.w[p + "ln1_w"], self.w[p + "ln1_b"] = e(D), e(D)
            self.w[p + "up"], self.w[p + "up_b"] = e(c.intermediate_size, D), e(c.intermediate_size)
            self.w[p + "down"], self.w[p + "down_b"] = e(D, c.intermediate_size), e(D)
            self.w[p + "ln2_w"], self.w[p + "ln2_b"] = e(D), e(D)
        if c.num_labels:
            # classifier padded to 16 rows so the MFMA GEMM path applies; only num_labels are used
            self.w["cls_dense"], self.w["cls_dense_b"] = e(D, D), e(D)
            self.w["cls_out"], self.w["cls_out_b"] = e(16, D), e(16)

    def _pad_heads(self, t: torch.Tensor, rows: bool) -> torch.Tensor:
        """[3*H*hd, D] / [3*H*hd] (rows=True) or [D, H*hd] (rows=False) -> zero-padded head dims."""
        c = self.cfg
        hd, hp, H = c.head_dim, c.head_dim_padded, c.num_heads
        if hp == hd:
            return t
        if rows:
            src = t.reshape(3, H, hd, *t.shape[1:])
            out = t.new_zeros(3, H, hp, *t.shape[1:])
            out[:, :, :hd] = src
            return out.reshape(3 * H * hp, *t.shape[1:])
        src = t.reshape(t.shape[0], H, hd)
        out = t.new_zeros(t.shape[0], H, hp)
        out[:, :, :hd] = src
        return out.reshape(t.shape[0], H * hp)

    def random_init(self, seed: int = 0):
        s = seed * 1000
        for k, t in self.w.items():
            if k.endswith("ln_w") or k.endswith("ln1_w") or k.endswith("ln2_w"):
                t.fill_(1.0)
            elif k.endswith("_b") or k.endswith("ln_b") or k.endswith("ln1_b") or k.endswith("ln2_b"):
                t.zero_()
            elif k in ("word", "pos", "type"):
                randn_like_(t, s, 0.02)
            else:
                randn_like_(t, s, 1.0 / math.sqrt(t.shape[1]))
            s += 1
        c = self.cfg
        if c.head_dim_padded != c.head_dim:
            hd, H = c.head_dim, c.num_heads
            for i in range(c.num_layers):
                p = f"l{i}."
                self.w[p + "qkv"].view(3, H, -1, c.hidden_size)[:, :, hd:].zero_()
                self.w[p + "qkv_b"].view(3, H, -1)[:, :, hd:].zero_()
                self.w[p + "o"].view(c.hidden_size, H, -1)[:, :, hd:].zero_()
        return self

    def load_hf_state(self, sd: Dict[str, torch.Tensor]):
        c = self.cfg
        pre = "bert." if any(k.startswith("bert.") for k in sd) else ""

        def g(n):
            return sd[pre + n]

        def put(name, t):
            self.w[name].copy_(t.to(self.dtype))

        put("word", g("embeddings.word_embeddings.weight"))
        put("pos", g("embeddings.position_embeddings.weight"))
        put("type", g("embeddings.token_type_embeddings.weight"))
        put("emb_ln_w", g("embeddings.LayerNorm.weight"))
        put("emb_ln_b", g("embeddings.LayerNorm.bias"))
        for i in range(c.num_layers):
            p, h = f"l{i}.", f"encoder.layer.{i}."
            put(p + "qkv", self._pad_heads(torch.cat([g(h + f"attention.self.{n}.weight")
                                                     for n in ("query", "key", "value")]), True))
            put(p + "qkv_b", self._pad_heads(torch.cat([g(h + f"attention.self.{n}.bias")
                                                       for n in ("query", "key", "value")]), True))
            put(p + "o", self._pad_heads(g(h + "attention.output.dense.weight"), False))
            put(p + "o_b", g(h + "attention.output.dense.bias"))
            put(p + "ln1_w", g(h + "attention.output.LayerNorm.weight"))
            put(p + "ln1_b", g(h + "attention.output.LayerNorm.bias"))
            put(p + "up", g(h + "intermediate.dense.weight"))
            put(p + "up_b", g(h + "intermediate.dense.bias"))
            put(p + "down", g(h + "output.dense.weight"))
            put(p + "down_b", g(h + "output.dense.bias"))
            put(p + "ln2_w", g(h + "output.LayerNorm.weight"))
            put(p + "ln2_b", g(h + "output.LayerNorm.bias"))
        if c.num_labels and "classifier.weight" in sd:
            w = sd["classifier.weight"]
            self.w["cls_out"].zero_()
            self.w["cls_out"][: w.shape[0]].copy_(w.to(self.dtype))
            self.w["cls_out_b"].zero_()
            self.w["cls_out_b"][: w.shape[0]].copy_(sd["classifier.bias"].to(self.dtype))
        return self

    def _unpad_heads(self, t: torch.Tensor, rows: bool) -> torch.Tensor:
        c = self.cfg
        hd, hp, H = c.head_dim, c.head_dim_padded, c.num_heads
        if hp == hd:
            return t
        if rows:
            return t.reshape(3, H, hp, *t.shape[1:])[:, :, :hd].reshape(3 * H * hd, *t.shape[1:])
        return t.reshape(t.shape[0], H, hp)[:, :, :hd].reshape(t.shape[0], H * hd)

    def export_hf_state(self) -> Dict[str, torch.Tensor]:
        """Inverse of :meth:`load_hf_state` (HF ``BertModel`` names, padded head dims removed)."""
        c, w = self.cfg, self.w
        sd = {"embeddings.word_embeddings.weight": w["word"], "embeddings.position_embeddings.weight": w["pos"],
              "embeddings.token_type_embeddings.weight": w["type"], "embeddings.LayerNorm.weight": w["emb_ln_w"],
              "embeddings.LayerNorm.bias": w["emb_ln_b"]}
        D = c.hidden_size
        for i in range(c.num_layers):
            p, h = f"l{i}.", f"encoder.layer.{i}."
            qkv, qkv_b = self._unpad_heads(w[p + "qkv"], True), self._unpad_heads(w[p + "qkv_b"], True)
            for j, n in enumerate(("query", "key", "value")):
                sd[h + f"attention.self.{n}.weight"] = qkv[j * D:(j + 1) * D]
                sd[h + f"attention.self.{n}.bias"] = qkv_b[j * D:(j + 1) * D]
            sd[h + "attention.output.dense.weight"] = self._unpad_heads(w[p + "o"], False)
            sd[h + "attention.output.dense.bias"] = w[p + "o_b"]
            sd[h + "attention.output.LayerNorm.weight"] = w[p + "ln1_w"]
            sd[h + "attention.output.LayerNorm.bias"] = w[p + "ln1_b"]
            sd[h + "intermediate.dense.weight"] = w[p + "up"]
            sd[h + "intermediate.dense.bias"] = w[p + "up_b"]
            sd[h + "output.dense.weight"] = w[p + "down"]
            sd[h + "output.dense.bias"] = w[p + "down_b"]
            sd[h + "output.LayerNorm.weight"] = w[p + "ln2_w"]
            sd[h + "output.LayerNorm.bias"] = w[p + "ln2_b"]
        return {k: v.detach().clone() for k, v in sd.items()}

    # ---------------------------------------------------------------------------- forward
    def encode_hidden(self, ids: torch.Tensor, cu_seqlens: torch.Tensor, seq_lens: List[int],
                      type_ids: Optional[torch.Tensor] = None, attn: Optional[PackedAttention] = None) -> torch.Tensor:
        """ids [T] int32 (varlen packed), cu_seqlens [B+1] int32 (device), seq_lens host list -> hidden [T, D].
        ``attn``: a prebuilt attention plan (the padded HIP-graph path, :meth:`embed_padded`)."""
        c, w = self.cfg, self.w
        T, D, H, hp = ids.numel(), c.hidden_size, c.num_heads, c.head_dim_padded
        dev = ids.device
        attn = attn if attn is not None else PackedAttention(seq_lens, H, hp, dev, self.dtype)
        pos = attn.positions  # restart at 0 for every sequence
        h = ops.embedding(ids, w["word"])
        h = h + w["pos"][pos.long()]
        h = h + (w["type"][0] if type_ids is None else w["type"][type_ids.long()])
        h = ops.layer_norm(h, w["emb_ln_w"], w["emb_ln_b"], c.ln_eps)
        out = torch.empty(T, H * hp, device=dev, dtype=self.dtype)
        for i in range(c.num_layers):
            p = f"l{i}."
            qkv = ops.linear(h, w[p + "qkv"], bias=w[p + "qkv_b"])
            a = attn(qkv, self.scale, out=out)
            x = ops.linear(a, w[p + "o"], bias=w[p + "o_b"], residual=h)
            h = ops.layer_norm(x, w[p + "ln1_w"], w[p + "ln1_b"], c.ln_eps)
            f = ops.linear(h, w[p + "up"], bias=w[p + "up_b"], act="gelu")
            x = ops.linear(f, w[p + "down"], bias=w[p + "down_b"], residual=h)
            h = ops.layer_norm(x, w[p + "ln2_w"], w[p + "ln2_b"], c.ln_eps)
        return h

    def embed(self, ids, cu_seqlens, seq_lens) -> torch.Tensor:
        """Pooled (and L2-normalised) sentence embeddings, fp32 [B, D]."""
        h = self.encode_hidden(ids, cu_seqlens, seq_lens)
        return ops.pool(h, cu_seqlens, self.cfg.pooling, self.cfg.normalize)

    # ---- fixed-shape query encoder (HIP graphs): B sequences padded to L tokens each
    def embed_padded(self, ids: torch.Tensor, lens: torch.Tensor, attn: PackedAttention, B: int, L: int) -> torch.Tensor:
        """ids [B*L] (sequence b in rows [bL, bL + lens[b]), padding after), lens [B] int32 on the device,
        ``attn`` built for q_lens = [L] * B whose ``ctx`` tensor holds ``lens``: every query row attends to the
        real keys of its sequence only (the kernel masks keys >= ctx), so real rows equal the packed forward;
        pooling runs over the real rows. All shapes are fixed: capturable once per (B, L) bucket."""
        c = self.cfg
        h = self.encode_hidden(ids, attn.cu_q, [L] * B, attn=attn).view(B, L, -1).float()
        if c.pooling == "cls":
            o = h[:, 0]
        elif c.pooling == "last":
            o = h[torch.arange(B, device=h.device), (lens.long() - 1).clamp_min(0)]
        else:
            m = (torch.arange(L, device=h.device)[None, :] < lens[:, None]).float()
            o = (h * m[..., None]).sum(1) / lens.clamp_min(1)[:, None].float()
        if c.normalize:
            o = torch.nn.functional.normalize(o, dim=-1, eps=1e-12)
        return o

    def score(self, ids, cu_seqlens, seq_lens, type_ids=None) -> torch.Tensor:
        """Cross-encoder relevance logits [B] (CLS -> dense+tanh -> classifier)."""
        c, w = self.cfg, self.w
        assert c.num_labels > 0
        h = self.encode_hidden(ids, cu_seqlens, seq_lens, type_ids)
        cls = h.index_select(0, cu_seqlens[:-1].long())
        x = ops.linear(cls, w["cls_dense"], bias=w["cls_dense_b"])
        x = torch.tanh(x.float()).to(self.dtype)
        logits = ops.linear(x, w["cls_out"], bias=w["cls_out_b"], out_dtype=torch.float32)
        return logits[:, 0]
