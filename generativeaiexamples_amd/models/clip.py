"""CLIP dual encoder (NV-CLIP / OpenAI ViT-L/14 geometry) on the gfx950 kernels - the image/text
embedder of the multimodal RAG config (BASELINE config 4; SURVEY S10, W14 "NV-CLIP search", K19).

Vision tower: normalise + im2col patchify kernel -> patch-projection MFMA GEMM (Conv2d(3, D, 14, 14)
as a GEMM against the zero-padded [D, Kp] weight) -> [CLS | patches] + position embedding kernel ->
pre-LN -> L pre-LN transformer layers (QKV GEMM+bias, bidirectional paged flash attention over the
packed batch, O GEMM with bias+residual fused, FC1 GEMM with bias+quick-GELU fused, FC2 GEMM with
bias+residual fused) -> post-LN on CLS -> projection -> L2 normalise.
Text tower: token + position embedding -> causal pre-LN layers -> final LN -> last-token pooling ->
projection. Any linear weight can be swapped for fp8 (``quantize_fp8``), which routes its GEMM to the
block-scaled fp8 MFMA kernel.

The reference consumes NV-CLIP through a NIM endpoint (``/v1/embeddings`` with ``input`` holding text
or ``data:image/...;base64`` strings); :mod:`engine.embedder` exposes this model the same way.
"""
from __future__ import annotations

import base64
import io
import json
import math
import os
from dataclasses import dataclass, field
from typing import Dict, List, Sequence

import torch
import torch.nn.functional as F

from .. import ops
from .common import PackedAttention, quantize_linear_weights_fp8, randn_like_

CLIP_MEAN = (0.48145466, 0.4578275, 0.40821073)
CLIP_STD = (0.26862954, 0.26130258, 0.27577711)


@dataclass
class TowerConfig:
    hidden_size: int
    num_layers: int
    num_heads: int
    intermediate_size: int
    ln_eps: float = 1e-5

    @property
    def head_dim(self) -> int:
        return self.hidden_size // self.num_heads


@dataclass
class ClipConfig:
    vision: TowerConfig = field(default_factory=lambda: TowerConfig(1024, 24, 16, 4096))
    text: TowerConfig = field(default_factory=lambda: TowerConfig(768, 12, 12, 3072))
    image_size: int = 224
    patch_size: int = 14
    vocab_size: int = 49408
    max_text_len: int = 77
    projection_dim: int = 768
    name: str = "nvidia/nvclip-vit-l-14"

    @property
    def grid(self) -> int:
        return self.image_size // self.patch_size

    @property
    def num_patches(self) -> int:
        return self.grid * self.grid

    @property
    def patch_k(self) -> int:
        k = 3 * self.patch_size * self.patch_size
        return (k + 127) // 128 * 128

    @staticmethod
    def vit_l_14(**kw):
        return ClipConfig(**kw)

    @staticmethod
    def vit_l_14_336(**kw):
        return ClipConfig(image_size=336, name="openai/clip-vit-large-patch14-336", **kw)

    @staticmethod
    def tiny(**kw):
        base = dict(vision=TowerConfig(128, 2, 2, 256), text=TowerConfig(128, 2, 2, 256), image_size=56,
                    vocab_size=1024, projection_dim=128, name="tiny-clip")
        base.update(kw)
        return ClipConfig(**base)

    @staticmethod
    def from_hf(path: str) -> "ClipConfig":
        with open(os.path.join(path, "config.json")) as f:
            c = json.load(f)
        v, t = c["vision_config"], c["text_config"]
        return ClipConfig(
            vision=TowerConfig(v["hidden_size"], v["num_hidden_layers"], v["num_attention_heads"],
                               v["intermediate_size"], v.get("layer_norm_eps", 1e-5)),
            text=TowerConfig(t["hidden_size"], t["num_hidden_layers"], t["num_attention_heads"],
                             t["intermediate_size"], t.get("layer_norm_eps", 1e-5)),
            image_size=v["image_size"], patch_size=v["patch_size"], vocab_size=t["vocab_size"],
            max_text_len=t.get("max_position_embeddings", 77), projection_dim=c.get("projection_dim", 768),
            name=os.path.basename(path.rstrip("/")))


class ClipModel:
    def __init__(self, cfg: ClipConfig, device=None, dtype=torch.bfloat16):
        self.cfg = cfg
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        self.dtype = dtype
        self.w: Dict[str, torch.Tensor] = {}
        c, d = cfg, self.device
        e = lambda *s: torch.empty(*s, device=d, dtype=dtype)  # noqa: E731
        V, T = c.vision, c.text
        self.w["v.patch"] = e(V.hidden_size, c.patch_k)
        self.w["v.cls"] = e(V.hidden_size)
        self.w["v.pos"] = e(c.num_patches + 1, V.hidden_size)
        self.w["v.pre_ln_w"], self.w["v.pre_ln_b"] = e(V.hidden_size), e(V.hidden_size)
        self.w["v.post_ln_w"], self.w["v.post_ln_b"] = e(V.hidden_size), e(V.hidden_size)
        self.w["v.proj"] = e(c.projection_dim, V.hidden_size)
        self.w["t.tok"] = e(c.vocab_size, T.hidden_size)
        self.w["t.pos"] = e(c.max_text_len, T.hidden_size)
        self.w["t.final_ln_w"], self.w["t.final_ln_b"] = e(T.hidden_size), e(T.hidden_size)
        self.w["t.proj"] = e(c.projection_dim, T.hidden_size)
        for tw, tc in (("v", V), ("t", T)):
            D, I = tc.hidden_size, tc.intermediate_size
            for i in range(tc.num_layers):
                p = f"{tw}{i}."
                self.w[p + "ln1_w"], self.w[p + "ln1_b"] = e(D), e(D)
                self.w[p + "qkv"], self.w[p + "qkv_b"] = e(3 * D, D), e(3 * D)
                self.w[p + "o"], self.w[p + "o_b"] = e(D, D), e(D)
                self.w[p + "ln2_w"], self.w[p + "ln2_b"] = e(D), e(D)
                self.w[p + "fc1"], self.w[p + "fc1_b"] = e(I, D), e(I)
                self.w[p + "fc2"], self.w[p + "fc2_b"] = e(D, I), e(D)
        self.logit_scale = math.log(100.0)
        self.mean = torch.tensor(CLIP_MEAN, dtype=torch.float32, device=d)
        self.inv_std = 1.0 / torch.tensor(CLIP_STD, dtype=torch.float32, device=d)

    # ------------------------------------------------------------------ weights
    def random_init(self, seed: int = 0):
        s = seed * 1000
        for k, t in self.w.items():
            if k.endswith("_w") and "ln" in k:
                t.fill_(1.0)
            elif k.endswith("_b"):
                t.zero_()
            elif k in ("v.cls", "v.pos", "t.tok", "t.pos"):
                randn_like_(t, s, 0.02)
            else:
                randn_like_(t, s, 1.0 / math.sqrt(t.shape[1]))
            s += 1
        self.w["v.patch"][:, 3 * self.cfg.patch_size ** 2:].zero_()
        return self

    def load_hf_state(self, sd: Dict[str, torch.Tensor]):
        c = self.cfg

        def put(name, t):
            self.w[name].copy_(t.to(self.dtype))

        pw = sd["vision_model.embeddings.patch_embedding.weight"].reshape(c.vision.hidden_size, -1)
        self.w["v.patch"].zero_()
        self.w["v.patch"][:, : pw.shape[1]].copy_(pw.to(self.dtype))
        put("v.cls", sd["vision_model.embeddings.class_embedding"])
        put("v.pos", sd["vision_model.embeddings.position_embedding.weight"])
        put("v.pre_ln_w", sd["vision_model.pre_layrnorm.weight"])
        put("v.pre_ln_b", sd["vision_model.pre_layrnorm.bias"])
        put("v.post_ln_w", sd["vision_model.post_layernorm.weight"])
        put("v.post_ln_b", sd["vision_model.post_layernorm.bias"])
        put("v.proj", sd["visual_projection.weight"])
        put("t.tok", sd["text_model.embeddings.token_embedding.weight"])
        put("t.pos", sd["text_model.embeddings.position_embedding.weight"])
        put("t.final_ln_w", sd["text_model.final_layer_norm.weight"])
        put("t.final_ln_b", sd["text_model.final_layer_norm.bias"])
        put("t.proj", sd["text_projection.weight"])
        if "logit_scale" in sd:
            self.logit_scale = float(sd["logit_scale"])
        for tw, tc, hp in (("v", c.vision, "vision_model"), ("t", c.text, "text_model")):
            for i in range(tc.num_layers):
                p, h = f"{tw}{i}.", f"{hp}.encoder.layers.{i}."
                put(p + "qkv", torch.cat([sd[h + f"self_attn.{n}_proj.weight"] for n in "qkv"]))
                put(p + "qkv_b", torch.cat([sd[h + f"self_attn.{n}_proj.bias"] for n in "qkv"]))
                put(p + "o", sd[h + "self_attn.out_proj.weight"])
                put(p + "o_b", sd[h + "self_attn.out_proj.bias"])
                for ln in ("1", "2"):
                    put(p + f"ln{ln}_w", sd[h + f"layer_norm{ln}.weight"])
                    put(p + f"ln{ln}_b", sd[h + f"layer_norm{ln}.bias"])
                for fc in ("fc1", "fc2"):
                    put(p + fc, sd[h + f"mlp.{fc}.weight"])
                    put(p + fc + "_b", sd[h + f"mlp.{fc}.bias"])
        return self

    def quantize_fp8(self, towers: str = "vt") -> int:
        """fp8 (e4m3fn, per-channel) weights for every transformer linear of the given towers."""
        keys = [k for k in self.w if k[0] in towers and k.split(".")[-1] in ("qkv", "o", "fc1", "fc2")]
        return quantize_linear_weights_fp8(self.w, keys)

    # ------------------------------------------------------------------ preprocessing
    def preprocess(self, images: Sequence) -> torch.Tensor:
        """PIL images / HWC uint8 arrays / base64 data-URIs / [C,H,W] tensors -> [B, 3, S, S] fp32 in [0, 1]
        (shortest side resized to S bicubic + antialias, centre crop; normalisation is fused into the
        patchify kernel)."""
        S = self.cfg.image_size
        out = []
        for im in images:
            t = _to_chw_float(im).to(self.device)
            _, h, w = t.shape
            sc = S / min(h, w)
            nh, nw = max(S, round(h * sc)), max(S, round(w * sc))
            t = F.interpolate(t[None], size=(nh, nw), mode="bicubic", antialias=True, align_corners=False)[0]
            y0, x0 = (nh - S) // 2, (nw - S) // 2
            out.append(t[:, y0:y0 + S, x0:x0 + S].clamp(0, 1))
        return torch.stack(out).contiguous()

    # ------------------------------------------------------------------ forward
    def _layers(self, tw: str, tc: TowerConfig, h: torch.Tensor, attn: PackedAttention) -> torch.Tensor:
        w, scale = self.w, 1.0 / math.sqrt(tc.head_dim)
        for i in range(tc.num_layers):
            p = f"{tw}{i}."
            x = ops.layer_norm(h, w[p + "ln1_w"], w[p + "ln1_b"], tc.ln_eps)
            qkv = ops.linear(x, w[p + "qkv"], bias=w[p + "qkv_b"])
            a = attn(qkv, scale)
            h = ops.linear(a, w[p + "o"], bias=w[p + "o_b"], residual=h)
            x = ops.layer_norm(h, w[p + "ln2_w"], w[p + "ln2_b"], tc.ln_eps)
            f = ops.linear(x, w[p + "fc1"], bias=w[p + "fc1_b"], act="quick_gelu")
            h = ops.linear(f, w[p + "fc2"], bias=w[p + "fc2_b"], residual=h)
        return h

    @torch.no_grad()
    def vision_hidden(self, pixels: torch.Tensor) -> torch.Tensor:
        """pixels [B, 3, S, S] fp32 in [0, 1] -> last hidden state [B * (NP + 1), D] (pre post-LN)."""
        c, w = self.cfg, self.w
        B, V = pixels.shape[0], c.vision
        x = ops.patchify(pixels, c.patch_size, self.mean, self.inv_std, c.patch_k)
        pe = ops.linear(x, w["v.patch"])
        h = ops.vit_embed(pe, w["v.cls"], w["v.pos"], B)
        h = ops.layer_norm(h, w["v.pre_ln_w"], w["v.pre_ln_b"], V.ln_eps)
        attn = PackedAttention([c.num_patches + 1] * B, V.num_heads, V.head_dim, pixels.device, self.dtype)
        return self._layers("v", V, h, attn)

    @torch.no_grad()
    def encode_image(self, pixels: torch.Tensor, normalize: bool = True) -> torch.Tensor:
        """[B, 3, S, S] -> image embeddings [B, projection_dim] fp32."""
        c, w = self.cfg, self.w
        B = pixels.shape[0]
        h = self.vision_hidden(pixels)
        cls = h.view(B, c.num_patches + 1, -1)[:, 0]
        x = ops.layer_norm(cls.contiguous(), w["v.post_ln_w"], w["v.post_ln_b"], c.vision.ln_eps)
        e = ops.linear(x, w["v.proj"], out_dtype=torch.float32)
        return F.normalize(e, dim=-1) if normalize else e

    @torch.no_grad()
    def encode_text(self, token_lists: List[List[int]], normalize: bool = True) -> torch.Tensor:
        """Token id lists (truncated to max_text_len, EOT last) -> text embeddings [B, projection_dim]."""
        c, w, T = self.cfg, self.w, self.cfg.text
        toks = [t[: c.max_text_len] if t else [0] for t in token_lists]
        lens = [len(t) for t in toks]
        ids = torch.tensor([x for t in toks for x in t], dtype=torch.int32).to(self.device, non_blocking=True)
        attn = PackedAttention(lens, T.num_heads, T.head_dim, self.device, self.dtype, causal=True)
        h = ops.embedding(ids, w["t.tok"])
        h = (h.float() + w["t.pos"][attn.positions.long()].float()).to(self.dtype)
        h = self._layers("t", T, h, attn)
        last = attn.cu_q[1:].long() - 1
        x = ops.layer_norm(h.index_select(0, last), w["t.final_ln_w"], w["t.final_ln_b"], T.ln_eps)
        e = ops.linear(x, w["t.proj"], out_dtype=torch.float32)
        return F.normalize(e, dim=-1) if normalize else e

    # ------------------------------------------------------------------ fp32 reference (tests)
    @torch.no_grad()
    def reference_encode_image(self, pixels: torch.Tensor) -> torch.Tensor:
        c = self.cfg
        V = c.vision
        wf = {k: (v.dequantize(torch.float32) if isinstance(v, ops.Fp8Weight) else v.float()).cpu()
              for k, v in self.w.items()}
        px = pixels.float().cpu()
        B = px.shape[0]
        x = (px - torch.tensor(CLIP_MEAN).view(1, 3, 1, 1)) / torch.tensor(CLIP_STD).view(1, 3, 1, 1)
        P = c.patch_size
        conv_w = wf["v.patch"][:, : 3 * P * P].reshape(V.hidden_size, 3, P, P)
        pe = F.conv2d(x, conv_w, stride=P).flatten(2).transpose(1, 2)  # [B, NP, D]
        h = torch.cat([wf["v.cls"].view(1, 1, -1).expand(B, 1, -1), pe], 1) + wf["v.pos"][None]
        h = F.layer_norm(h, (V.hidden_size,), wf["v.pre_ln_w"], wf["v.pre_ln_b"], V.ln_eps)
        H, hd = V.num_heads, V.head_dim
        for i in range(V.num_layers):
            p = f"v{i}."
            x = F.layer_norm(h, (V.hidden_size,), wf[p + "ln1_w"], wf[p + "ln1_b"], V.ln_eps)
            qkv = x @ wf[p + "qkv"].t() + wf[p + "qkv_b"]
            q, k, v = qkv.view(B, -1, 3, H, hd).permute(2, 0, 3, 1, 4)
            a = F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(B, -1, H * hd)
            h = h + a @ wf[p + "o"].t() + wf[p + "o_b"]
            x = F.layer_norm(h, (V.hidden_size,), wf[p + "ln2_w"], wf[p + "ln2_b"], V.ln_eps)
            f = x @ wf[p + "fc1"].t() + wf[p + "fc1_b"]
            f = f * torch.sigmoid(1.702 * f)
            h = h + f @ wf[p + "fc2"].t() + wf[p + "fc2_b"]
        x = F.layer_norm(h[:, 0], (V.hidden_size,), wf["v.post_ln_w"], wf["v.post_ln_b"], V.ln_eps)
        return F.normalize(x @ wf["v.proj"].t(), dim=-1)


def _to_chw_float(im) -> torch.Tensor:
    if isinstance(im, str):
        data = im.split(",", 1)[1] if im.startswith("data:") else im
        im = base64.b64decode(data)
    if isinstance(im, (bytes, bytearray)):
        from PIL import Image
        im = Image.open(io.BytesIO(im))
    if hasattr(im, "convert"):  # PIL
        import numpy as np
        im = np.asarray(im.convert("RGB"))
    if isinstance(im, torch.Tensor):
        t = im.float()
        return t / 255.0 if t.max() > 1.5 else t
    t = torch.from_numpy(im.copy())  # HWC uint8
    if t.dim() == 2:
        t = t[..., None].expand(-1, -1, 3)
    return t.permute(2, 0, 1).float() / 255.0
