"""Llama-3.2-Vision (Mllama) on the gfx950 kernels - the multimodal generator of BASELINE config 4
(the reference calls NeVA-22B / DePlot / Nemotron-VL through API endpoints,
RAG/examples/advanced_rag/multimodal_rag/vectorstore/custom_pdf_parser.py:54-64; W12 image_url chat).

Vision encoder (ViT-H/14 class, 560-px tiles, up to 4 tiles per image):
  patchify kernel -> patch GEMM -> + tanh-gated pre-tile embedding -> [CLS | patches] ->
  gated position + tile embedding -> LN -> 32 encoder layers (intermediate outputs of 5 of them kept)
  -> LN -> post-tile embedding -> 8 gated "global" layers -> concat(final, 5 intermediates) [*, 7680]
  -> multimodal projector GEMM -> cross-attention states [tiles * 1601, 4096].
  Head dim 80 is zero-padded to 96 inside the QKV / O weights so attention runs on the D=96 MFMA
  flash-attention kernel (padded q/k dims add 0 to the scores, padded v dims produce 0 columns that
  the zero O-proj columns ignore); the softmax scale stays 1/sqrt(80). The tanh gates of the gated
  layers are folded into the O / FC2 weights at load time, so every layer is the plain fused path.
Text decoder: Llama-3.1-8B geometry with 8 of 40 layers replaced by gated cross-attention layers
  (q_norm / k_norm per head, no RoPE). Each request's image is encoded once when the request is
  registered; its cross K/V for all cross layers is written into a separate paged *cross cache*
  (K/V-only launch of the RoPE/KV kernel with Hq = 0) and every later step - prefill chunks and
  HIP-graph decode steps - attends to it with the same paged prefill / split-KV decode kernels.
  Sequences without an image get a zero row mask (their cross layers contribute nothing), matching
  the reference semantics of skipping cross-attention for text-only input.

Deviation (documented, parity unpinned - no HF checkpoint offline): the vision encoder attends over
the real 1601 tokens of the real tiles only (HF pads each tile to 1608 tokens and pads to 4 tiles,
masking only pad-to-pad pairs).
"""
from __future__ import annotations

import json
import math
import os
from dataclasses import dataclass, field, replace
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

from .. import ops
from .clip import _to_chw_float
from .common import ForwardBatch, PackedAttention, quantize_linear_weights_fp8, randn_like_
from .llama import LlamaConfig, LlamaModel, hf_rope

MLLAMA_MEAN = (0.48145466, 0.4578275, 0.40821073)
MLLAMA_STD = (0.26862954, 0.26130258, 0.27577711)


def supported_aspect_ratios(max_tiles: int) -> List[Tuple[int, int]]:
    """(width_tiles, height_tiles) canvases with w * h <= max_tiles; aspect_ratio_id = index + 1."""
    return [(w, h) for w in range(1, max_tiles + 1) for h in range(1, max_tiles + 1) if w * h <= max_tiles]


@dataclass
class MllamaVisionConfig:
    hidden_size: int = 1280
    num_layers: int = 32
    num_global_layers: int = 8
    num_heads: int = 16
    intermediate_size: int = 5120
    image_size: int = 560
    patch_size: int = 14
    max_num_tiles: int = 4
    intermediate_layers: Tuple[int, ...] = (3, 7, 15, 23, 30)
    ln_eps: float = 1e-5

    @property
    def head_dim(self) -> int:
        return self.hidden_size // self.num_heads

    @property
    def head_dim_padded(self) -> int:
        return 64 if self.head_dim <= 64 else 96 if self.head_dim <= 96 else 128

    @property
    def num_patches(self) -> int:
        return (self.image_size // self.patch_size) ** 2

    @property
    def tokens_per_tile(self) -> int:
        return self.num_patches + 1

    @property
    def output_dim(self) -> int:
        return self.hidden_size * (1 + len(self.intermediate_layers))

    @property
    def patch_k(self) -> int:
        return (3 * self.patch_size ** 2 + 127) // 128 * 128

    @property
    def aspect_ratios(self) -> List[Tuple[int, int]]:
        return supported_aspect_ratios(self.max_num_tiles)


@dataclass
class MllamaConfig:
    text: LlamaConfig = field(default_factory=lambda: LlamaConfig(
        name="meta/llama-3.2-11b-vision-instruct", num_layers=40, max_position=131072,
        rope_scaling={"factor": 8.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
                      "original_max_position_embeddings": 8192}))
    vision: MllamaVisionConfig = field(default_factory=MllamaVisionConfig)
    cross_layers: Tuple[int, ...] = (3, 8, 13, 18, 23, 28, 33, 38)
    image_token_id: int = 128256
    extra_vocab: int = 8  # embed_tokens has vocab_size + 8 rows (<|image|> and reserved ids)
    name: str = "meta/llama-3.2-11b-vision-instruct"

    @staticmethod
    def llama32_11b_vision(**kw):
        return MllamaConfig(**kw)

    @staticmethod
    def tiny(**kw):
        base = dict(text=LlamaConfig.tiny(num_layers=4, max_position=4096),
                    vision=MllamaVisionConfig(hidden_size=128, num_layers=2, num_global_layers=1, num_heads=2,
                                              intermediate_size=256, image_size=56, intermediate_layers=(1,)),
                    cross_layers=(1, 3), image_token_id=511, extra_vocab=0, name="tiny-mllama")
        base.update(kw)
        return MllamaConfig(**base)

    @staticmethod
    def from_hf(path: str) -> "MllamaConfig":
        with open(os.path.join(path, "config.json")) as f:
            c = json.load(f)
        t, v = c["text_config"], c["vision_config"]
        eos = t.get("eos_token_id", 128009)
        text = LlamaConfig(vocab_size=t["vocab_size"], hidden_size=t["hidden_size"],
                           intermediate_size=t["intermediate_size"], num_layers=t["num_hidden_layers"],
                           num_heads=t["num_attention_heads"], num_kv_heads=t["num_key_value_heads"],
                           head_dim=t["hidden_size"] // t["num_attention_heads"], rope_theta=hf_rope(t)[0],
                           rope_scaling=hf_rope(t)[1], rms_eps=t.get("rms_norm_eps", 1e-5),
                           max_position=t.get("max_position_embeddings", 131072),
                           bos_token_id=t.get("bos_token_id", 128000),
                           eos_token_ids=tuple(eos) if isinstance(eos, list) else (eos,),
                           name=os.path.basename(path.rstrip("/")))
        vis = MllamaVisionConfig(hidden_size=v["hidden_size"], num_layers=v["num_hidden_layers"],
                                 num_global_layers=v["num_global_layers"], num_heads=v["attention_heads"],
                                 intermediate_size=v["intermediate_size"], image_size=v["image_size"],
                                 patch_size=v["patch_size"], max_num_tiles=v["max_num_tiles"],
                                 intermediate_layers=tuple(v["intermediate_layers_indices"]),
                                 ln_eps=v.get("norm_eps", 1e-5))
        return MllamaConfig(text=text, vision=vis, cross_layers=tuple(t["cross_attention_layers"]),
                            image_token_id=c.get("image_token_index", 128256),
                            extra_vocab=8, name=text.name)


class _TileMaskAttention(PackedAttention):
    """Vision self-attention under the reference's tile mask (see MllamaModel._tile_layout): per image, valid
    queries see all L keys, masked queries the first nvalid keys; both segments read the image's one set of
    paged K/V blocks (two varlen sequences sharing a block table)."""

    def __init__(self, nvalid: Sequence[int], L: int, num_heads: int, head_dim: int, device, dtype=torch.bfloat16):
        BS = ops.BLOCK
        nb = (L + BS - 1) // BS
        q_lens, rows, ctx = [], [], []
        for b, nv in enumerate(nvalid):
            blocks = torch.arange(b * nb, (b + 1) * nb, dtype=torch.int32)
            for ql, kl in ((nv, L), (L - nv, nv)):
                if ql:
                    q_lens.append(ql)
                    rows.append(blocks)
                    ctx.append(kl)
        self.H = self.Hkv = num_heads
        self.hd, self.causal, self.dtype, self.device = head_dim, False, dtype, torch.device(device)
        self.q_lens, self.kv_lens, self.T = q_lens, ctx, len(nvalid) * L
        dev = self.device
        self.positions = torch.zeros(self.T, dtype=torch.int32, device=dev)
        self.block_tables = torch.stack(rows).to(dev, non_blocking=True)
        self.slots = torch.cat([b * nb * BS + torch.arange(L, dtype=torch.int32)
                                for b in range(len(nvalid))]).to(dev, non_blocking=True)
        cu = [0]
        for n in q_lens:
            cu.append(cu[-1] + n)
        self.cu_q = torch.tensor(cu, dtype=torch.int32).to(dev, non_blocking=True)
        self.ctx = torch.tensor(ctx, dtype=torch.int32).to(dev, non_blocking=True)
        self.tiles = (ops.build_prefill_tiles(q_lens, self.H, self.Hkv, dev, head_dim=head_dim) if dev.type == "cuda"
                      else None)
        nblk = len(nvalid) * nb
        self.k_cache = torch.zeros(nblk + 1, self.Hkv, BS, head_dim, device=dev, dtype=dtype)
        self.v_cache = torch.zeros(nblk + 1, self.Hkv, head_dim, BS, device=dev, dtype=dtype)
        self.q = torch.empty(self.T, self.H, head_dim, device=dev, dtype=dtype)
        self.rope = False
        self.cs = torch.zeros(1, head_dim, dtype=torch.float32, device=dev)
        # every image's tokens fill its nb pages in order: packed straight from the QKV rows (PackedAttention.pack)
        self.pack = None
        if dtype == torch.bfloat16:
            tok = [b * L + BS * i for b in range(len(nvalid)) for i in range(nb)]
            cnt = [min(BS, L - BS * i) for _ in nvalid for i in range(nb)]
            self.pack = (torch.tensor(tok, dtype=torch.int32).to(dev, non_blocking=True),
                         torch.tensor(cnt, dtype=torch.int32).to(dev, non_blocking=True))


@dataclass
class ImageInput:
    pixels: torch.Tensor           # [n_tiles, 3, S, S] fp32 in [0, 1]
    aspect_ratio_id: int           # 1-based index into supported aspect ratios
    num_tiles: int


class CrossCache:
    """Paged cross-attention K/V for all cross layers: per request, ceil(n_img_tokens / 16) blocks."""

    def __init__(self, num_layers: int, num_blocks: int, hkv: int, hd: int, device, dtype):
        self.k = torch.zeros(num_layers, num_blocks + 1, hkv, ops.BLOCK, hd, device=device, dtype=dtype)
        self.v = torch.zeros(num_layers, num_blocks + 1, hkv, hd, ops.BLOCK, device=device, dtype=dtype)
        self.pad_block = num_blocks  # zero page for rows without an image
        self.free = list(range(num_blocks - 1, -1, -1))
        self.seqs: Dict[int, Tuple[List[int], int]] = {}

    @staticmethod
    def blocks_for_memory(nbytes: int, num_layers: int, hkv: int, hd: int, dtype) -> int:
        per = num_layers * 2 * hkv * ops.BLOCK * hd * torch.tensor([], dtype=dtype).element_size()
        return max(1, nbytes // per)

    def alloc(self, sid: int, ntok: int) -> List[int]:
        nb = (ntok + ops.BLOCK - 1) // ops.BLOCK
        if nb > len(self.free):
            raise RuntimeError(f"cross-attention cache exhausted ({nb} blocks needed, {len(self.free)} free)")
        blocks = [self.free.pop() for _ in range(nb)]
        self.seqs[sid] = (blocks, ntok)
        return blocks

    def release(self, sid: int):
        ent = self.seqs.pop(sid, None)
        if ent:
            self.free.extend(ent[0])


class MllamaModel(LlamaModel):
    supports_tp_sampling = False  # own forward (cross-attention layers) returns gathered logits
    """Vision encoder + projector + Llama decoder with cross-attention layers (TP = 1)."""

    supports_fp8_kv = False  # own attention call sites (no per-layer KV scales)

    def __init__(self, cfg: MllamaConfig, device=None, dtype=torch.bfloat16, dist_ctx=None,
                 max_images_in_flight: int = 64):
        self.mcfg = cfg
        self.cross_set = set(cfg.cross_layers)
        self.self_layers = [i for i in range(cfg.text.num_layers) if i not in self.cross_set]
        self.kv_index = {i: j for j, i in enumerate(self.self_layers)}
        self.cross_index = {i: j for j, i in enumerate(sorted(self.cross_set))}
        super().__init__(cfg.text, device, dtype, dist_ctx)
        assert self.ctx.tp_size == 1, "MllamaModel runs TP=1 (11B fits one MI355X many times over)"
        self.num_kv_layers = len(self.self_layers)
        V = cfg.vision
        self.max_cross_tokens = V.max_num_tiles * V.tokens_per_tile
        self.max_images_in_flight = max_images_in_flight
        self.cross: Optional[CrossCache] = None
        self.img_start: Dict[int, int] = {}  # sequence id -> position of its first <|image|> token
        self.vscale = 1.0 / math.sqrt(V.head_dim)
        self.mean = torch.tensor(MLLAMA_MEAN, dtype=torch.float32, device=self.device)
        self.inv_std = 1.0 / torch.tensor(MLLAMA_STD, dtype=torch.float32, device=self.device)
        self._alloc_vision()

    # ------------------------------------------------------------------ weights
    def _alloc(self):
        c, d, dt = self.cfg, self.device, self.dtype
        D, hd = c.hidden_size, c.head_dim
        e = lambda *s: torch.empty(*s, device=d, dtype=dt)  # noqa: E731
        self.w["embed"] = e(c.vocab_size + self.mcfg.extra_vocab, D)
        for i in range(c.num_layers):
            p = f"l{i}."
            self.w[p + "attn_norm"] = e(D)
            if i in self.cross_set:
                self.w[p + "q"] = e(self.hq * hd, D)
                self.w[p + "k"] = e(self.hkv * hd, D)
                self.w[p + "v"] = e(self.hkv * hd, D)
                self.w[p + "q_norm"] = e(hd)
                self.w[p + "k_norm"] = e(hd)
            else:
                self.w[p + "qkv"] = e((self.hq + 2 * self.hkv) * hd, D)
            self.w[p + "o"] = e(D, self.hq * hd)
            self.w[p + "mlp_norm"] = e(D)
            self.w[p + "gate_up"] = e(2 * self.inter, D)
            self.w[p + "down"] = e(D, self.inter)
        self.w["norm"] = e(D)
        self.w["lm_head"] = e(c.vocab_size, D)

    def _alloc_vision(self):
        V, d, dt = self.mcfg.vision, self.device, self.dtype
        D, I, hp, H = V.hidden_size, V.intermediate_size, V.head_dim_padded, V.num_heads
        e = lambda *s: torch.empty(*s, device=d, dtype=dt)  # noqa: E731
        nar = len(V.aspect_ratios) + 1
        self.w["v.patch"] = e(D, V.patch_k)
        self.w["v.cls"] = e(D)
        self.w["v.pos"] = e(V.tokens_per_tile, D)
        self.w["v.tile_pos"] = e(nar, V.max_num_tiles * V.tokens_per_tile * D)
        self.w["v.pre_tile"] = e(nar, V.max_num_tiles * D)
        self.w["v.post_tile"] = e(nar, V.max_num_tiles * D)
        self.gates = {"pos": 0.0, "pre_tile": 0.0, "post_tile": 0.0}
        for n in ("ln_pre", "ln_post"):
            self.w[f"v.{n}_w"], self.w[f"v.{n}_b"] = e(D), e(D)
        for i in range(V.num_layers + V.num_global_layers):
            p = f"v{i}."
            self.w[p + "ln1_w"], self.w[p + "ln1_b"] = e(D), e(D)
            self.w[p + "qkv"] = e(3 * H * hp, D)
            self.w[p + "o"] = e(D, H * hp)
            self.w[p + "ln2_w"], self.w[p + "ln2_b"] = e(D), e(D)
            self.w[p + "fc1"], self.w[p + "fc1_b"] = e(I, D), e(I)
            self.w[p + "fc2"], self.w[p + "fc2_b"] = e(D, I), e(D)
        self.w["proj"] = e(self.cfg.hidden_size, V.output_dim)
        self.w["proj_b"] = e(self.cfg.hidden_size)

    def random_init(self, seed: int = 0):
        s = seed * 1000
        V = self.mcfg.vision
        for k, t in self.w.items():
            if isinstance(t, ops.Fp8Weight):
                continue
            if k.endswith("norm") or k.endswith("ln1_w") or k.endswith("ln2_w") or k.endswith("_pre_w") \
                    or k.endswith("_post_w"):
                t.fill_(1.0)
            elif k.endswith("_b"):
                t.zero_()
            elif k in ("embed", "v.cls", "v.pos", "v.tile_pos", "v.pre_tile", "v.post_tile"):
                randn_like_(t, s, 0.02)
            else:
                randn_like_(t, s, 1.0 / math.sqrt(t.shape[1]))
            s += 1
        self.w["v.patch"][:, 3 * V.patch_size ** 2:].zero_()
        self._zero_vision_head_padding()
        self.gates = {"pos": 0.5, "pre_tile": 0.5, "post_tile": 0.5}
        return self

    def _zero_vision_head_padding(self):
        V = self.mcfg.vision
        hd, hp, H = V.head_dim, V.head_dim_padded, V.num_heads
        if hp == hd:
            return
        for i in range(V.num_layers + V.num_global_layers):
            p = f"v{i}."
            for k, view in (("qkv", lambda t: t.view(3, H, hp, -1)[:, :, hd:]), ("o", lambda t: t.view(-1, H, hp)[:, :, hd:])):
                w = self.w[p + k]
                if ops.is_frag(w):  # zero the padding in row-major order, then store fragment-ordered again
                    nat = ops.natural_weight(w)
                    view(nat).zero_()
                    w.copy_(ops.shuffle_fragments(nat))
                elif isinstance(w, torch.Tensor):
                    view(w).zero_()

    def quantize_fp8(self, vision: bool = True, text: bool = True) -> int:
        """e4m3fn per-channel weights for the transformer linears (BASELINE config 4 'CDNA4 fp8 MFMA')."""
        keys = []
        for k in self.w:
            last = k.split(".")[-1]
            if text and k.startswith("l") and last in ("qkv", "q", "o", "gate_up", "down"):
                keys.append(k)
            if vision and k.startswith("v") and k[1].isdigit() and last in ("qkv", "o", "fc1", "fc2"):
                keys.append(k)
        if vision:
            keys.append("proj")
        return quantize_linear_weights_fp8(self.w, keys)

    def load_hf_state(self, sd: Dict[str, torch.Tensor]):
        c, V = self.cfg, self.mcfg.vision
        hd, hp, H = V.head_dim, V.head_dim_padded, V.num_heads

        put = self._put  # re-shuffles into the fragment-ordered layout a serving engine may have given the weight

        lm = "language_model.model."
        put("embed", sd[lm + "embed_tokens.weight"])
        for i in range(c.num_layers):
            p, h = f"l{i}.", f"{lm}layers.{i}."
            put(p + "attn_norm", sd[h + "input_layernorm.weight"])
            put(p + "mlp_norm", sd[h + "post_attention_layernorm.weight"])
            g = sd[h + "mlp.gate_proj.weight"]
            u = sd[h + "mlp.up_proj.weight"]
            dn = sd[h + "mlp.down_proj.weight"]
            if i in self.cross_set:
                ga = math.tanh(float(sd[h + "cross_attn_attn_gate"].float().reshape(-1)[0]))
                gm = math.tanh(float(sd[h + "cross_attn_mlp_gate"].float().reshape(-1)[0]))
                put(p + "q", sd[h + "cross_attn.q_proj.weight"])
                put(p + "k", sd[h + "cross_attn.k_proj.weight"])
                put(p + "v", sd[h + "cross_attn.v_proj.weight"])
                put(p + "q_norm", sd[h + "cross_attn.q_norm.weight"])
                put(p + "k_norm", sd[h + "cross_attn.k_norm.weight"])
                put(p + "o", sd[h + "cross_attn.o_proj.weight"].float() * ga)
                dn = dn.float() * gm
            else:
                put(p + "qkv", torch.cat([sd[h + f"self_attn.{n}_proj.weight"] for n in "qkv"]))
                put(p + "o", sd[h + "self_attn.o_proj.weight"])
            put(p + "gate_up", ops.interleave_gate_up(g, u))
            put(p + "down", dn)
        put("norm", sd[lm + "norm.weight"])
        put("lm_head", sd["language_model.lm_head.weight"])
        vm = "vision_model."
        pw = sd[vm + "patch_embedding.weight"].reshape(V.hidden_size, -1)
        self.w["v.patch"].zero_()
        self.w["v.patch"][:, : pw.shape[1]].copy_(pw.to(self.dtype))
        put("v.cls", sd[vm + "class_embedding"])
        put("v.pos", sd[vm + "gated_positional_embedding.embedding"])
        put("v.tile_pos", sd[vm + "gated_positional_embedding.tile_embedding.weight"])
        put("v.pre_tile", sd[vm + "pre_tile_positional_embedding.embedding.weight"])
        put("v.post_tile", sd[vm + "post_tile_positional_embedding.embedding.weight"])
        self.gates = {"pos": math.tanh(float(sd[vm + "gated_positional_embedding.gate"].reshape(-1)[0])),
                      "pre_tile": math.tanh(float(sd[vm + "pre_tile_positional_embedding.gate"].reshape(-1)[0])),
                      "post_tile": math.tanh(float(sd[vm + "post_tile_positional_embedding.gate"].reshape(-1)[0]))}
        for n, hn in (("ln_pre", "layernorm_pre"), ("ln_post", "layernorm_post")):
            put(f"v.{n}_w", sd[vm + hn + ".weight"])
            put(f"v.{n}_b", sd[vm + hn + ".bias"])
        layers = [(f"{vm}transformer.layers.{i}.", False) for i in range(V.num_layers)] + \
                 [(f"{vm}global_transformer.layers.{i}.", True) for i in range(V.num_global_layers)]
        for i, (h, gated) in enumerate(layers):
            p = f"v{i}."
            ga = math.tanh(float(sd[h + "gate_attn"].reshape(-1)[0])) if gated else 1.0
            gf = math.tanh(float(sd[h + "gate_ffn"].reshape(-1)[0])) if gated else 1.0
            qkv = torch.zeros(3, H, hp, V.hidden_size)
            for j, n in enumerate("qkv"):
                qkv[j, :, :hd] = sd[h + f"self_attn.{n}_proj.weight"].float().view(H, hd, -1)
            put(p + "qkv", qkv.reshape(3 * H * hp, -1))
            o = torch.zeros(V.hidden_size, H, hp)
            o[:, :, :hd] = sd[h + "self_attn.o_proj.weight"].float().view(-1, H, hd) * ga
            put(p + "o", o.reshape(V.hidden_size, -1))
            put(p + "ln1_w", sd[h + "input_layernorm.weight"])
            put(p + "ln1_b", sd[h + "input_layernorm.bias"])
            put(p + "ln2_w", sd[h + "post_attention_layernorm.weight"])
            put(p + "ln2_b", sd[h + "post_attention_layernorm.bias"])
            put(p + "fc1", sd[h + "mlp.fc1.weight"])
            put(p + "fc1_b", sd[h + "mlp.fc1.bias"])
            put(p + "fc2", sd[h + "mlp.fc2.weight"].float() * gf)
            put(p + "fc2_b", sd[h + "mlp.fc2.bias"].float() * gf)
        put("proj", sd["multi_modal_projector.weight"])
        put("proj_b", sd["multi_modal_projector.bias"])
        return self

    # ------------------------------------------------------------------ image preprocessing
    def preprocess(self, image) -> ImageInput:
        """Fit the image into the best tile canvas (aspect ratio closest to the image's, as many tiles as
        its resolution warrants), resize keeping the aspect ratio, zero-pad, split into SxS tiles."""
        V = self.mcfg.vision
        S = V.image_size
        t = _to_chw_float(image).to(self.device)
        _, h, w = t.shape
        best, best_key = None, None
        for idx, (tw, th) in enumerate(V.aspect_ratios):
            scale = min(th * S / h, tw * S / w)
            # prefer the least downscaling, then the least upscaling/wasted canvas
            key = (min(scale, 1.0) * -1, abs(math.log(max(scale, 1e-6))) if scale > 1 else 0.0, th * tw)
            if best_key is None or key < best_key:
                best, best_key = (idx, th, tw, scale), key
        idx, th, tw, scale = best
        nh, nw = max(1, min(th * S, round(h * scale))), max(1, min(tw * S, round(w * scale)))
        r = F.interpolate(t[None], size=(nh, nw), mode="bilinear", antialias=True, align_corners=False)[0]
        canvas = torch.zeros(3, th * S, tw * S, device=self.device)
        canvas[:, :nh, :nw] = r.clamp(0, 1)
        tiles = canvas.view(3, th, S, tw, S).permute(1, 3, 0, 2, 4).reshape(th * tw, 3, S, S).contiguous()
        return ImageInput(tiles, idx + 1, th * tw)

    # ------------------------------------------------------------------ vision encoder
    def _vision_layers(self, h, lo, hi, attn, keep=()):
        V, w = self.mcfg.vision, self.w
        kept = []
        for i in range(lo, hi):
            p = f"v{i}."
            x = ops.layer_norm(h, w[p + "ln1_w"], w[p + "ln1_b"], V.ln_eps)
            qkv = ops.linear(x, w[p + "qkv"])
            a = attn(qkv, self.vscale)
            h = ops.linear(a, w[p + "o"], residual=h)
            x = ops.layer_norm(h, w[p + "ln2_w"], w[p + "ln2_b"], V.ln_eps)
            f = ops.linear(x, w[p + "fc1"], bias=w[p + "fc1_b"], act="gelu")
            h = ops.linear(f, w[p + "fc2"], bias=w[p + "fc2_b"], residual=h)
            if (i + 1) in keep:
                kept.append(h)
        return h, kept

    def _tile_layout(self, images: Sequence[ImageInput]):
        """Token layout of the vision encoder, the reference's (HF / Meta Mllama): every image runs ALL
        max_num_tiles tiles (absent tiles are zero pixels), each tile's 1 + num_patches tokens zero-padded to a
        multiple of 8 (P8). A token is *valid* when its tile is present and it is not padding. The reference's
        mask blocks attention only between two masked tokens: a valid token attends to every token of its image
        (padding and absent tiles included), a masked one to the valid ones. Tokens are kept valid-first per image
        (the encoder has no positional term inside attention, so order is free): the mask becomes two query
        segments over ONE key image, so the paged varlen kernel runs it as two sequences sharing blocks.
        Returns (perm [B * L] natural -> valid-first index, per-image valid counts, L)."""
        V = self.mcfg.vision
        NT, TPT = V.max_num_tiles, V.tokens_per_tile
        P8 = (TPT + 7) // 8 * 8
        L = NT * P8
        perm, nvalid = [], []
        for b, im in enumerate(images):
            nat = torch.arange(L).view(NT, P8)
            valid = torch.zeros(NT, P8, dtype=torch.bool)
            valid[: im.num_tiles, :TPT] = True
            perm.append(torch.cat([nat[valid], nat[~valid]]) + b * L)
            nvalid.append(im.num_tiles * TPT)
        return torch.cat(perm), nvalid, L

    @torch.no_grad()
    def encode_images(self, images: Sequence[ImageInput]) -> List[torch.Tensor]:
        """-> per image cross-attention states [n_tiles * 1601, text hidden] (bf16)."""
        V, w, g = self.mcfg.vision, self.w, self.gates
        D, NT, TPT = V.hidden_size, V.max_num_tiles, V.tokens_per_tile
        P8 = (TPT + 7) // 8 * 8
        B = len(images)
        pix = torch.cat([im.pixels for im in images]).contiguous()
        ntiles = [im.num_tiles for im in images]
        nt = sum(ntiles)
        x = ops.patchify(pix, V.patch_size, self.mean, self.inv_std, V.patch_k)
        pe_live = ops.linear(x, w["v.patch"]).view(nt, V.num_patches, D)
        # every image carries NT tiles: absent tiles are zero pixels = zero patch embeddings (no bias)
        pe = torch.zeros(B, NT, V.num_patches, D, device=self.device, dtype=self.dtype)
        o = 0
        for b, n in enumerate(ntiles):
            pe[b, :n] = pe_live[o:o + n]
            o += n
        ar = torch.tensor([im.aspect_ratio_id for im in images], device=self.device)
        # tanh-gated embeddings (tiny elementwise work next to the 40 layers; plain torch ops)
        pre = w["v.pre_tile"][ar].view(B, NT, 1, D).float()
        pe = (pe.float() + g["pre_tile"] * pre).to(self.dtype)
        pos = (1 - g["pos"]) * w["v.pos"].float().view(1, 1, TPT, D) + \
            g["pos"] * w["v.tile_pos"][ar].view(B, NT, TPT, D).float()
        cls = w["v.cls"].view(1, 1, 1, D).expand(B, NT, 1, D)
        h = (torch.cat([cls, pe], 2).float() + pos).to(self.dtype).reshape(B * NT * TPT, D)
        h = ops.layer_norm(h, w["v.ln_pre_w"], w["v.ln_pre_b"], V.ln_eps).view(B, NT, TPT, D)
        h = F.pad(h, (0, 0, 0, P8 - TPT))  # padding tokens enter the encoder as exact zeros
        perm, nvalid, L = self._tile_layout(images)
        perm = perm.to(self.device)
        h = h.reshape(B * L, D).index_select(0, perm).contiguous()
        attn = _TileMaskAttention(nvalid, L, V.num_heads, V.head_dim_padded, self.device, self.dtype)
        h, kept = self._vision_layers(h, 0, V.num_layers, attn, keep=set(V.intermediate_layers))
        h = ops.layer_norm(h, w["v.ln_post_w"], w["v.ln_post_b"], V.ln_eps)
        post = w["v.post_tile"][ar].view(B, NT, 1, D).expand(B, NT, P8, D).reshape(B * L, D).index_select(0, perm)
        h = (h.float() + g["post_tile"] * post.float()).to(self.dtype)
        h, _ = self._vision_layers(h, V.num_layers, V.num_layers + V.num_global_layers, attn)
        # valid tokens only (valid-first layout: the first n * TPT of each image, tile-major like the reference)
        sel = torch.cat([torch.arange(nv) + b * L for b, nv in enumerate(nvalid)]).to(self.device)
        # intermediate features interleaved per channel (the reference stacks them on a new last dim):
        # column D + d * n_kept + j = channel d of kept layer j
        inter = torch.stack([k.index_select(0, sel) for k in kept], dim=-1).flatten(-2)
        feats = torch.cat([h.index_select(0, sel), inter], dim=-1)
        states = ops.linear(feats, w["proj"], bias=w["proj_b"])
        out, o = [], 0
        for n in ntiles:
            out.append(states[o:o + n * TPT])
            o += n * TPT
        return out

    # ------------------------------------------------------------------ per-request cross state
    def _ensure_cross(self):
        if self.cross is None:
            c = self.cfg
            nb = self.max_images_in_flight * ((self.max_cross_tokens + ops.BLOCK - 1) // ops.BLOCK)
            self.cross = CrossCache(len(self.cross_set), nb, self.hkv, c.head_dim, self.device, self.dtype)
        return self.cross

    @torch.no_grad()
    def image_start(self, prompt_ids: Optional[Sequence[int]]) -> int:
        """Position of the first <|image|> token: text before it attends to no image (HF Mllama's
        ``full_text_row_masked_out_mask``: those rows get neither the cross-attention nor the cross layer's MLP
        output). A prompt without the token attends from position 0."""
        if prompt_ids is None:
            return 0
        for i, t in enumerate(prompt_ids):
            if t == self.mcfg.image_token_id:
                return i
        return 0

    def register_request(self, sid: int, images: Sequence, prompt_ids: Optional[Sequence[int]] = None) -> int:
        """Encode the request's image(s) and write the cross K/V of every cross layer. Returns #tokens.
        ``images`` holds raw images / :class:`ImageInput` or already-encoded cross states [n, hidden]
        (``encode_images`` batches many requests' images through one vision forward)."""
        if not images:
            return 0
        cc, c, w = self._ensure_cross(), self.cfg, self.w
        self.img_start[sid] = self.image_start(prompt_ids)
        if all(isinstance(x, torch.Tensor) and x.dim() == 2 and x.shape[1] == c.hidden_size for x in images):
            states = torch.cat(list(images))  # cross states already encoded (batched by the caller)
        else:
            ims = [im if isinstance(im, ImageInput) else self.preprocess(im) for im in images]
            states = torch.cat(self.encode_images(ims))
        n = states.shape[0]
        blocks = cc.alloc(sid, n)
        slots = (torch.tensor(blocks, dtype=torch.int32)[:, None] * ops.BLOCK +
                 torch.arange(ops.BLOCK, dtype=torch.int32)[None]).reshape(-1)[:n].to(self.device)
        pos = torch.zeros(n, dtype=torch.int32, device=self.device)
        hd = c.head_dim
        q_dummy = torch.empty(n, 0, hd, device=self.device, dtype=self.dtype)
        for j, i in enumerate(sorted(self.cross_set)):
            p = f"l{i}."
            k = ops.linear(states, w[p + "k"])
            k = ops.rms_norm(k.view(-1, hd), w[p + "k_norm"], c.rms_eps).view(n, -1)
            v = ops.linear(states, w[p + "v"])
            ops.rope_kv_write(torch.cat([k, v], 1), pos, self.cos_sin, slots, q_dummy, cc.k[j], cc.v[j], 0,
                              self.hkv, hd, rope=False)
        return n

    def release_request(self, sid: int):
        self.img_start.pop(sid, None)
        if self.cross is not None:
            self.cross.release(sid)

    def _cross_rows(self, seq_ids):
        cc = self.cross
        maxb = (self.max_cross_tokens + ops.BLOCK - 1) // ops.BLOCK
        bt = torch.full((len(seq_ids), maxb), cc.pad_block if cc else 0, dtype=torch.int32)
        lens = torch.ones(len(seq_ids), dtype=torch.int32)
        has = torch.zeros(len(seq_ids), dtype=torch.bool)
        for r, sid in enumerate(seq_ids):
            ent = cc.seqs.get(sid) if cc else None
            if ent:
                blocks, n = ent
                bt[r, : len(blocks)] = torch.tensor(blocks, dtype=torch.int32)
                lens[r], has[r] = n, True
        return bt, lens, has

    def prepare_batch(self, fb: ForwardBatch):
        """Engine hook: cross block tables / lengths / token row mask for the sequences of this step."""
        if fb.seq_ids is None or self.cross is None or not any(s in self.cross.seqs for s in fb.seq_ids):
            fb.extra = None  # text-only step: cross layers are skipped
            return
        bt, lens, has = self._cross_rows(fb.seq_ids)
        # per token: -1 = no image (masked), else the position its image starts at (masked before it)
        starts = []
        for i, n in enumerate(fb.prefill_qlen):
            starts += [self.img_start.get(fb.seq_ids[i], 0) if has[i] else -1] * n
        starts += [0 if x else -1 for x in has[len(fb.prefill_qlen):]]  # decode rows are past their prompt
        d = self.device
        st = torch.tensor(starts, dtype=torch.int32).to(d, non_blocking=True)
        row_mask = ((st >= 0) & (fb.positions >= st)).to(self.dtype).view(-1, 1)
        fb.extra = dict(cross_bt=bt.to(d, non_blocking=True), cross_len=lens.to(d, non_blocking=True),
                        row_mask=row_mask, max_cross=int(lens.max()), num_prefill_seqs=len(fb.prefill_qlen))

    def graph_static_inputs(self, bs: int) -> dict:
        self._ensure_cross()
        maxb = (self.max_cross_tokens + ops.BLOCK - 1) // ops.BLOCK
        d = self.device
        return dict(cross_bt=torch.full((bs, maxb), self.cross.pad_block, dtype=torch.int32, device=d),
                    cross_len=torch.ones(bs, dtype=torch.int32, device=d),
                    row_mask=torch.zeros(bs, 1, dtype=self.dtype, device=d),
                    max_cross=self.max_cross_tokens, num_prefill_seqs=0)

    def fill_graph_inputs(self, extra: dict, seq_ids: Sequence[int], n: int):
        bt, lens, has = self._cross_rows(list(seq_ids))
        extra["cross_bt"][:n].copy_(bt, non_blocking=True)
        extra["cross_len"][:n].copy_(lens, non_blocking=True)
        extra["row_mask"][:n].copy_(has.to(self.dtype).view(-1, 1), non_blocking=True)
        extra["cross_bt"][n:].fill_(self.cross.pad_block)
        extra["cross_len"][n:].fill_(1)
        extra["row_mask"][n:].zero_()

    # ------------------------------------------------------------------ text forward
    def forward(self, fb: ForwardBatch, kv, decode_ws=None) -> torch.Tensor:
        c, w = self.cfg, self.w
        T, P = fb.num_tokens, fb.num_prefill_tokens
        hd = c.head_dim
        ex = getattr(fb, "extra", None)
        res = ops.embedding(fb.token_ids, w["embed"])
        q = torch.empty(T, self.hq, hd, device=res.device, dtype=self.dtype)
        attn = torch.empty_like(q)
        h = None
        for i in range(c.num_layers):
            p = f"l{i}."
            is_cross = i in self.cross_set
            if is_cross and ex is None:
                continue
            x = ops.rms_norm(res, w[p + "attn_norm"], c.rms_eps) if h is None else \
                ops.rms_norm(h, w[p + "attn_norm"], c.rms_eps, residual=res)
            if is_cross:
                j = self.cross_index[i]
                ck, cv = self.cross.k[j], self.cross.v[j]
                qq = ops.linear(x, w[p + "q"])
                qn = ops.rms_norm(qq.view(-1, hd), w[p + "q_norm"], c.rms_eps).view(T, self.hq, hd)
                npf = ex["num_prefill_seqs"]
                if P > 0:
                    ops.attention_prefill(qn[:P], ck, cv, ex["cross_bt"][:npf], fb.cu_q, ex["cross_len"][:npf],
                                          self.scale, False, tiles=fb.prefill_tiles, q_lens=fb.prefill_qlen,
                                          out=attn[:P])
                if T > P:
                    ops.attention_decode(qn[P:], ck, cv, ex["cross_bt"][npf:], ex["cross_len"][npf:], self.scale,
                                         ws=decode_ws, max_ctx=ex["max_cross"], out=attn[P:])
                h = ops.linear(attn.view(T, -1), w[p + "o"]) * ex["row_mask"]
            else:
                qkv = ops.linear(x, w[p + "qkv"])
                kc, vc = kv.layer(self.kv_index[i])
                ops.rope_kv_write(qkv, fb.positions, self.cos_sin, fb.slots, q, kc, vc, self.hq, self.hkv, hd, True)
                if P > 0:
                    ops.attention_prefill(q[:P], kc, vc, fb.prefill_block_tables, fb.cu_q, fb.prefill_ctx,
                                          self.scale, True, tiles=fb.prefill_tiles, q_lens=fb.prefill_qlen,
                                          out=attn[:P])
                if T > P:
                    ops.attention_decode(q[P:], kc, vc, fb.decode_block_tables, fb.decode_ctx, self.scale,
                                         ws=decode_ws, max_ctx=fb.max_decode_ctx, out=attn[P:])
                h = ops.linear(attn.view(T, -1), w[p + "o"])
            x = ops.rms_norm(h, w[p + "mlp_norm"], c.rms_eps, residual=res)
            g = ops.linear(x, w[p + "gate_up"], act="swiglu")
            h = ops.linear(g, w[p + "down"])
            if is_cross:
                h = h * ex["row_mask"]
        if fb.sample_rows is not None:
            h = h.index_select(0, fb.sample_rows)
            res = res.index_select(0, fb.sample_rows)
        x = ops.rms_norm(h, w["norm"], c.rms_eps, residual=res)
        return ops.linear(x, w["lm_head"], out_dtype=torch.float32)[:, : c.vocab_size]

    # ------------------------------------------------------------------ fp32 reference (tests)
    @torch.no_grad()
    def reference_forward(self, token_ids: torch.Tensor, image: Optional[ImageInput] = None) -> torch.Tensor:
        """Dense fp32 PyTorch forward of one sequence (+ optional image) -> logits [T, vocab]."""
        c, V = self.cfg, self.mcfg.vision
        wf = {k: (v.dequantize(torch.float32) if isinstance(v, ops.Fp8Weight) else ops.natural_weight(v).float()).cpu()
              for k, v in self.w.items()}
        hd, H, Hkv = c.head_dim, c.num_heads, c.num_kv_heads
        states = None
        if image is not None:
            states = self._reference_vision(image, wf)
        ids = token_ids.long().cpu()
        T = ids.numel()
        x = wf["embed"][ids]
        cs = self.cos_sin.float().cpu()[:T]
        cos, sin = cs[:, : hd // 2], cs[:, hd // 2:]

        def rope(t):  # [T, h, hd]
            a, b = t[..., : hd // 2], t[..., hd // 2:]
            return torch.cat([a * cos[:, None] - b * sin[:, None], b * cos[:, None] + a * sin[:, None]], -1)

        def rms(v, g):
            return v * torch.rsqrt(v.pow(2).mean(-1, keepdim=True) + c.rms_eps) * g

        live = (torch.arange(T) >= self.image_start(ids.tolist())).float()[:, None]
        for i in range(c.num_layers):
            p = f"l{i}."
            if i in self.cross_set:
                if states is None:
                    continue
                x_in = x
                hn = rms(x, wf[p + "attn_norm"])
                q = rms((hn @ wf[p + "q"].t()).view(T, H, hd), wf[p + "q_norm"])
                k = rms((states @ wf[p + "k"].t()).view(-1, Hkv, hd), wf[p + "k_norm"])
                v = (states @ wf[p + "v"].t()).view(-1, Hkv, hd)
                k, v = k.repeat_interleave(H // Hkv, 1), v.repeat_interleave(H // Hkv, 1)
                a = F.scaled_dot_product_attention(q.transpose(0, 1), k.transpose(0, 1), v.transpose(0, 1))
                x = x + live * (a.transpose(0, 1).reshape(T, -1) @ wf[p + "o"].t())
                hn = rms(x, wf[p + "mlp_norm"])
                y = ops.reference.linear(hn, wf[p + "gate_up"], act="swiglu", out_dtype=torch.float32)
                x = x + live * (y @ wf[p + "down"].t())
                assert torch.equal(x[live[:, 0] == 0], x_in[live[:, 0] == 0])
                continue
            else:
                hn = rms(x, wf[p + "attn_norm"])
                qkv = hn @ wf[p + "qkv"].t()
                q, k, v = qkv.split([H * hd, Hkv * hd, Hkv * hd], -1)
                q, k = rope(q.view(T, H, hd)), rope(k.view(T, Hkv, hd))
                v = v.view(T, Hkv, hd)
                k, v = k.repeat_interleave(H // Hkv, 1), v.repeat_interleave(H // Hkv, 1)
                a = F.scaled_dot_product_attention(q.transpose(0, 1), k.transpose(0, 1), v.transpose(0, 1),
                                                   is_causal=True)
                x = x + a.transpose(0, 1).reshape(T, -1) @ wf[p + "o"].t()
            hn = rms(x, wf[p + "mlp_norm"])
            y = ops.reference.linear(hn, wf[p + "gate_up"], act="swiglu", out_dtype=torch.float32)
            x = x + y @ wf[p + "down"].t()
        x = rms(x, wf["norm"])
        return x @ wf["lm_head"].t()

    def _reference_vision(self, im: ImageInput, wf) -> torch.Tensor:
        """fp32 oracle in the reference's own layout: NT tiles x P8 tokens, mask(i, j) = valid_i or valid_j."""
        V, g = self.mcfg.vision, self.gates
        D, NT, TPT, P = V.hidden_size, V.max_num_tiles, V.tokens_per_tile, V.patch_size
        P8 = (TPT + 7) // 8 * 8
        n, ar = im.num_tiles, im.aspect_ratio_id
        px = im.pixels.float().cpu()
        x = (px - torch.tensor(MLLAMA_MEAN).view(1, 3, 1, 1)) / torch.tensor(MLLAMA_STD).view(1, 3, 1, 1)
        conv = wf["v.patch"][:, : 3 * P * P].reshape(D, 3, P, P)
        pe = torch.zeros(NT, V.num_patches, D)
        pe[:n] = F.conv2d(x, conv, stride=P).flatten(2).transpose(1, 2)
        pe = pe + g["pre_tile"] * wf["v.pre_tile"][ar].view(NT, 1, D)
        h = torch.cat([wf["v.cls"].view(1, 1, D).expand(NT, 1, D), pe], 1)
        h = h + (1 - g["pos"]) * wf["v.pos"][None] + g["pos"] * wf["v.tile_pos"][ar].view(NT, TPT, D)
        h = F.layer_norm(h, (D,), wf["v.ln_pre_w"], wf["v.ln_pre_b"], V.ln_eps)
        h = F.pad(h, (0, 0, 0, P8 - TPT)).reshape(1, NT * P8, D)
        valid = torch.zeros(NT, P8, dtype=torch.bool)
        valid[:n, :TPT] = True
        valid = valid.reshape(-1)
        allowed = valid[:, None] | valid[None, :]
        H, hp, hd = V.num_heads, V.head_dim_padded, V.head_dim

        def layers(h, lo, hi, keep=()):
            kept = []
            for i in range(lo, hi):
                p = f"v{i}."
                xx = F.layer_norm(h, (D,), wf[p + "ln1_w"], wf[p + "ln1_b"], V.ln_eps)
                qkv = (xx @ wf[p + "qkv"].t()).view(1, -1, 3, H, hp)[..., :hd]
                q, k, v = qkv.permute(2, 0, 3, 1, 4)
                a = F.scaled_dot_product_attention(q, k, v, attn_mask=allowed)  # [1, H, N, hd]
                a = F.pad(a, (0, hp - hd)).transpose(1, 2).reshape(1, -1, H * hp)
                h = h + a @ wf[p + "o"].t()
                xx = F.layer_norm(h, (D,), wf[p + "ln2_w"], wf[p + "ln2_b"], V.ln_eps)
                h = h + F.gelu(xx @ wf[p + "fc1"].t() + wf[p + "fc1_b"]) @ wf[p + "fc2"].t() + wf[p + "fc2_b"]
                if (i + 1) in keep:
                    kept.append(h)
            return h, kept

        h, kept = layers(h, 0, V.num_layers, set(V.intermediate_layers))
        h = F.layer_norm(h, (D,), wf["v.ln_post_w"], wf["v.ln_post_b"], V.ln_eps)
        h = h.view(NT, P8, D) + g["post_tile"] * wf["v.post_tile"][ar].view(NT, 1, D)
        h, _ = layers(h.reshape(1, NT * P8, D), V.num_layers, V.num_layers + V.num_global_layers)
        feats = torch.cat([h, torch.stack(kept, -1).flatten(-2)], -1)[0][valid]
        return feats @ wf["proj"].t() + wf["proj_b"]
