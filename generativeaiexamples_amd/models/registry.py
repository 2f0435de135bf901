"""Model presets -> (model, tokenizer). Weights come from a local HF directory (safetensors +
tokenizer.json) when given, else random init of the real architecture (benchmarks / offline)."""
from __future__ import annotations

import os
from typing import Optional, Tuple

import torch

from ..engine.tokenizer import Tokenizer, bert_byte_tokenizer, load_tokenizer, llama3_byte_tokenizer, small_byte_tokenizer
from .bert import BertConfig, BertModel
from .clip import ClipConfig, ClipModel
from .decoder_reranker import DecoderRerankerConfig, DecoderRerankerModel
from .llama import LlamaConfig, LlamaModel
from .mixtral import MixtralConfig, MixtralModel
from .mllama import MllamaConfig, MllamaModel
from .opt import OPTConfig, OPTModel
from .qwen3_next import Qwen3NextConfig, Qwen3NextModel

LLM_PRESETS = {
    "llama3-8b": ("meta/llama3-8b-instruct", lambda: LlamaConfig.llama3_8b()),
    "llama3-70b": ("meta/llama3-70b-instruct", lambda: LlamaConfig.llama3_70b()),
    "llama3.1-8b": ("meta/llama-3.1-8b-instruct", lambda: LlamaConfig.llama31_8b()),
    "mistral-7b": ("mistralai/mistral-7b-instruct-v0.3", lambda: LlamaConfig.mistral_7b()),
    "tiny-llama": ("tiny-llama", lambda: LlamaConfig.tiny(max_position=4096)),
    # other dense decoder families of the reference's fine-tuning / NIM notebooks
    "gemma-7b": ("google/gemma-7b", lambda: LlamaConfig.gemma_7b()),
    "gemma-2b": ("google/gemma-2b", lambda: LlamaConfig.gemma_2b()),
    "codegemma-7b": ("google/codegemma-7b", lambda: LlamaConfig.codegemma_7b()),
    "starcoder2-15b": ("bigcode/starcoder2-15b", lambda: LlamaConfig.starcoder2_15b()),
    "starcoder2-7b": ("bigcode/starcoder2-7b", lambda: LlamaConfig.starcoder2_7b()),
    "qwen2.5-7b": ("qwen/qwen2.5-7b-instruct", lambda: LlamaConfig.qwen25_7b()),
    "qwen3-8b": ("qwen/qwen3-8b", lambda: LlamaConfig.qwen3_8b()),
    # hybrid Gated-DeltaNet / gated-attention MoE (the reference's Qwen3-Next agent notebook)
    "qwen3-next-80b-a3b": ("qwen/qwen3-next-80b-a3b-instruct", lambda: Qwen3NextConfig.qwen3_next_80b_a3b()),
    "qwen3-next-80b-a3b-thinking": ("qwen/qwen3-next-80b-a3b-thinking",
                                    lambda: Qwen3NextConfig.qwen3_next_80b_a3b(name="qwen/qwen3-next-80b-a3b-thinking")),
    "tiny-qwen3-next": ("tiny-qwen3-next", lambda: Qwen3NextConfig.tiny()),
    "opt-125m": ("facebook/opt-125m", lambda: OPTConfig.opt_125m()),
    "mixtral-8x7b": ("mistralai/mixtral-8x7b-instruct-v0.1", lambda: MixtralConfig.mixtral_8x7b()),
    "tiny-moe": ("tiny-moe", lambda: MixtralConfig.tiny_moe()),
    "llama3.2-11b-vision": ("meta/llama-3.2-11b-vision-instruct", lambda: MllamaConfig.llama32_11b_vision()),
    "tiny-mllama": ("tiny-mllama", lambda: MllamaConfig.tiny()),
}
# any LLM preset + "-fp8": e4m3fn per-channel weights on the fp8 MFMA GEMM (BASELINE config 4)

ENCODER_PRESETS = {
    "e5-large-v2": ("nvidia/nv-embedqa-e5-v5", lambda: BertConfig.e5_large_v2()),
    "e5-base-v2": ("intfloat/e5-base-v2", lambda: BertConfig.e5_base_v2()),
    "tiny-e5": ("tiny-e5", lambda: BertConfig.tiny()),
    "all-minilm-l6-v2": ("sentence-transformers/all-MiniLM-L6-v2", lambda: BertConfig.minilm_l6_v2()),
    "nvclip": ("nvidia/nvclip", lambda: ClipConfig.vit_l_14()),
    "tiny-clip": ("tiny-clip", lambda: ClipConfig.tiny()),
}

RERANKER_PRESETS = {
    "nv-rerankqa-mistral-4b": ("nvidia/nv-rerankqa-mistral-4b-v3", lambda: DecoderRerankerConfig.nv_rerankqa_mistral_4b()),
    "tiny-decoder-reranker": ("tiny-decoder-reranker", lambda: DecoderRerankerConfig.tiny()),
    "bge-reranker-large": ("BAAI/bge-reranker-large", lambda: BertConfig.bge_reranker_large()),
    "tiny-reranker": ("tiny-reranker", lambda: BertConfig.tiny(num_labels=1, pooling="cls", normalize=False)),
}


def _is_hf_dir(p: Optional[str]) -> bool:
    return bool(p) and os.path.isfile(os.path.join(p, "config.json"))


def build_llm(preset: str = "llama3-8b", weights: Optional[str] = None, device=None, seed: int = 0, dtype=None):
    """-> (model, tokenizer, served_name). Under a tensor-parallel context (parallel.dist.init_distributed
    with tp_size > 1) Llama-family models are built as this rank's shard (checkpoints are sliced on load)."""
    if _is_hf_dir(weights):
        import json

        arch = json.load(open(os.path.join(weights, "config.json"))).get("model_type", "llama")
        if arch == "opt":
            m = OPTModel(OPTConfig.from_hf(weights), device=device)
        elif arch == "mixtral":
            m = MixtralModel(MixtralConfig.from_hf(weights), device=device)
        elif arch == "mllama":
            m = MllamaModel(MllamaConfig.from_hf(weights), device=device)
        elif arch == "qwen3_next":
            m = Qwen3NextModel(Qwen3NextConfig.from_hf(weights), device=device)
        elif dtype is not None:
            m = LlamaModel(LlamaConfig.from_hf(weights), device=device, dtype=dtype)
        else:
            m = LlamaModel(LlamaConfig.from_hf(weights), device=device)
        m.load_safetensors_dir(weights) if hasattr(m, "load_safetensors_dir") else _load_st(m, weights)
        tok = load_tokenizer(weights, "llama3", m.cfg.vocab_size)
        return m, tok, os.path.basename(weights.rstrip("/"))
    fp8 = preset.endswith("-fp8")
    name, mk = LLM_PRESETS[preset[:-4] if fp8 else preset]
    cfg = mk()
    if isinstance(cfg, OPTConfig):
        m = OPTModel(cfg, device=device).random_init(seed)
        tok: Tokenizer = small_byte_tokenizer(512) if cfg.vocab_size < 1000 else _opt_tok(cfg.vocab_size)
        return m, tok, name
    if isinstance(cfg, MllamaConfig):
        m = MllamaModel(cfg, device=device).random_init(seed)
        vocab = cfg.text.vocab_size
    elif isinstance(cfg, MixtralConfig):
        m = MixtralModel(cfg, device=device).random_init(seed)
        vocab = cfg.vocab_size
    elif isinstance(cfg, Qwen3NextConfig):
        m = Qwen3NextModel(cfg, device=device).random_init(seed)
        vocab = cfg.vocab_size
    else:
        m = LlamaModel(cfg, device=device).random_init(seed)
        vocab = cfg.vocab_size
    if fp8:
        if hasattr(m, "quantize_fp8"):
            m.quantize_fp8()
        else:
            from .common import quantize_linear_weights_fp8
            quantize_linear_weights_fp8(m.w, [k for k in m.w if k.split(".")[-1] in ("qkv", "o", "gate_up", "fc", "down")])
        name += "-fp8"
    tok = llama3_byte_tokenizer(vocab) if vocab >= 128256 else small_byte_tokenizer(vocab) \
        if vocab <= 4096 else _generic_tok(m.cfg)
    return m, tok, name


def _opt_tok(vocab):
    from ..engine.tokenizer import ByteTokenizer

    return ByteTokenizer(vocab, 4, {"<s>": 2, "</s>": 2, "<pad>": 1}, bos="<s>", eos=("</s>",), pad="<pad>")


def _generic_tok(cfg):
    from ..engine.tokenizer import ByteTokenizer

    return ByteTokenizer(cfg.vocab_size, 3, {"<s>": 1, "</s>": 2}, bos="<s>", eos=("</s>",))


def _load_st(m, path):
    from safetensors.torch import load_file

    sd = {}
    for f in sorted(os.listdir(path)):
        if f.endswith(".safetensors"):
            sd.update(load_file(os.path.join(path, f)))
    m.load_hf_state(sd)


def build_encoder(preset: str = "e5-large-v2", weights: Optional[str] = None, device=None, seed: int = 0,
                  reranker: bool = False) -> Tuple[BertModel, Tokenizer, str]:
    if _is_hf_dir(weights):
        import json
        if json.load(open(os.path.join(weights, "config.json"))).get("model_type") == "clip":
            m = ClipModel(ClipConfig.from_hf(weights), device=device)
            _load_st(m, weights)
            return m, load_tokenizer(weights, "clip", m.cfg.vocab_size), os.path.basename(weights.rstrip("/"))
        cfg = BertConfig.from_hf(weights)
        m = BertModel(cfg, device=device)
        _load_st(m, weights)
        return m, load_tokenizer(weights, "bert", cfg.vocab_size), os.path.basename(weights.rstrip("/"))
    table = RERANKER_PRESETS if reranker else ENCODER_PRESETS
    name, mk = table[preset]
    cfg = mk()
    if isinstance(cfg, ClipConfig):
        m = ClipModel(cfg, device=device).random_init(seed)
        return m, small_byte_tokenizer(cfg.vocab_size) if cfg.vocab_size <= 4096 else _clip_tok(cfg.vocab_size), name
    m = BertModel(cfg, device=device).random_init(seed)
    return m, bert_byte_tokenizer(cfg.vocab_size), name


def build_embedder_service(preset: str = "e5-large-v2", weights: Optional[str] = None, device=None, seed: int = 0):
    """-> (Embedder | ClipEmbedder, served_name) ready for the /v1/embeddings route."""
    from ..engine.embedder import ClipEmbedder, Embedder
    m, tok, name = build_encoder(preset, weights, device, seed)
    if isinstance(m, ClipModel):
        return ClipEmbedder(m, tok, model_name=name), name
    return Embedder(m, tok, model_name=name), name


def build_reranker_service(preset: str = "nv-rerankqa-mistral-4b", weights: Optional[str] = None, device=None,
                           seed: int = 0):
    """-> (Reranker | DecoderReranker, served_name) for /v1/ranking."""
    from ..engine.embedder import DecoderReranker, Reranker
    if _is_hf_dir(weights):
        import json
        arch = json.load(open(os.path.join(weights, "config.json"))).get("model_type", "bert")
        if arch in ("mistral", "llama"):
            cfg = DecoderRerankerConfig(**LlamaConfig.hf_fields(
                json.load(open(os.path.join(weights, "config.json"))), os.path.basename(weights.rstrip("/"))))
            m = DecoderRerankerModel(cfg, device=device)
            _load_st(m, weights)
            return DecoderReranker(m, load_tokenizer(weights, "llama3", cfg.vocab_size)), os.path.basename(weights.rstrip("/"))
        m, tok, name = build_encoder(preset, weights, device, seed, reranker=True)
        return Reranker(m, tok, model_name=name), name
    name, mk = RERANKER_PRESETS[preset]
    cfg = mk()
    if isinstance(cfg, DecoderRerankerConfig):
        m = DecoderRerankerModel(cfg, device=device).random_init(seed)
        tok = small_byte_tokenizer(cfg.vocab_size) if cfg.vocab_size <= 4096 else _generic_tok(cfg)
        return DecoderReranker(m, tok, model_name=name), name
    m = BertModel(cfg, device=device).random_init(seed)
    return Reranker(m, bert_byte_tokenizer(cfg.vocab_size), model_name=name), name


def _clip_tok(vocab):
    from ..engine.tokenizer import ByteTokenizer

    return ByteTokenizer(vocab, 3, {"<|startoftext|>": vocab - 2, "<|endoftext|>": vocab - 1},
                         bos="<|startoftext|>", eos=("<|endoftext|>",))


def default_device():
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
