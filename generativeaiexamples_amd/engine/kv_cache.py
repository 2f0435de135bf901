"""Paged KV cache storage (one K and one V^T tensor per layer, views of one HBM allocation).

Sizing is HBM-first: with 288 GB per MI355X the cache is sized from the memory left after
weights and activations (``gpu_memory_fraction``), not from a fixed token count.
Llama-3-8B bf16 uses 128 KiB/token, so e.g. 200 GB of cache holds ~1.6M tokens.
"""
from __future__ import annotations

import torch

from ..ops import BLOCK


FP8 = torch.float8_e4m3fn


def cache_dtype(name: str, model_dtype):
    """EngineConfig.kv_cache_dtype -> torch dtype: "auto" (the model's), "fp8" / "fp8_e4m3" (OCP e4m3fn)."""
    if name in (None, "", "auto"):
        return model_dtype
    if name in ("fp8", "fp8_e4m3", "float8_e4m3fn"):
        return FP8
    if name in ("bf16", "bfloat16"):
        return torch.bfloat16
    raise ValueError(f"unsupported kv_cache_dtype {name!r} (auto | fp8 | bf16)")


class KVCache:
    """``dtype=torch.float8_e4m3fn`` is the fp8 KV option (the NIM / TRT-LLM ``kv_cache_dtype=fp8``): the cache
    stores K / scale and V / scale (static per-layer scales, default 1.0 like vLLM's uncalibrated fp8 KV),
    the attention kernels dequantise while loading - half the HBM bytes per cached token, twice the tokens."""

    def __init__(self, num_layers: int, num_blocks: int, num_kv_heads: int, head_dim: int, device,
                 dtype=torch.bfloat16, k_scale: float = 1.0, v_scale: float = 1.0):
        self.num_layers, self.num_blocks = num_layers, num_blocks
        self.dtype = dtype
        fp8 = dtype == FP8
        self.k_scales = [float(k_scale) if fp8 else 1.0] * num_layers
        self.v_scales = [float(v_scale) if fp8 else 1.0] * num_layers
        self.hkv, self.hd = num_kv_heads, head_dim
        per = num_blocks * num_kv_heads * BLOCK * head_dim
        # zero-filled: masked tail slots of a page are read (and multiplied by p=0) by the kernels
        self.storage = torch.zeros(num_layers, 2, per, dtype=dtype, device=device)
        self.k = [self.storage[i, 0].view(num_blocks, num_kv_heads, BLOCK, head_dim) for i in range(num_layers)]
        self.v = [self.storage[i, 1].view(num_blocks, num_kv_heads, head_dim, BLOCK) for i in range(num_layers)]

    def layer(self, i: int):
        return self.k[i], self.v[i]

    def scales(self, i: int):
        return self.k_scales[i], self.v_scales[i]

    @staticmethod
    def bytes_per_block(num_layers, num_kv_heads, head_dim, dtype=torch.bfloat16) -> int:
        return num_layers * 2 * num_kv_heads * BLOCK * head_dim * torch.finfo(dtype).bits // 8

    @staticmethod
    def blocks_for_memory(nbytes: int, num_layers, num_kv_heads, head_dim, dtype=torch.bfloat16) -> int:
        return max(16, int(nbytes // KVCache.bytes_per_block(num_layers, num_kv_heads, head_dim, dtype)))

    @property
    def nbytes(self) -> int:
        return self.storage.numel() * self.storage.element_size()
