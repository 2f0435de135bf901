"""Paged KV cache storage (one K and one V^T tensor per layer, views of one HBM allocation).

Sizing is HBM-first: with 288 GB per MI355X the cache is sized from the memory left after
weights and activations (``gpu_memory_fraction``), not from a fixed token count.
Llama-3-8B bf16 uses 128 KiB/token, so e.g. 200 GB of cache holds ~1.6M tokens.
"""
from __future__ import annotations

import torch

from ..ops import BLOCK


class KVCache:
    def __init__(self, num_layers: int, num_blocks: int, num_kv_heads: int, head_dim: int, device,
                 dtype=torch.bfloat16):
        self.num_layers, self.num_blocks = num_layers, num_blocks
        self.hkv, self.hd = num_kv_heads, head_dim
        per = num_blocks * num_kv_heads * BLOCK * head_dim
        # zero-filled: masked tail slots of a page are read (and multiplied by p=0) by the kernels
        self.storage = torch.zeros(num_layers, 2, per, dtype=dtype, device=device)
        self.k = [self.storage[i, 0].view(num_blocks, num_kv_heads, BLOCK, head_dim) for i in range(num_layers)]
        self.v = [self.storage[i, 1].view(num_blocks, num_kv_heads, head_dim, BLOCK) for i in range(num_layers)]

    def layer(self, i: int):
        return self.k[i], self.v[i]

    @staticmethod
    def bytes_per_block(num_layers, num_kv_heads, head_dim, dtype=torch.bfloat16) -> int:
        return num_layers * 2 * num_kv_heads * BLOCK * head_dim * torch.finfo(dtype).bits // 8

    @staticmethod
    def blocks_for_memory(nbytes: int, num_layers, num_kv_heads, head_dim, dtype=torch.bfloat16) -> int:
        return max(16, int(nbytes // KVCache.bytes_per_block(num_layers, num_kv_heads, head_dim, dtype)))

    @property
    def nbytes(self) -> int:
        return self.storage.numel() * self.storage.element_size()
