"""Model families on the gfx950 kernels (random-init or HF safetensors weights)."""
from .llama import LlamaConfig, LlamaModel  # noqa: F401
