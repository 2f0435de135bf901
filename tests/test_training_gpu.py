"""LoRA SFT on the GPU (bf16 base weights, hipBLASLt GEMMs + SDPA under autograd)."""
import pytest
import torch

from generativeaiexamples_amd.engine.tokenizer import small_byte_tokenizer
from generativeaiexamples_amd.models.llama import LlamaConfig, LlamaModel
from generativeaiexamples_amd.parallel.dist import DistContext
from generativeaiexamples_amd.training.lora import LoRAConfig
from generativeaiexamples_amd.training.trainer import LoRATrainer, TrainConfig

pytestmark = pytest.mark.gpu


def test_lora_sft_gpu_loss_falls(cuda):
    ctx = DistContext(device=torch.device("cuda", 0))
    m = LlamaModel(LlamaConfig.tiny(num_layers=2), device="cuda", dist_ctx=ctx).random_init(seed=3)
    tr = LoRATrainer(m, small_byte_tokenizer(m.cfg.vocab_size), LoRAConfig(r=8, alpha=16, targets=("qkv", "o", "gate_up", "down")),
                     TrainConfig(steps=20, global_batch=8, micro_batch=4, seq_len=128, lr=3e-3, warmup=2,
                                 checkpoint_activations=True))
    h = tr.train()
    assert all(x == x for x in h) and h[-1] < 0.5 * h[0]
    assert tr.lora.params["l0.qkv.A"].device.type == "cuda"
