"""LoRA SFT: loss falls, checkpoint resume is exact, merge == adapter forward,
TP=2 loss/grads equal the single-process ones, DP=2 replicas stay identical (gloo, 127.0.0.1)."""
import socket

import pytest
import torch
import torch.multiprocessing as mp

from generativeaiexamples_amd.engine.tokenizer import small_byte_tokenizer
from generativeaiexamples_amd.models.llama import LlamaConfig, LlamaModel
from generativeaiexamples_amd.parallel.dist import DistContext
from generativeaiexamples_amd.training.forward import lm_loss
from generativeaiexamples_amd.training.lora import LoRAAdapter, LoRAConfig
from generativeaiexamples_amd.training.trainer import LoRATrainer, TrainConfig
from tests import _dist_workers as W


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model():
    cfg = LlamaConfig.tiny(num_layers=2)
    return LlamaModel(cfg, device="cpu", dist_ctx=DistContext(), dtype=torch.float32).random_init(seed=3)


def _trainer(m, out=None, steps=6):
    return LoRATrainer(m, small_byte_tokenizer(m.cfg.vocab_size), LoRAConfig(r=4, alpha=8, targets=("qkv", "o")),
                       TrainConfig(steps=steps, global_batch=2, micro_batch=1, seq_len=64, lr=3e-3, warmup=2,
                                   save_every=3, out=out))


def test_loss_decreases_and_resume_is_exact(tmp_path):
    straight = _trainer(_model(), steps=6)
    h = straight.train()
    assert h[-1] < h[0]
    first = _trainer(_model(), out=str(tmp_path / "run"), steps=3)
    first.train()
    resumed = _trainer(_model(), out=str(tmp_path / "run"), steps=6)
    assert resumed.step == 3  # picked up step_000003
    resumed.train()
    for k, v in straight.lora.params.items():
        torch.testing.assert_close(resumed.lora.params[k], v, rtol=1e-5, atol=1e-6)


def test_merge_equals_adapter_forward(tmp_path):
    m = _model()
    ad = LoRAAdapter(m, LoRAConfig(r=4, alpha=8, targets=("qkv", "o", "gate_up", "down")), seed=1)
    with torch.no_grad():
        for k, v in ad.params.items():
            if k.endswith(".B"):
                v.normal_(0, 0.05)
    ids = torch.randint(3, 500, (1, 20))
    labels = ids.clone()
    with torch.no_grad():
        l_adapter = lm_loss(m, ad, ids, labels)
        ad.save(str(tmp_path / "ad"))
        ad2 = LoRAAdapter.load(str(tmp_path / "ad"), m)
        ad2.merge_into(m)
        l_merged = lm_loss(m, None, ids, labels)
    torch.testing.assert_close(l_merged, l_adapter, rtol=1e-4, atol=1e-4)


@pytest.mark.timeout(300)
def test_tp2_lora_forward_backward(tmp_path):
    mp.spawn(W.lora_tp_worker, args=(2, _port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        d = torch.load(tmp_path / f"lora_tp_{r}.pt", weights_only=True)
        torch.testing.assert_close(d["loss"], d["loss_ref"], rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(d["g"], d["g_ref"], rtol=1e-3, atol=1e-5)      # replicated factor (all-reduced)
        torch.testing.assert_close(d["gA"], d["gA_ref"], rtol=1e-3, atol=1e-5)    # column-parallel A


@pytest.mark.timeout(300)
def test_dp2_bucketed_allreduce(tmp_path):
    mp.spawn(W.lora_dp_worker, args=(2, _port(), str(tmp_path)), nprocs=2, join=True)
    d0, d1 = (torch.load(tmp_path / f"lora_dp_{r}.pt", weights_only=True) for r in range(2))
    torch.testing.assert_close(d0["A"], d1["A"])  # replicas identical after 12 averaged steps
    assert d0["hist"][-1] < d0["hist"][0]
    torch.testing.assert_close(d0["hist"], d1["hist"])
