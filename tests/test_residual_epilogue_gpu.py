"""TP = 1 prefill writes the O / down projections' residual add in the GEMM epilogue (models/llama.py ``res_epi``):
bf16(bf16(h) + residual) is the rounding the residual-adding norm kernel applies, and the GEMM kernel choice does not
depend on the epilogue, so logits and KV caches must be bitwise equal to the unfused path (GAI_RES_EPI=0) - for a
256x256-walk prefill (T >= 1024) and a small-M prefill on the 128x128 kernel."""
import pytest
import torch

from generativeaiexamples_amd.engine.kv_cache import KVCache
from generativeaiexamples_amd.models import LlamaConfig, LlamaModel
from generativeaiexamples_amd.models.common import ForwardBatch
from generativeaiexamples_amd import ops

pytestmark = pytest.mark.gpu


def _prefill_batch(m, T, dev):
    nb = (T + ops.BLOCK - 1) // ops.BLOCK
    bt = torch.arange(1, nb + 1, device=dev, dtype=torch.int32).view(1, nb)
    pos = torch.arange(T, device=dev, dtype=torch.int32)
    g = torch.Generator().manual_seed(T)
    return ForwardBatch(token_ids=torch.randint(10, 1000, (T,), generator=g).to(dev, torch.int32), positions=pos,
                        slots=(bt[0, pos.long() // ops.BLOCK] * ops.BLOCK + pos % ops.BLOCK).int(),
                        num_prefill_tokens=T, cu_q=torch.tensor([0, T], device=dev, dtype=torch.int32),
                        prefill_ctx=torch.tensor([T], device=dev, dtype=torch.int32), prefill_block_tables=bt,
                        prefill_tiles=ops.build_prefill_tiles([T], m.hq, m.hkv, dev, head_dim=m.cfg.head_dim),
                        prefill_qlen=[T], prefill_ctx_host=[T], sample_rows=None), nb


@pytest.mark.parametrize("T", [1100, 300])
def test_prefill_residual_epilogue_bitwise(cuda, T, monkeypatch):
    cfg = LlamaConfig.tiny(num_heads=8, num_kv_heads=2, head_dim=128, hidden_size=1024, intermediate_size=2048,
                           vocab_size=1024, num_layers=3)
    m = LlamaModel(cfg, device="cuda").random_init(7)
    outs = []
    for flag in ("1", "0"):
        monkeypatch.setenv("GAI_RES_EPI", flag)
        fb, nb = _prefill_batch(m, T, "cuda")
        kv = KVCache(cfg.num_layers, nb + 2, m.hkv, cfg.head_dim, m.device, m.dtype)
        with torch.inference_mode():
            logits = m.forward(fb, kv)
        torch.cuda.synchronize()
        outs.append((logits.float().cpu(), kv.storage.float().cpu()))
    assert torch.equal(outs[0][0], outs[1][0]), (outs[0][0] - outs[1][0]).abs().max()
    assert torch.equal(outs[0][1], outs[1][1])
