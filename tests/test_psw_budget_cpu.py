"""Decode weight copies under an HBM budget (LlamaModel.preshuffle_decode_weights): whole projection kinds in
PSW_PRIORITY order while they fit, kinds that do not fit are skipped (a later, smaller kind may still fit), and
fp8 weights count their bf16 copy. The copying itself is stubbed (it needs a GPU; tests/test_splitk_gpu.py runs it)."""
import torch

from generativeaiexamples_amd import ops
from generativeaiexamples_amd.models import LlamaConfig, LlamaModel


def _stub(monkeypatch):
    done = []
    monkeypatch.setattr(ops, "psw_qualifies", lambda w: True)
    monkeypatch.setattr(ops, "preshuffle_weight", lambda w: done.append(w) or True)
    return done


def _kind_bytes(m, kind):
    return sum(ops.psw_bytes(v) for k, v in m.w.items() if k.rsplit(".", 1)[-1] == kind)


def test_budget_takes_kinds_in_priority_order(monkeypatch):
    m = LlamaModel(LlamaConfig.tiny(), device="cpu")
    done = _stub(monkeypatch)
    gu, down, lm = _kind_bytes(m, "gate_up"), _kind_bytes(m, "down"), _kind_bytes(m, "lm_head")
    added = m.preshuffle_decode_weights(budget_bytes=gu + lm)  # down does not fit after gate_up; lm_head does
    assert added == gu + lm
    names = {k for k, v in m.w.items() for d in done if v is d}
    assert any(n.endswith("gate_up") for n in names) and "lm_head" in names
    assert not any(n.endswith(("down", "qkv", ".o")) for n in names)
    assert down > lm  # the skip above is a size decision


def test_unbounded_budget_takes_everything_once(monkeypatch):
    m = LlamaModel(LlamaConfig.tiny(), device="cpu")
    done = _stub(monkeypatch)
    added = m.preshuffle_decode_weights()
    kinds = {k.rsplit(".", 1)[-1] for k in m.w} & set(LlamaModel.PSW_PRIORITY)
    assert added == sum(_kind_bytes(m, k) for k in kinds)
    assert len({id(d) for d in done}) == len(done)


def test_fp8_weight_counts_its_bf16_copy():
    q = torch.zeros(64, 512, dtype=torch.float8_e4m3fn)
    w = ops.Fp8Weight(q, torch.ones(64))
    assert ops.psw_bytes(w) == 64 * 512 * 2 and w.dec is None
