"""Deployment sizing (SURVEY §2.9 vgpu-sizing-advisor): reference formulas reproduce BASELINE.md rows 2-7,
the MI355X planner's memory / TP choices follow the real attention geometry."""
import pytest

from generativeaiexamples_amd import sizing


@pytest.mark.parametrize("gpu,n,ttft,tpot,tps", [("L40S", 1, 0.062, 18.5, 53.5), ("A40", 1, 0.077, 23.0, 43.1),
                                                 ("L4", 1, 0.119, 53.3, 18.7), ("RTX-PRO-6000", 1, 0.042, 10.0, 98.7)])
def test_reference_formula_reproduces_baseline_rows(gpu, n, ttft, tpot, tps):
    r = sizing.reference_estimate(8, gpu, n)
    assert r["ttft_s"] == pytest.approx(ttft, abs=1.5e-3)
    assert r["tpot_ms"] == pytest.approx(tpot, abs=0.1)
    assert r["tokens_per_s"] == pytest.approx(tps, abs=0.2)


def test_reference_formula_70b_tp8():
    r = sizing.reference_estimate(70, "L40S", 8)
    assert r["tpot_ms"] == pytest.approx(20.3, abs=0.1) and r["tokens_per_s"] == pytest.approx(48.9, abs=0.3)


def test_mi355x_plan_geometry():
    p8 = sizing.plan("llama3-8b", concurrency=64, index_vectors=1_000_000)
    assert p8["tp"] == 1 and p8["fits"]
    assert p8["kv_bytes_per_token"] == 2 * 32 * 8 * 128 * 2  # GQA: 8 KV heads, not d_model
    assert 7.5 < p8["memory_gb"]["weights"] < 16.5
    p70 = sizing.plan("llama3-70b", concurrency=64)
    assert p70["tp"] == 1 and p70["fits"]  # 141 GB bf16 weights fit one 288 GB MI355X
    big = sizing.plan("llama3-70b", concurrency=512, prompt=8192, response=1024)
    assert big["tp"] > 1
    fp8 = sizing.plan("llama3-70b", concurrency=64, dtype="fp8", kv_dtype="fp8")
    assert fp8["memory_gb"]["weights"] < p70["memory_gb"]["weights"] / 1.9 and fp8["tpot_ms"] < p70["tpot_ms"]
    # more concurrency: more tokens/s, longer step
    lo, hi = sizing.plan("llama3-8b", concurrency=8), sizing.plan("llama3-8b", concurrency=128)
    assert hi["decode_tokens_per_s"] > lo["decode_tokens_per_s"] and hi["tpot_ms"] > lo["tpot_ms"]


def test_cli_runs(capsys):
    sizing.main(["--model", "mixtral-8x7b", "--reference"])
    out = capsys.readouterr().out
    assert '"reference_formula"' in out and '"tp"' in out
