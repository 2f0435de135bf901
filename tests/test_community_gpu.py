"""Community apps on the MI355X: the sizing advisor's GPU detection and its measured test run of a configuration on
this framework's engine (tiny preset so the run is seconds)."""
import pytest

pytestmark = pytest.mark.gpu


def test_detect_gpu_reports_mi355x():
    from generativeaiexamples_amd.community.sizing_advisor.deploy import detect_gpu

    info = detect_gpu()
    assert info is not None and info["gpu_count"] >= 1 and info["gpu_memory_mb"] > 100_000
    assert info["gpu_model"] == "MI355X" or "gfx950" in info["arch"], info


def test_measure_config_runs_engine_wave():
    from generativeaiexamples_amd.community.sizing_advisor.deploy import measure_config

    m = measure_config("tiny-llama", concurrency=4, prompt=64, response=16, use_graphs=True)
    assert m["concurrency"] == 4 and 0 < m["ttft_p50_s"] <= m["ttft_max_s"] < 30
    assert m["tpot_ms"] > 0 and m["output_tokens_per_s"] > 0 and m["wall_s"] > 0
