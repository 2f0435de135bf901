"""bench.py's multi-rank contract on the CPU (gloo, tiny models): launched the way the driver launches N > 1
(``python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N``),
every rank runs its own engine and index shard, queries search every shard, and rank 0 prints ONE JSON line
with the whole-job value, n_gpus = N, dp parallelism and the global batch (max step time over ranks)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(600)
def test_bench_torchrun_two_ranks_tiny():
    n, batch, steps = 2, 3, 1
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", str(n), "--steps", str(steps), "--warmup", "0", "--model", "tiny", "--embedder", "tiny",
           "--index-size", "1500", "--batch", str(batch), "--max-tokens", "6", "--chunk-tokens", "48",
           "--no-probes", "--no-graphs", "--served-steps", "1"]
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=560)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == n and out["steps"] == steps and out["warmup"] == 0
    assert out["config"]["parallelism"] == f"dp{n}" and out["config"]["global_batch"] == n * batch
    assert out["value"] > 0 and out["ms_per_step"] > 0 and out["higher_is_better"] is True
    assert out["scaling"] == "weak" and out["tokens_per_query"] == 6
    # value is the whole-job rate: n * batch * steps queries over the slowest rank's timed seconds
    assert abs(out["value"] - n * batch * steps / (out["ms_per_step"] * steps / 1000)) < 1e-3 * out["value"] + 1e-3
    # the served pass (POST /generate SSE through each rank's chain server) rides along, outside the timed steps
    sv = out["served"]
    assert sv["value"] > 0 and sv["steps"] == 1 and sv["p50_ttft_s"] > 0 and "vs_in_process" in sv
