"""Hardware side of the sizing advisor (reference: /root/reference/community/vgpu-sizing-advisor/src/server.py:
1455-1743 - ``/detect-gpu`` parses nvidia-smi, ``/apply-configuration`` and ``/test-configuration`` start vLLM in
Docker with the recommended configuration and stream its progress).

* ``detect_gpu``: the device name, count and memory from the HIP runtime (no vendor CLI), mapped to the sizing table's
  GPU names (MI355X / MI325X / MI300X).
* ``measure_config``: runs the recommended configuration on THIS framework's engine - the preset's architecture with
  random weights, ``concurrency`` prompts of ``prompt`` tokens decoded for ``response`` tokens - and reports measured
  TTFT / TPOT / throughput next to the analytic plan, so a recommendation is checked on the hardware it targets.
* ``launch_server``: starts the framework's own OpenAI-compatible server (``python -m generativeaiexamples_amd.serving``,
  tensor-parallel over ``tp`` GPUs) as a child process and streams its progress until ``/v1/models`` answers.
"""
from __future__ import annotations

import os
import subprocess
import sys
import tempfile
import time
from typing import Dict, Iterator, Optional

_GPU_CODES = (("MI355", "MI355X"), ("MI350", "MI355X"), ("MI325", "MI325X"), ("MI300", "MI300X"))


def gpu_code(name: str) -> str:
    up = name.upper()
    return next((code for key, code in _GPU_CODES if key in up), name)


def detect_gpu() -> Optional[Dict[str, object]]:
    import torch

    if not torch.cuda.is_available() or torch.cuda.device_count() == 0:
        return None
    p = torch.cuda.get_device_properties(0)
    return {"gpu_model": gpu_code(p.name), "gpu_name": p.name, "gpu_count": torch.cuda.device_count(),
            "gpu_memory_mb": int(p.total_memory // (1 << 20)), "arch": getattr(p, "gcnArchName", "")}


def measure_config(preset: str, concurrency: int = 8, prompt: int = 512, response: int = 64, device: str = "cuda",
                   use_graphs: bool = True, seed: int = 0) -> Dict[str, float]:
    """One measured wave on the engine: all prompts submitted together, decoded to exactly ``response`` tokens."""
    import torch

    from ...engine import EngineConfig, LLMEngine, SamplingParams
    from ...models.registry import build_llm
    from ...ops import BLOCK as block

    m, tok, name = build_llm(preset, device=device, seed=seed)
    per_seq = -(-(prompt + response + 8) // block)
    eng = LLMEngine(m, tok, EngineConfig(max_num_seqs=max(concurrency, 1), max_model_len=prompt + response + 8,
                                         num_blocks=concurrency * per_seq + 64, use_graphs=use_graphs,
                                         prefix_cache=False))
    g = torch.Generator().manual_seed(seed)
    vocab = getattr(getattr(m, "cfg", None), "vocab_size", 512)
    hi = min(int(vocab), 32000)

    def run(n, max_tokens):
        reqs = [eng.add_request(torch.randint(16, hi, (prompt,), generator=g).tolist(),
                                SamplingParams(temperature=0.0, max_tokens=max_tokens, ignore_eos=True))
                for _ in range(n)]
        t0 = time.perf_counter()
        while eng.has_work():
            eng.step()
        if str(device).startswith("cuda"):
            torch.cuda.synchronize()
        return reqs, time.perf_counter() - t0

    # warm-up at the measured batch size, long enough for the multi-step decode graphs: every graph bucket the timed
    # wave replays is captured here, not inside the timed wave
    run(concurrency, 2 * EngineConfig().decode_steps)
    reqs, wall = run(concurrency, response)
    ttft = sorted(r.ttft for r in reqs)
    tpot = [(r.finish_time - r.first_token_time) / max(1, len(r.output_ids) - 1) for r in reqs]
    out_tokens = sum(len(r.output_ids) for r in reqs)
    # decode-only step time: from the moment every prompt has its first token to the end (the plan's TPOT); the
    # per-request TPOT above also holds the time a request waits while later prompts prefill
    t_all_first = max(r.first_token_time for r in reqs)
    dec_step = (max(r.finish_time for r in reqs) - t_all_first) / max(1, response - 1)
    del eng, m
    if str(device).startswith("cuda"):
        torch.cuda.empty_cache()
    return {"model": name, "concurrency": concurrency, "prompt": prompt, "response": response,
            "ttft_p50_s": round(ttft[len(ttft) // 2], 4), "ttft_max_s": round(ttft[-1], 4),
            "tpot_ms": round(1000 * sum(tpot) / len(tpot), 3), "decode_step_ms": round(1000 * dec_step, 3),
            "wall_s": round(wall, 3),
            "output_tokens_per_s": round(out_tokens / wall, 1), "queries_per_s": round(concurrency / wall, 3)}


def launch_server(preset: str, tp: int = 1, port: int = 8000, max_num_seqs: int = 256, timeout_s: float = 900.0,
                  extra_args=(), poll_s: float = 2.0, python: str = sys.executable) -> Iterator[Dict[str, object]]:
    """Start the serving process and yield progress events until it answers (or dies / times out)."""
    import httpx

    cmd = [python, "-m", "generativeaiexamples_amd.serving", "--llm", preset, "--tp", str(tp), "--port", str(port),
           "--max-num-seqs", str(max_num_seqs), *extra_args]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    # the server's output goes to a log file: a pipe nobody drains would stall a long-running server
    log_path = os.path.join(tempfile.gettempdir(), f"gai-serve-{port}.log")
    with open(log_path, "wb") as log:
        proc = subprocess.Popen(cmd, env=env, stdout=log, stderr=subprocess.STDOUT)
    yield {"status": "starting", "pid": proc.pid, "command": " ".join(cmd), "log": log_path}
    t0 = time.time()
    url = f"http://127.0.0.1:{port}/v1/models"
    while time.time() - t0 < timeout_s:
        if proc.poll() is not None:
            with open(log_path, "rb") as f:
                err = f.read()[-2000:].decode("utf-8", "replace")
            yield {"status": "error", "message": f"server exited with code {proc.returncode}", "error": err}
            return
        try:
            r = httpx.get(url, timeout=2.0)
            if r.status_code == 200:
                yield {"status": "ready", "pid": proc.pid, "endpoint": f"http://127.0.0.1:{port}/v1",
                       "models": [m.get("id") for m in r.json().get("data", [])],
                       "startup_s": round(time.time() - t0, 1)}
                return
        except httpx.HTTPError:
            pass
        yield {"status": "loading", "elapsed_s": round(time.time() - t0, 1)}
        time.sleep(poll_s)
    proc.terminate()
    yield {"status": "error", "message": f"server did not become ready within {timeout_s:.0f} s"}
