"""Decode-step anatomy of the serving engine: steady-state wall time per generated token (TPOT at --batch
concurrent sequences), plain engine.step() time, and the engine's own phase timers (schedule, upload, replay,
sample, process).

python tools/decode_profile.py [--model llama3-8b] [--batch 64] [--prompt 2400] [--steps 50]
"""
import argparse
import json
import time

import torch

from generativeaiexamples_amd.engine import EngineConfig, LLMEngine, SamplingParams
from generativeaiexamples_amd.models.registry import build_llm


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--prompt", type=int, default=2400)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--no-graphs", action="store_true")
    a = ap.parse_args()
    m, tok, name = build_llm(a.model, device="cuda")
    eng = LLMEngine(m, tok, EngineConfig(max_num_seqs=a.batch, max_model_len=a.prompt + 16 * (a.steps + 30) + 128,
                                         max_batched_tokens=16384, use_graphs=not a.no_graphs))
    if not a.no_graphs:
        eng.capture_graphs(max_bs=a.batch)
    g = torch.Generator().manual_seed(0)
    p = SamplingParams(temperature=0.2, top_p=0.7, max_tokens=16 * (a.steps + 30), ignore_eos=True)
    for i in range(a.batch):
        eng.add_request(torch.randint(10, 120000, (a.prompt,), generator=g).tolist(), p)
    while eng.stats["decode_tokens"] == 0:  # run through prefill
        eng.step()
    torch.cuda.synchronize()
    # steady-state decode: wall time per generated token (engine.step() runs `decode_steps` tokens per call)
    n0 = eng.stats["decode_tokens"]
    t0 = time.perf_counter()
    for _ in range(a.steps):
        eng.step()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    toks = (eng.stats["decode_tokens"] - n0) / a.batch
    out = {"model": name, "batch": a.batch, "ctx": a.prompt, "steps": a.steps,
           "ms_per_token": round(1000 * wall / max(toks, 1), 3), "tokens_per_seq": toks,
           "graph_steps": eng.stats.get("graph_steps")}
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        eng.step()
    torch.cuda.synchronize()
    out["plain_step_ms"] = round(100 * (time.perf_counter() - t0), 3)
    eng._timing, eng.phase_ms = True, {}
    for _ in range(10):
        eng.step()
    out["step_phases_ms"] = {k: round(v / 10, 3) for k, v in eng.phase_ms.items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
