"""Check the MI355X sizing planner against measured runs on this framework's engine (the sizing advisor's
``/test-configuration``): for each (model, concurrency) the analytic plan's TPOT / single-query TTFT next to one
measured wave (random-init weights of the named architecture, all prompts submitted together, exactly ``response``
tokens each).

  python tools/sizing_validate.py --model llama3-8b --concurrency 1 16 64 --prompt 2407 --response 128 \
      --out gpurun_out/sizing/validate.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from generativeaiexamples_amd import sizing  # noqa: E402
from generativeaiexamples_amd.community.sizing_advisor.deploy import measure_config  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--concurrency", type=int, nargs="+", default=[1, 16, 64])
    ap.add_argument("--prompt", type=int, default=2407)
    ap.add_argument("--response", type=int, default=128)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rows = []
    for c in a.concurrency:
        plan = sizing.plan(a.model, "MI355X", 1, c, a.prompt, a.response, embedder=None)
        m = measure_config(a.model, concurrency=c, prompt=a.prompt, response=a.response)
        row = {"model": a.model, "concurrency": c, "prompt": a.prompt, "response": a.response,
               "plan_tpot_ms": plan["tpot_ms"], "measured_decode_step_ms": m["decode_step_ms"],
               "measured_tpot_per_request_ms": m["tpot_ms"],
               "plan_ttft_single_s": plan["ttft_s_single"], "measured_ttft_p50_s": m["ttft_p50_s"],
               "measured_ttft_max_s": m["ttft_max_s"], "plan_wave_s": plan["wave_s"], "measured_wall_s": m["wall_s"],
               "measured_output_tokens_per_s": m["output_tokens_per_s"]}
        row["decode_step_measured_over_plan"] = round(m["decode_step_ms"] / plan["tpot_ms"], 3)
        row["wave_measured_over_plan"] = round(m["wall_s"] / plan["wave_s"], 3)
        print(json.dumps(row), flush=True)
        rows.append(row)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
