"""Throughput of the community GPU paths on one MI355X:

* the FM-radio signal chain (``csrc/kernels/dsp.hip``): the reference's burst (500,000 payload bytes = 62,500 complex64
  samples at 1 MS/s, 101-tap low-pass, FM discriminator, 1 MS/s -> 16 kHz polyphase resampler) and a 4 M-sample
  block, each kernel timed alone and the whole chain, next to the same chain on the CPU (torch path);
* the DFP autoencoder: training rows/s of the reference's network (encoder [512, 500], decoder [512], batch 512,
  swap noise) on a synthetic 100K-row log frame, GPU vs CPU.

  python tools/community_bench.py --out gpurun_out/community/bench.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from generativeaiexamples_amd.community.fm_asr import dsp  # noqa: E402
from generativeaiexamples_amd.community.fm_asr.pipeline import SdrParams, SignalChain  # noqa: E402


def _time(fn, dev, iters):
    fn()
    if dev == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    if dev == "cuda":
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def dsp_bench(dev: str, n: int, iters: int) -> dict:
    p = SdrParams()
    chain = SignalChain(p, device=dev)
    g = torch.Generator().manual_seed(0)
    x = torch.complex(torch.randn(n, generator=g), torch.randn(n, generator=g)).to(dev)
    y = dsp.lowpass(chain.taps, x)
    d = dsp.fm_demod(y)
    out = {"samples": n}
    out["fir_ms"] = 1e3 * _time(lambda: dsp.lowpass(chain.taps, x), dev, iters)
    out["demod_ms"] = 1e3 * _time(lambda: dsp.fm_demod(y), dev, iters)
    out["resample_ms"] = 1e3 * _time(lambda: dsp.resample_poly(d, chain.up, chain.down, window="hamming",
                                                               gain=p.gain), dev, iters)
    out["chain_ms"] = 1e3 * _time(lambda: chain(x), dev, iters)
    out["chain_msamples_per_s"] = n / (out["chain_ms"] / 1e3) / 1e6
    # FIR: each output reads 101 taps x 8 B of (LDS-staged) input; HBM traffic is 8 B in + 8 B out per sample
    out["fir_hbm_gb_per_s"] = 16 * n / (out["fir_ms"] / 1e3) / 1e9
    out["realtime_factor_1msps"] = (n / p.sample_rate) / (out["chain_ms"] / 1e3)
    return {k: (round(v, 4) if isinstance(v, float) else v) for k, v in out.items()}


def dfp_bench(dev: str, rows: int, epochs: int) -> dict:
    import pandas as pd

    from generativeaiexamples_amd.community.dfp.autoencoder import TabularAutoEncoder

    rng = np.random.default_rng(0)
    df = pd.DataFrame({
        "app": rng.choice([f"app{i}" for i in range(40)], rows),
        "location": rng.choice([f"city{i}" for i in range(120)], rows),
        "device": rng.choice(["ios", "android", "windows", "mac", "linux"], rows),
        "logcount": rng.poisson(20, rows).astype(float),
        "locincrement": rng.integers(0, 10, rows).astype(float),
        "appincrement": rng.integers(0, 30, rows).astype(float),
        "success": rng.random(rows) < 0.9,
    })
    m = TabularAutoEncoder(device=dev)
    m.fit(df.head(2048), epochs=1)  # warm-up (kernels, allocator)
    if dev == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    hist = m.fit(df, epochs=epochs)
    if dev == "cuda":
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    t1 = time.perf_counter()
    res = m.get_results(df)
    score_s = time.perf_counter() - t1
    return {"rows": rows, "epochs": epochs, "train_s": round(dt, 3), "train_rows_per_s": round(rows * epochs / dt, 1),
            "score_rows_per_s": round(rows / score_s, 1), "final_loss": round(hist[-1], 4),
            "max_abs_z_p99": round(float(np.percentile(res["max_abs_z"], 99)), 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--cpu", action="store_true", help="also time the CPU paths")
    a = ap.parse_args()
    devs = (["cuda"] if torch.cuda.is_available() else []) + (["cpu"] if a.cpu or not torch.cuda.is_available() else [])
    res = {"device_name": torch.cuda.get_device_name(0) if torch.cuda.is_available() else "cpu"}
    for dev in devs:
        res[f"dsp_burst_{dev}"] = dsp_bench(dev, 62_500, 50 if dev == "cuda" else 5)
        res[f"dsp_4m_{dev}"] = dsp_bench(dev, 4_000_000, 20 if dev == "cuda" else 1)
        res[f"dfp_{dev}"] = dfp_bench(dev, 100_000 if dev == "cuda" else 20_000, 3 if dev == "cuda" else 1)
        print(json.dumps({k: v for k, v in res.items() if dev in k}), flush=True)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
