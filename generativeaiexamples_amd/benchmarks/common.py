"""Shared timing / reporting for the config benchmarks (same contract as bench.py: W untimed warmup
steps, then exactly K timed steps bracketed by barrier + synchronize, slowest rank's time)."""
from __future__ import annotations

import os
import statistics
import sys
import time
from typing import Callable, List

import torch


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


def sync(ctx):
    ctx.barrier()
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def timed_steps(ctx, step: Callable[[int], dict], steps: int, warmup: int):
    """step(i) -> dict of per-step stats (ttft list etc.). Returns (total_seconds_max_over_ranks, stats)."""
    for w in range(warmup):
        sync(ctx)
        t0 = time.perf_counter()
        step(10_000 + w)
        sync(ctx)
        log(f"warmup {w}: {time.perf_counter() - t0:.2f}s")
    total, stats = 0.0, []
    for s in range(steps):
        sync(ctx)
        t0 = time.perf_counter()
        st = step(s)
        sync(ctx)
        dt = time.perf_counter() - t0
        total += dt
        stats.append(st)
        log(f"step {s}: {dt:.3f}s " + " ".join(f"{k}={v:.4g}" for k, v in st.items() if isinstance(v, (int, float))))
    if ctx.is_distributed:
        total = max(ctx.all_gather_obj(total))
    return total, stats


def percentile(xs: List[float], q: float) -> float:
    if not xs:
        return float("nan")
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * len(xs)))]


def gather_list(ctx, xs: list) -> list:
    if not ctx.is_distributed:
        return list(xs)
    return [x for part in ctx.all_gather_obj(list(xs)) for x in part]


def median(xs):
    return statistics.median(xs) if xs else float("nan")
