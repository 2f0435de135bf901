"""Reduce the rocprofv3 counter passes written by tools/pmc_gemm.sh into one JSON per shape.

usage: python tools/pmc_reduce.py gpurun_out/pmc_o "M=16384 N=4096 K=4096" OUT.json

For every arm directory (t_<arm>, p1_<arm>, p2_<arm>, p3_<arm>) the GEMM kernel is the one with the
largest total time in the kernel-trace pass; counter values are summed over a dispatch's instances and
averaged over its dispatches. Derived: MFMA busy fraction = SQ_VALU_MFMA_BUSY_CYCLES (summed over all
SIMDs; = 16 x the 16x16x32 MFMAs) / (1024 SIMDs x GRBM_GUI_ACTIVE / 8: GRBM counts are summed over the 8
XCDs), the matching shader clock, wave wait fraction and L2 hit rate.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def _rows(pattern):
    for f in glob.glob(pattern, recursive=True):
        with open(f, newline="") as fh:
            yield from csv.DictReader(fh)


def _gemm_kernel(d):
    tot = defaultdict(float)
    cnt = defaultdict(int)
    for r in _rows(os.path.join(d, "**", "*kernel_stats.csv")):
        tot[r["Name"]] = float(r["TotalDurationNs"])
        cnt[r["Name"]] = int(r["Calls"])
    name = max(tot, key=tot.get)
    return name, tot[name] / cnt[name] / 1e3


def _counters(d, kernel):
    per = defaultdict(lambda: defaultdict(float))  # dispatch -> counter -> sum
    for r in _rows(os.path.join(d, "**", "*counter_collection.csv")):
        if r["Kernel_Name"] != kernel:
            continue
        per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    out = defaultdict(float)
    for c in per.values():
        for k, v in c.items():
            out[k] += v / len(per)
    return dict(out)


def main():
    base, shape, dst = sys.argv[1], sys.argv[2], sys.argv[3]
    arms = sorted({os.path.basename(p)[2:] for p in glob.glob(os.path.join(base, "t_*")) if os.path.isdir(p)})
    res = {"shape": shape, "arms": {}}
    for arm in arms:
        kern, avg_us = _gemm_kernel(os.path.join(base, f"t_{arm}"))
        c = {}
        for p in ("p1", "p2", "p3"):
            c.update(_counters(os.path.join(base, f"{p}_{arm}"), kern))
        ncu, nxcd = 256, 8
        if c.get("GRBM_GUI_ACTIVE"):
            xcd_cycles = c["GRBM_GUI_ACTIVE"] / nxcd
            c["mfma_busy_frac"] = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (4 * ncu * xcd_cycles)
            c["clock_ghz"] = xcd_cycles / (avg_us * 1e3)
        if c.get("SQ_WAVE_CYCLES"):
            c["wait_frac"] = c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"]
        hits, miss = c.get("TCC_HIT_sum", 0), c.get("TCC_MISS_sum", 0)
        if hits + miss:
            c["l2_hit_rate"] = hits / (hits + miss)
        c.update(kernel=kern[:100], avg_us=avg_us)
        res["arms"][arm] = c
    with open(dst, "w") as f:
        json.dump(res, f, indent=1)
    for arm, c in res["arms"].items():
        print(arm, round(c["avg_us"], 1), "mfma_busy", round(c.get("mfma_busy_frac", 0), 3), "wait",
              round(c.get("wait_frac", 0), 3), "tcp_tcc_req", c.get("TCP_TCC_READ_REQ_sum"), "l2_hit",
              round(c.get("l2_hit_rate", 0), 3))


if __name__ == "__main__":
    main()
