"""Reduce tools/pmc_decode.sh (kernel trace + FETCH_SIZE + WRITE_SIZE passes) into per-kernel traffic.

usage: python tools/pmc_decode_reduce.py gpurun_out/r5pmcd [known.json]

Prints per kernel: median duration (us), FETCH_SIZE / WRITE_SIZE per dispatch (MB, as reported: the counter's KB
units) and, for the kernels named in the built-in table of Llama-3-8B batch-64 decode tensor sizes, the ratio of the
reported fetch to the bytes the kernel must read at least once.
"""
import collections
import csv
import glob
import os
import sys

# bytes each kernel must read at least once (Llama-3-8B, batch 64, ctx 2535, bf16): KV of one layer, weights
KNOWN_MB = {"attn_decode_kernel": 64 * 2535 * 8 * 128 * 2 * 2 / 1e6, "gemm_dec2_kernel<4, 8, 4": 28672 * 4096 * 2 / 1e6,
            "gemm_dec2_kernel<4, 8, 0": 128256 * 4096 * 2 / 1e6, "gemm_dec2_kernel<4, 4, 0": 4096 * 14336 * 2 / 1e6}


def main():
    d = sys.argv[1]
    dur = collections.defaultdict(list)
    for r in csv.DictReader(open(glob.glob(os.path.join(d, "t", "*kernel_trace.csv"))[0])):
        dur[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)

    def counters(sub, name):
        agg = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(glob.glob(os.path.join(d, sub, "*counter_collection.csv"))[0])):
            if r["Counter_Name"] == name:
                agg[r["Kernel_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
        return {k: sum(v.values()) / len(v) for k, v in agg.items()}

    f, w = counters("p", "FETCH_SIZE"), counters("w", "WRITE_SIZE")
    rows = []
    for k in f:
        if k in dur:
            ds = sorted(dur[k])
            rows.append((sum(ds), k, ds[len(ds) // 2], f[k] / 1024, w.get(k, 0.0) / 1024))
    rows.sort(reverse=True)
    print("| kernel | median us | FETCH_SIZE MB | WRITE_SIZE MB | must-read MB | fetch / must-read |")
    print("|---|---|---|---|---|---|")
    for _, k, dt, fm, wm in rows[:12]:
        known = next((v for key, v in KNOWN_MB.items() if key in k), None)
        name = k.replace("void ", "").replace("(anonymous namespace)::", "")[:60]
        print(f"| `{name}` | {dt:.1f} | {fm:.1f} | {wm:.2f} | {known:.1f} | {fm / known:.3f} |" if known else
              f"| `{name}` | {dt:.1f} | {fm:.1f} | {wm:.2f} | - | - |")


if __name__ == "__main__":
    main()
