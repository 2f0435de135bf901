"""Reduce a rocprofv3 ``--stats`` kernel_stats.csv to the compact per-kernel CSV kept under profiles/
(kernel, calls, total_ms, avg_us, pct), plus the total GPU kernel time.

python tools/rocprof_summary.py gpurun_out/prof/<host>/<pid>_kernel_stats.csv [-o profiles/rN/x.csv] [--top 40]
"""
import argparse
import csv
import glob
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path", help="kernel_stats.csv (a glob is accepted)")
    ap.add_argument("-o", "--out", default=None)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--by-grid", action="store_true",
                    help="path is a kernel_trace.csv: one row per (kernel, grid size) - tells apart the shapes "
                         "one template serves (e.g. QKV vs O projections)")
    a = ap.parse_args()
    files = sorted(glob.glob(a.path, recursive=True))
    if not files:
        sys.exit(f"no file matches {a.path}")
    rows = {}
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if a.by_grid:
                    grid = "x".join(r.get(f"Grid_Size_{d}", "?") for d in "XYZ")
                    name = f"{r.get('Kernel_Name', '?')} grid={grid}"
                    calls, tot = 1, float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
                else:
                    name = r.get("Name") or r.get("KernelName")
                    calls = int(r.get("Calls", 0))
                    tot = float(r.get("TotalDurationNs", 0))
                c, t = rows.get(name, (0, 0.0))
                rows[name] = (c + calls, t + tot)
    total = sum(t for _, t in rows.values()) or 1.0
    out = [(n, c, t / 1e6, t / max(c, 1) / 1e3, 100 * t / total) for n, (c, t) in rows.items()]
    out.sort(key=lambda x: -x[2])
    w = csv.writer(open(a.out, "w", newline="") if a.out else sys.stdout)
    w.writerow(["kernel", "calls", "total_ms", "avg_us", "pct"])
    for n, c, t, avg, pct in out[: a.top]:
        w.writerow([n[:120] + (n[n.rfind(' grid='):] if ' grid=' in n[120:] else ''), c, round(t, 3), round(avg, 2), round(pct, 2)])
    print(f"# total GPU kernel time {total / 1e6:.1f} ms over {sum(c for _, (c, _) in rows.items())} launches",
          file=sys.stderr)


if __name__ == "__main__":
    main()
