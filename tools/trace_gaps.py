"""GPU idle time from a rocprofv3 kernel_trace.csv: union of kernel intervals over the traced window, the
idle gaps between them bucketed by length, and the largest gaps with the kernels on either side (what the
host was doing then is the question the gap asks).

python tools/trace_gaps.py '/tmp/prof_b/**/*kernel_trace.csv' [--from-frac 0.5 | --last-ms 7000] [--top 25] [-o gaps.json]
--from-frac: only the last part of the trace (skip model build / warmup: the timed steps are at the end).
"""
import argparse
import csv
import glob
import json
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--from-frac", type=float, default=0.0)
    ap.add_argument("--last-ms", type=float, default=0.0, help="only the last this-many ms of the trace")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("-o", "--out", default=None)
    a = ap.parse_args()
    ev = []
    for f in sorted(glob.glob(a.path, recursive=True)):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Kernel_Name", "?")))
    if not ev:
        sys.exit(f"no trace rows in {a.path}")
    ev.sort()
    t0, t1 = ev[0][0], max(e for _, e, _ in ev)
    cut = t1 - a.last_ms * 1e6 if a.last_ms else t0 + a.from_frac * (t1 - t0)
    ev = [x for x in ev if x[0] >= cut]
    busy, gaps = 0, []
    cs, ce, last = ev[0][0], ev[0][1], ev[0][2]
    for s, e, n in ev[1:]:
        if s > ce:
            busy += ce - cs
            gaps.append((s - ce, last, n, ce))
            cs, ce = s, e
        elif e > ce:
            ce = e
        last = n if e >= ce else last
    busy += ce - cs
    span = ce - ev[0][0]
    buckets = {"<5us": 0, "5-50us": 0, "50-500us": 0, "0.5-5ms": 0, ">5ms": 0}
    counts = dict.fromkeys(buckets, 0)
    for g, *_ in gaps:
        k = "<5us" if g < 5e3 else "5-50us" if g < 5e4 else "50-500us" if g < 5e5 else "0.5-5ms" if g < 5e6 else ">5ms"
        buckets[k] += g
        counts[k] += 1
    gaps.sort(reverse=True)
    res = {"span_ms": span / 1e6, "busy_ms": busy / 1e6, "busy_frac": busy / span, "kernels": len(ev),
           "idle_ms_by_gap_length": {k: round(v / 1e6, 3) for k, v in buckets.items()},
           "gaps_by_length": counts,
           "largest": [{"gap_us": round(g / 1e3, 1), "at_ms": round((t - ev[0][0]) / 1e6, 2), "after": p[:90],
                        "before": n[:90]} for g, p, n, t in gaps[: a.top]]}
    txt = json.dumps(res, indent=1)
    if a.out:
        open(a.out, "w").write(txt)
    print(txt)


if __name__ == "__main__":
    main()
