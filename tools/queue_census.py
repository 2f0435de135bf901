"""Census of GPU hardware queues and GPU-attached processes from KFD sysfs (/sys/class/kfd/kfd/proc/<pid>/queues):
how many processes and queues the hardware scheduler must map at once. Used by the one-GPU multi-rank rehearsals
to record the process / queue load next to a slow or hung run.

python tools/queue_census.py [--interval 1 --samples 30]   (or import census())
"""
import argparse
import json
import os
import time

ROOT = "/sys/class/kfd/kfd/proc"


def census() -> dict:
    """{'procs': n, 'queues': n, 'per_pid': {pid: queues}, 'per_gpu': {gpu_id: {pid: queues}}} over the whole node
    (KFD lists every process of every GPU; queues/<q>/gpuid says which GPU a queue is on). Empty when KFD sysfs is
    not visible."""
    out = {"procs": 0, "queues": 0, "per_pid": {}, "per_gpu": {}}
    if not os.path.isdir(ROOT):
        out["error"] = "no KFD sysfs"
        return out
    for pid in os.listdir(ROOT):
        qd = os.path.join(ROOT, pid, "queues")
        try:
            qs = os.listdir(qd)
        except OSError:
            qs = None
        out["per_pid"][pid] = -1 if qs is None else len(qs)
        out["procs"] += 1
        out["queues"] += len(qs or [])
        for q in qs or []:
            try:
                with open(os.path.join(qd, q, "gpuid")) as f:
                    gid = f.read().strip()
            except OSError:
                continue
            g = out["per_gpu"].setdefault(gid, {})
            g[pid] = g.get(pid, 0) + 1
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--interval", type=float, default=1.0)
    ap.add_argument("--samples", type=int, default=1)
    a = ap.parse_args()
    for _ in range(a.samples):
        print(json.dumps(census()), flush=True)
        time.sleep(a.interval)


if __name__ == "__main__":
    main()
