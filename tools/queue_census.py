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
    """{'procs': n, 'queues': n, 'per_pid': {pid: queues}} (empty when KFD sysfs is not visible)."""
    out = {"procs": 0, "queues": 0, "per_pid": {}}
    if not os.path.isdir(ROOT):
        out["error"] = "no KFD sysfs"
        return out
    for pid in os.listdir(ROOT):
        qd = os.path.join(ROOT, pid, "queues")
        try:
            n = len(os.listdir(qd))
        except OSError:
            n = -1
        out["per_pid"][pid] = n
        out["procs"] += 1
        out["queues"] += max(n, 0)
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
