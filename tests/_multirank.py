"""Parent side of the one-GPU multi-rank rehearsals (custom all-reduce, TP and EP decode graphs): start the ranks,
sample the node's KFD queue census while they run, and judge co-residency from the ranks' own probes
(`_dist_workers.coresidency_probe`) instead of a timeout."""
import json
import socket
import threading
import time
from dataclasses import dataclass, field
from typing import Dict, List

import torch.multiprocessing as mp

from tests import _dist_workers as W


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@dataclass
class RankRun:
    procs: list
    late: List[bool]
    wall_s: float
    peak: Dict = field(default_factory=dict)  # max processes / queues on the node while the ranks ran
    base: Dict = field(default_factory=dict)  # census before the ranks started

    @property
    def exitcodes(self):
        return [p.exitcode for p in self.procs]


def run_ranks(target, world: int, args, deadline_s: float) -> RankRun:
    """Spawn ``world`` ranks of ``target(rank, world, *args)``, join them within ``deadline_s`` (late ranks are
    killed), sampling the KFD census every 0.5 s."""
    from tools.queue_census import census

    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=target, args=(r, world, *args)) for r in range(world)]
    peak, stop = {"procs": 0, "queues": 0}, threading.Event()

    def sample():
        while not stop.wait(0.5):
            c = census()
            if c["queues"] > peak["queues"] or c["procs"] > peak["procs"]:
                peak.update(procs=max(peak["procs"], c["procs"]), queues=max(peak["queues"], c["queues"]))
            for g, pids in c.get("per_gpu", {}).items():
                seen = peak.setdefault("per_gpu", {}).setdefault(g, {})
                for pid, n in pids.items():
                    seen[pid] = max(seen.get(pid, 0), n)

    base = census()
    mon = threading.Thread(target=sample, daemon=True)
    mon.start()
    t0 = time.monotonic()
    for p in procs:
        p.start()
    deadline = t0 + deadline_s
    for p in procs:
        p.join(max(1.0, deadline - time.monotonic()))
    stop.set()
    late = [p.is_alive() for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
            p.join(10)
    return RankRun(procs, late, time.monotonic() - t0, peak, base)


def probes(out_dir, tag: str, world: int) -> Dict[int, float]:
    res = {}
    for r in range(world):
        f = out_dir / f"{tag}_probe_{r}.json"
        if f.exists():
            res[r] = json.loads(f.read_text())["us_per_call"]
    return res


def assert_coresident(out_dir, tag: str, world: int, run: RankRun) -> Dict[int, float]:
    """Fail (never skip) when a rank's probe all-reduce shows time-slicing, with the census that explains it."""
    pr = probes(out_dir, tag, world)
    slow = {r: round(us, 1) for r, us in pr.items() if us > W.CORESIDENT_US}
    assert not slow, (f"{world} ranks are not co-resident on the GPU (time-sliced): probe us/all-reduce {slow} > "
                      f"{W.CORESIDENT_US}; KFD census before {run.base.get('per_gpu')} peak {run.peak}")
    return pr
