"""One-shot peer-memory all-reduce (csrc/comm/custom_ar.hip, parallel/custom_ar.py) on a one-GPU
box: 2, 4 and 8 ranks (the Llama-3-70B TP8 instantiation) share cuda:0 and exchange IPC handles over gloo; the result must equal the
fp32 sum of every rank's input (eager and HIP-graph replay). Multi-GPU xGMI runs go through the
same kernel with peers on other devices."""
import json
import socket

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


@pytest.mark.parametrize("world", [2, 4, 8])
def test_custom_allreduce_matches_sum(tmp_path, world, cuda):
    ctx = mp.get_context("spawn")
    port = _port()
    procs = [ctx.Process(target=W.custom_ar_worker, args=(r, world, port, str(tmp_path))) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(100)
    for p in procs:
        if p.is_alive():
            p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    for r in range(world):
        res = json.loads((tmp_path / f"car_{r}.json").read_text())
        assert res["errors"] == [], res["errors"]
        print(f"world {world} rank {r}: 1 MiB all-reduce {res['us_1MiB']:.1f} us (shared GPU)")
