"""One-shot peer-memory all-reduce (csrc/comm/custom_ar.hip, parallel/custom_ar.py) on a one-GPU
box: 2, 4 and 8 ranks (the Llama-3-70B TP8 instantiation) share cuda:0 and exchange IPC handles over gloo; the result must equal the
fp32 sum of every rank's input (eager and HIP-graph replay). Multi-GPU xGMI runs go through the
same kernel with peers on other devices. Co-residency of the ranks is a checked precondition (a probe
all-reduce per rank, tests/_multirank.py), so a time-sliced world fails with the queue census, not a timeout."""
import json

import pytest

from tests import _dist_workers as W
from tests import _multirank as M

pytestmark = [pytest.mark.gpu, pytest.mark.multirank]


@pytest.mark.parametrize("world", [2, 4, 8])
def test_custom_allreduce_matches_sum(tmp_path, world, gpu_box):
    run = M.run_ranks(W.custom_ar_worker, world, (M.free_port(), str(tmp_path)), 100)
    pr = M.assert_coresident(tmp_path, "car", world, run)
    assert not any(run.late), f"ranks still running at the deadline: {run.late}; census {run.peak}"
    assert all(c == 0 for c in run.exitcodes), run.exitcodes
    for r in range(world):
        res = json.loads((tmp_path / f"car_{r}.json").read_text())
        assert res["errors"] == [], res["errors"]
        print(f"world {world} rank {r}: probe {pr.get(r, float('nan')):.1f} us, 1 MiB all-reduce {res['us_1MiB']:.1f} us "
              "(shared GPU)")
