"""TP=2/4/8 decode captured in HIP graphs on ONE GPU: every rank shares
cuda:0 over a gloo control plane; the only collectives inside the multi-step decode graph are the
peer-memory custom all-reduce kernels (including ops.sample_tp's candidate exchange, which replaces the
[B, vocab] logits all-gather). Every greedy token must be the fp32 reference argmax of its prefix up to a
bf16 near-tie (the criterion of the CPU engine tests).

World 8 (tiny and Llama-3-70B widths) runs in the suite and must PASS: the ranks' co-residency on the GPU is a
checked precondition (each rank's probe all-reduce, tests/_multirank.py) - a time-sliced run fails with the KFD
queue census, a stall of co-resident ranks fails as a hang. There is no environment skip."""
import json

import pytest

from tests import _dist_workers as W
from tests import _multirank as M

pytestmark = [pytest.mark.gpu, pytest.mark.multirank]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world,shape", [(2, "tiny"), (4, "tiny"), (8, "tiny"), (8, "70b")])
def test_tp_decode_graph_one_gpu(tmp_path, world, shape, gpu_box):
    run = M.run_ranks(W.tp_graph_rehearsal_worker, world, (M.free_port(), str(tmp_path), shape),
                      300 if world == 8 else 170)
    print(f"TP={world}: wall {run.wall_s:.1f}s, KFD census peak {run.peak}")
    for r in range(world):
        f = tmp_path / f"tpg_progress_{r}.txt"
        lines = f.read_text().splitlines() if f.exists() else []
        if any(run.late) or r == 0:
            print(f"rank {r} progress ({len(lines)} lines): " + " | ".join(lines[:3] + (["..."] if len(lines) > 6 else [])
                                                                       + lines[max(3, len(lines) - 3):]))
    pr = M.assert_coresident(tmp_path, "tpg", world, run)
    print(f"TP={world}: co-residency probe us/all-reduce {[round(v, 1) for v in pr.values()]}")
    errs = [f.read_text() for f in tmp_path.glob("tpg_err_*.txt")]
    assert not errs, errs[0]
    assert not any(run.late), f"co-resident ranks hung: still running at the deadline {run.late}"
    assert all(c == 0 for c in run.exitcodes), run.exitcodes
    res = json.loads((tmp_path / "tpg.json").read_text())
    print(f"TP={world} ({shape}): {res['total'] - len(res['bad'])}/{res['total']} tokens fp32-consistent, stats {res['stats']}, "
          f"flags {res['flags']}")
    assert res["multi_graphs"], "no multi-step decode graph captured"
    assert res["stats"]["graph_steps"] > 0 and res["stats"]["chained_runs"] > 0
    assert not res["bad"], res["bad"][:5]
