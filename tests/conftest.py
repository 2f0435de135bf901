import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built _C extension")
    config.addinivalue_line("markers", "slow: long-running test")
    config.addinivalue_line("markers", "multirank: spawns several GPU processes that share one GPU (run first)")


def pytest_collection_modifyitems(session, config, items):
    """Multi-rank one-GPU rehearsals run before every other test: their ranks' spin-waiting collectives need all
    of the ranks' queues mapped on the GPU at once, and the hardware scheduler maps at most 8 processes with
    queues concurrently - a pytest parent that has already launched kernels (and so holds queues) would make an
    8-rank rehearsal the 9th process and time-slice it (evidence in profiles/r4/tp8_suite)."""
    first = [it for it in items if it.get_closest_marker("multirank") is not None]
    if first:
        rest = [it for it in items if it.get_closest_marker("multirank") is None]
        items[:] = first + rest


@pytest.fixture(scope="session")
def gpu_box():
    """For the multi-rank rehearsals: a GPU is present and the extension loads, checked WITHOUT initialising HIP in
    this (parent) process - device_count() does not on this image - so the parent holds no hardware queue while the
    ranks it spawns spin-wait on each other."""
    import torch

    if torch.cuda.device_count() < 1:
        pytest.skip("no GPU")
    from generativeaiexamples_amd import ops

    ops.native()


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from generativeaiexamples_amd import ops

    ops.native()  # fail loudly if the extension is missing on a GPU box
    return torch.device("cuda:0")
