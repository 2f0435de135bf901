import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built _C extension")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from generativeaiexamples_amd import ops

    ops.native()  # fail loudly if the extension is missing on a GPU box
    return torch.device("cuda:0")
