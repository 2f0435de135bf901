"""Graph capture order: the engine captures its decode graphs lazily inside ``LLMEngine.step()`` (inference mode);
a later capture outside inference mode in the same process must still work (utils/graphs.py registers the CUDA
generator's graph state outside inference mode first). Run in a fresh process so the order is the one under test."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

SCRIPT = r"""
import torch
from generativeaiexamples_amd.utils.graphs import hip_graph_capture

x = torch.zeros(4, device="cuda")
s = torch.cuda.Stream()
with torch.inference_mode():
    g1 = torch.cuda.CUDAGraph()
    with hip_graph_capture(g1, s):
        y = x + 1
g2 = torch.cuda.CUDAGraph()
with hip_graph_capture(g2, s):
    x.mul_(2)
g1.replay(); g2.replay()
torch.cuda.synchronize()
print("capture-order ok", float(y.sum()))
"""


def test_capture_in_inference_mode_then_outside():
    env = dict(os.environ, PYTHONPATH=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    r = subprocess.run([sys.executable, "-c", SCRIPT], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "capture-order ok 4.0" in r.stdout, r.stderr[-2000:]
