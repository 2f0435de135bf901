"""Ring attention on the gfx950 prefill kernel: the kernel's LSE output matches the fp32 reference,
and a 2-rank ring (both ranks on cuda:0, K/V shards over gloo) matches full attention."""
import json
import math
import socket

import pytest
import torch
import torch.multiprocessing as mp

from generativeaiexamples_amd.ops import reference as ref
from generativeaiexamples_amd.parallel import context_parallel as cp
from tests import _dist_workers as W

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("D", [64, 128])
def test_prefill_kernel_lse(cuda, causal, D):
    torch.manual_seed(0)
    Tq, Tk, Hq, Hkv = 100, 100 if causal else 173, 8, 2
    q = torch.randn(Tq, Hq, D, device=cuda).bfloat16()
    k = torch.randn(Tk, Hkv, D, device=cuda).bfloat16()
    v = torch.randn(Tk, Hkv, D, device=cuda).bfloat16()
    s = 1 / math.sqrt(D)
    o, lse = cp.block_attention(q, k, v, s, causal)
    o_ref, lse_ref = cp.block_attention(q.cpu(), k.cpu(), v.cpu(), s, causal)
    assert (o.float().cpu() - o_ref.float()).abs().max() < 2e-2
    assert (lse.cpu() - lse_ref).abs().max() < 1e-2


@pytest.mark.multirank
def test_ring_attention_gpu_two_ranks(tmp_path, cuda):
    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=W.cp_ring_worker, args=(r, 2, port, str(tmp_path), 1, "cuda")) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(100)
    for p in ps:
        if p.is_alive():
            p.kill()
    assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]
    for r in range(2):
        assert json.loads((tmp_path / f"cp_{r}.json").read_text())["err"] < 3e-2
