"""Context parallelism: zigzag sharding, exact LSE merge of partial attentions, and ring
attention over 2 / 4 gloo ranks matching full attention (causal and bidirectional)."""
import json
import math
import socket

import pytest
import torch
import torch.multiprocessing as mp

from generativeaiexamples_amd.ops import reference as ref
from generativeaiexamples_amd.parallel import context_parallel as cp
from tests import _dist_workers as W


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_zigzag_roundtrip_and_balance():
    x = torch.arange(48).view(48, 1)
    shards = [cp.zigzag_shard(x, r, 3) for r in range(3)]
    assert torch.equal(cp.zigzag_unshard(shards), x)
    assert torch.equal(cp.zigzag_positions(48, 1, 3), shards[1].view(-1))
    # causal work (sum of key counts over a rank's rows) is equal across ranks
    work = [int((shards[r].view(-1) + 1).sum()) for r in range(3)]
    assert len(set(work)) == 1, work


def test_lse_merge_is_exact():
    torch.manual_seed(0)
    T, Hq, Hkv, D = 40, 4, 2, 64
    q = torch.randn(T, Hq, D).bfloat16()
    k = torch.randn(2 * T, Hkv, D).bfloat16()
    v = torch.randn(2 * T, Hkv, D).bfloat16()
    s = 1 / math.sqrt(D)
    o1, l1 = cp.block_attention(q, k[:T], v[:T], s, causal=False)
    o2, l2 = cp.block_attention(q, k[T:], v[T:], s, causal=True)
    o, _ = cp.merge_partial(*cp.merge_partial(None, None, o1, l1), o2, l2)
    # causal over the second half with queries aligned to its end == full causal over [first, second]
    # for the last T queries of a 2T sequence:
    qq = torch.cat([torch.zeros(T, Hq, D).bfloat16(), q])
    want = ref.attention_dense(qq, k, v, torch.tensor([0, 2 * T], dtype=torch.int32), s, True)[T:]
    assert (o - want.float()).abs().max() < 2e-2


@pytest.mark.timeout(240)
@pytest.mark.parametrize("world,causal", [(2, 1), (4, 1), (2, 0)])
def test_ring_attention_matches_full(tmp_path, world, causal):
    mp.spawn(W.cp_ring_worker, args=(world, _port(), str(tmp_path), causal), nprocs=world, join=True)
    for r in range(world):
        err = json.loads((tmp_path / f"cp_{r}.json").read_text())["err"]
        assert err < 3e-2, (r, err)
