"""Distributed correctness on the CPU tier: 2 processes over gloo (127.0.0.1).

* tensor-parallel Llama (column/row-parallel linears, vocab-parallel embedding + LM head, TP
  all-reduces) reproduces the single-process logits;
* the DP-sharded index (all-gather of queries and candidates + merge) equals a global exact top-k.
"""
import json
import socket

import pytest
import torch
import torch.multiprocessing as mp

from tests import _dist_workers as W


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(300)
@pytest.mark.parametrize("overlap_rows", [None, 8])
def test_tp2_llama_matches_tp1(tmp_path, overlap_rows):
    """TP=2 logits == TP=1; with overlap_rows the O / down projections take the row-chunked GEMM +
    asynchronous all-reduce path of TP prefill (chunks of 8 rows on these short prompts)."""
    mp.spawn(W.tp_llama_worker, args=(2, _port(), str(tmp_path), overlap_rows), nprocs=2, join=True)
    for r in range(2):
        d = torch.load(tmp_path / f"tp_{r}.pt", weights_only=True)
        err = (d["tp"] - d["ref"]).abs().max().item()
        assert err < 0.03 * d["ref"].abs().max().item() + 0.03, err


@pytest.mark.timeout(300)
def test_expert_parallel_all_to_all(tmp_path):
    mp.spawn(W.ep_worker, args=(2, _port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        d = torch.load(tmp_path / f"ep_{r}.pt", weights_only=True)
        assert (d["out"] - d["exp"]).abs().max().item() < 2e-2


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 4, 8])
def test_ep_padded_dispatch(tmp_path, world):
    """Fixed-capacity, sync-free EP exchange (the graph-capturable decode path) at 2, 4 and 8 ranks."""
    mp.spawn(W.ep_padded_worker, args=(world, _port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        d = torch.load(tmp_path / f"ep_padded_{r}.pt", weights_only=True)
        assert (d["out"] - d["exp"]).abs().max().item() < 3e-2
        assert torch.isfinite(d["out1"]).all()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("max_queries", [None, 8])
def test_sharded_index_matches_global(tmp_path, max_queries):
    """max_queries: the padded, sync-free exchange (no count all-gather), uneven batches per rank."""
    mp.spawn(W.sharded_index_worker, args=(2, _port(), str(tmp_path), max_queries), nprocs=2, join=True)
    for r in range(2):
        d = torch.load(tmp_path / f"idx_{r}.pt", weights_only=True)
        assert d["got"] == d["exp"]
        assert torch.allclose(d["rel"].float(), d["exp_v"].float(), atol=2e-2)


@pytest.mark.timeout(300)
def test_tp2_sequence_parallel_matches(tmp_path):
    """reduce-scatter / all-gather sequence parallelism gives the all-reduce TP logits (and TP=1),
    including a token count that is not a multiple of tp (padded rows) and biased row-parallel layers."""
    mp.spawn(W.tp_sp_worker, args=(2, _port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        d = torch.load(tmp_path / f"sp_{r}.pt", weights_only=True)
        for name, res in d.items():
            scale = res["ref"].abs().max().item()
            assert (res["sp"] - res["tp"]).abs().max().item() < 0.02 * scale + 0.02, name
            assert (res["sp"] - res["ref"]).abs().max().item() < 0.03 * scale + 0.03, name


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [2, 4, 8])
def test_tp_engine_follows_leader_plans(tmp_path, world):
    """Rank-0-scheduled TP engine (step plans over the shared-memory channel) == single-process engine."""
    import json

    mp.spawn(W.tp_engine_worker, args=(world, _port(), str(tmp_path)), nprocs=world, join=True)
    d = json.loads((tmp_path / "tp_engine.json").read_text())
    assert d["tp"] == d["ref"], (d["tp"], d["ref"])
    assert d["victim"] == "abort" and d["victim_len"] < 40
    assert d["free_ok"] and d["multi"] > 0 and d["plans"] > 5


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [2, 4])
def test_tp_serving_hub(tmp_path, world):
    """/v1 chat on a TP=world generator served from rank 0 == single-process engine on the same checkpoint;
    an aborted stream leaves the ranks in step; shutdown ends the follower loops."""
    import json

    ckpt = str(tmp_path / "ckpt")
    W.write_tiny_llama_ckpt(ckpt)
    mp.spawn(W.tp_serving_worker, args=(world, _port(), str(tmp_path), ckpt), nprocs=world, join=True)
    d = json.loads((tmp_path / "tp_serving.json").read_text())
    assert d["api"] == d["ref"], (d["api"], d["ref"])
    assert d["after_abort"] == d["ref"][1]


@pytest.mark.timeout(300)
def test_tp_linear_all_reduce_overlap(tmp_path):
    """Row-chunked row-parallel GEMM with asynchronous per-chunk all-reduces (the TP prefill overlap path)
    matches the plain GEMM + all-reduce, fp32 and bf16, 2 ranks."""
    mp.spawn(W.tp_linear_overlap_worker, args=(2, _port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        d = torch.load(tmp_path / f"ovl_{r}.pt", weights_only=True)
        assert d["torch.float32"] < 1e-4
        assert d["torch.bfloat16"] < 1e-2


@pytest.mark.parametrize("world,chunk", [(2, 0), (4, 0), (8, 0), (2, 5)])
def test_ep_engine_matches_single_rank(tmp_path, monkeypatch, world, chunk):
    """Mixtral EP mode: DP attention + experts over the ranks with all-to-all exchange, lockstep steps (ranks
    own different request sets): every rank's greedy tokens equal the single-process model's. chunk > 0: prefill
    exchanges run in row chunks of that many tokens (the path for slabs beyond the peer-memory buffers), ranks that
    run out of rows join with a zero-weight dummy row."""
    if chunk:
        monkeypatch.setenv("GAI_EP_PREFILL_CHUNK_TOKENS", str(chunk))
    mp.spawn(W.ep_engine_worker, args=(world, _port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        d = json.loads((tmp_path / f"ep_{r}.json").read_text())
        assert d["e_local"] == 8 // world
        assert d["ep"] == d["ref"], (r, d)
