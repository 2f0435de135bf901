"""Embedding fine-tuning: differentiable encoder == serving encoder, contrastive training
improves retrieval, checkpoint/resume, HF export round trip, DP=2 over gloo."""
import socket

import pytest
import torch
import torch.multiprocessing as mp

from generativeaiexamples_amd.engine.embedder import Embedder
from generativeaiexamples_amd.engine.tokenizer import bert_byte_tokenizer
from generativeaiexamples_amd.models.bert import BertConfig, BertModel
from generativeaiexamples_amd.training import embed_ft as E

from . import _dist_workers as W


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _emb(**kw):
    enc = BertModel(BertConfig.tiny(**kw), device="cpu").random_init(1)
    return Embedder(enc, bert_byte_tokenizer(2048))


@pytest.mark.parametrize("kw", [{}, dict(hidden_size=192, num_heads=6, intermediate_size=384)])
def test_training_forward_matches_serving(kw):
    emb = _emb(**kw)  # second case: head_dim 32 zero-padded to 64
    texts = ["a short one", "a somewhat longer passage of text for the encoder", "x"]
    ref = emb.embed(texts, "passage").float()
    ft = E.EmbedFineTuner(emb, E.EmbedFTConfig(global_batch=2, micro_batch=2), E.synthetic_pairs(4))
    with torch.no_grad():
        got = ft._encode(texts, "passage")
    torch.testing.assert_close(got, ref, rtol=0, atol=3e-2)


def test_contrastive_training_improves_recall(tmp_path):
    torch.manual_seed(0)
    emb = _emb(num_layers=1)
    rows = E.synthetic_pairs(64)
    before = E.recall_at_k(emb, rows[:32], k=1)
    cfg = E.EmbedFTConfig(global_batch=16, micro_batch=8, lr=3e-4, max_steps=24, tau=0.05, save_every=12,
                          out=str(tmp_path / "run"))
    ft = E.EmbedFineTuner(emb, cfg, rows)
    hist = ft.fit()
    after = E.recall_at_k(emb, rows[:32], k=1)  # fit() synced the tuned weights into the serving model
    assert sum(hist[-4:]) < sum(hist[:4]), hist
    assert after > before, (before, after)
    # resume: a fresh tuner on the same --out picks up step 24 and does nothing more
    ft2 = E.EmbedFineTuner(_emb(num_layers=1), cfg, rows)
    ft2._maybe_resume()
    assert ft2.step == 24
    torch.testing.assert_close(ft2.w["l0.up"], ft.w["l0.up"])
    # HF export -> build_encoder(weights=dir) reproduces the tuned embeddings
    from generativeaiexamples_amd.models.registry import build_encoder

    ft.export_hf(str(tmp_path / "hf"))
    m2, _, _ = build_encoder("tiny-e5", str(tmp_path / "hf"), device="cpu")
    e2 = Embedder(m2, bert_byte_tokenizer(2048))
    torch.testing.assert_close(e2.embed(["query: hello"], "query"), emb.embed(["query: hello"], "query"))


@pytest.mark.timeout(300)
def test_embed_ft_dp2(tmp_path):
    mp.spawn(W.embed_ft_dp_worker, args=(2, _port(), str(tmp_path)), nprocs=2, join=True)
    d0, d1 = (torch.load(tmp_path / f"eft_{r}.pt", weights_only=True) for r in range(2))
    torch.testing.assert_close(d0["w"], d1["w"])
    torch.testing.assert_close(d0["hist"], d1["hist"])
    assert d0["hist"][-1] < d0["hist"][0]
