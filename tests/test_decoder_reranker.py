"""Decoder-based (NV-RerankQA-Mistral-4B class) cross-encoder reranker vs its dense fp32 reference."""
import pytest
import torch

from generativeaiexamples_amd.engine.embedder import DecoderReranker
from generativeaiexamples_amd.engine.tokenizer import small_byte_tokenizer
from generativeaiexamples_amd.models.decoder_reranker import DecoderRerankerConfig, DecoderRerankerModel


def _check(dev):
    m = DecoderRerankerModel(DecoderRerankerConfig.tiny(), device=dev).random_init(2)
    lens = [7, 33, 5, 70]
    ids = torch.randint(3, 500, (sum(lens),), dtype=torch.int32)
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32)
    got = m.score(ids.to(dev), cu.to(dev), lens).cpu()
    ref = m.reference_score(ids, lens)
    torch.testing.assert_close(got, ref, rtol=0.05, atol=0.03)
    svc = DecoderReranker(m, small_byte_tokenizer(512), max_batch_tokens=64)  # forces several micro-batches
    many = svc.score_many([("what is hbm", ["high bandwidth memory", "a fruit", "x" * 50]), ("q2", ["p"])])
    assert [len(x) for x in many] == [3, 1]
    assert abs(svc.score("q2", ["p"])[0] - many[1][0]) < 1e-3


def test_decoder_reranker_cpu():
    _check("cpu")


@pytest.mark.gpu
def test_decoder_reranker_gpu(cuda):
    _check("cuda")
