"""Community apps on the MI355X: the sizing advisor's GPU detection and its measured test run of a configuration on
this framework's engine (tiny preset so the run is seconds)."""
import pytest

pytestmark = pytest.mark.gpu


def test_detect_gpu_reports_mi355x():
    from generativeaiexamples_amd.community.sizing_advisor.deploy import detect_gpu

    info = detect_gpu()
    assert info is not None and info["gpu_count"] >= 1 and info["gpu_memory_mb"] > 100_000
    assert info["gpu_model"] == "MI355X" or "gfx950" in info["arch"], info


def test_measure_config_runs_engine_wave():
    from generativeaiexamples_amd.community.sizing_advisor.deploy import measure_config

    m = measure_config("tiny-llama", concurrency=4, prompt=64, response=16, use_graphs=True)
    assert m["concurrency"] == 4 and 0 < m["ttft_p50_s"] <= m["ttft_max_s"] < 30
    assert m["tpot_ms"] > 0 and m["output_tokens_per_s"] > 0 and m["wall_s"] > 0


def test_multi_query_retrieval_one_batch_on_gpu():
    """The assistants' augmented queries go through the store's batcher as ONE encoder batch + ONE index scan on the
    GPU, and return what per-query searches return."""
    import torch

    from generativeaiexamples_amd.chain_server.connectors import LocalEmbeddings
    from generativeaiexamples_amd.chain_server.vectorstore import VectorStore
    from generativeaiexamples_amd.engine.embedder import Embedder
    from generativeaiexamples_amd.index.hbm_index import Document
    from generativeaiexamples_amd.models.registry import build_encoder
    from generativeaiexamples_amd.rag import query_strategies as qs

    m, tok, name = build_encoder("tiny-e5", device="cuda")
    store = VectorStore("mq", LocalEmbeddings(Embedder(m, tok, model_name=name)), device="cuda")
    texts = [f"passage {i} about topic {i % 7} and subject {i % 5}" for i in range(300)]
    store.add_documents([Document(t, {"filename": f"f{i}"}) for i, t in enumerate(texts)])
    queries = [f"topic {i} subject {i % 5}" for i in range(6)]
    store.batcher.batch_sizes.clear()
    batched = qs.batched_search(store, queries, 4)
    assert store.batcher.batch_sizes == [6]
    for q, hits in zip(queries, batched):
        single = store.similarity_search_with_relevance_scores(q, 4)
        # a batch of 6 and a batch of 1 may take different encoder GEMM walks: equal up to bf16 rounding
        assert hits[0][0].page_content == single[0][0].page_content or abs(hits[0][1] - single[0][1]) < 2e-2
        torch.testing.assert_close(torch.tensor([s for _, s in hits]), torch.tensor([s for _, s in single]),
                                   atol=2e-2, rtol=0)
