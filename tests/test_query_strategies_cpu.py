"""Retrieval strategies + fact check of the multimodal / O-RAN assistants: plain, multi-query (one
batched embed + scan for all augmented queries), HyDE, rephrasing multi-query, history-aware rewrite, fact-check
verdicts and the assistant turn - scripted LLM, crc32 hashing embedder, CPU."""
import zlib

import pytest
import torch

from generativeaiexamples_amd.chain_server.connectors import Embeddings
from generativeaiexamples_amd.chain_server.vectorstore import VectorStore
from generativeaiexamples_amd.index.hbm_index import Document
from generativeaiexamples_amd.rag import query_strategies as qs

PASSAGES = [("O-RAN fronthaul uses the 7.2x split between the O-DU and the O-RU.", "fronthaul.pdf"),
            ("The near-RT RIC hosts xApps that control RAN functions over the E2 interface.", "ric.pdf"),
            ("The non-RT RIC runs rApps and provides A1 policies to the near-RT RIC.", "ric.pdf"),
            ("Bananas are rich in potassium.", "fruit.txt")]


class _Emb(Embeddings):
    dim = 64

    def embed_tensor(self, texts, input_type):
        out = torch.zeros(len(texts), self.dim)
        for i, t in enumerate(texts):
            for w in t.lower().replace("-", " ").split():
                out[i, zlib.crc32(w.strip(".,?").encode()) % self.dim] += 1.0
        return torch.nn.functional.normalize(out + 1e-3, dim=-1)


class _LLM:
    def __init__(self, check="TRUE - every claim is in the context."):
        self.check, self.calls = check, []

    def invoke(self, messages, **kw):
        sys_ = messages[0]["content"]
        self.calls.append(sys_[:16])
        if sys_ == qs.RELATED_QUESTIONS:
            return "1. What is the near-RT RIC?\n2. What are xApps?\n- What does the E2 interface carry?\n\n"
        if sys_ == qs.REPHRASINGS:
            return "Which split does fronthaul use?\nFronthaul split option?\nWhat split is used between O-DU and O-RU?"
        if sys_ == qs.HYPOTHETICAL_ANSWER:
            return "xApps run on the near-RT RIC and use the E2 interface."
        if sys_ == qs.REWRITE_WITH_HISTORY:
            return "What interface do xApps on the near-RT RIC use?"
        return "?"

    def stream(self, messages, **kw):
        if messages[0]["content"] == qs.FACT_CHECK:
            yield from [self.check[:4], self.check[4:]]
        else:
            yield from ["They use ", "E2."]


@pytest.fixture()
def store():
    s = VectorStore("oran", _Emb(), device="cpu")
    s.add_documents([Document(t, {"source": src}) for t, src in PASSAGES])
    return s


def test_plain_and_multi_query_batched(store):
    r = qs.retrieve("plain", _LLM(), store, "What does the near-RT RIC host?", k=2)
    assert r.queries == ["What does the near-RT RIC host?"] and len(r.documents) == 2
    store.batcher.batch_sizes.clear()
    r = qs.retrieve("multi_query", _LLM(), store, "What does the near-RT RIC host?", k=2)
    assert len(r.queries) == 4 and r.queries[1] == "What is the near-RT RIC?"
    assert store.batcher.batch_sizes == [4]  # all augmented queries in ONE embed + scan batch
    texts = [d.page_content for d in r.documents]
    assert len(texts) == len(set(texts)) and PASSAGES[1][0] in texts
    scores = [d.metadata["relevance_score"] for d in r.documents]
    assert scores == sorted(scores, reverse=True)
    assert set(r.sources()) <= {"fronthaul.pdf", "ric.pdf", "fruit.txt"}


def test_hyde_rephrase_and_rewrite(store):
    r = qs.retrieve("hyde", _LLM(), store, "What do xApps use?", k=1)
    assert r.queries[0].startswith("What do xApps use? xApps run on") and r.documents[0].page_content == PASSAGES[1][0]
    r = qs.retrieve("multi_query_retriever", _LLM(), store, "fronthaul split?", k=1, top_n=2)
    assert len(r.queries) == 4 and r.documents[0].page_content == PASSAGES[0][0] and len(r.documents) <= 2
    assert qs.rewrite_with_history(_LLM(), "and which interface?", []) == "and which interface?"
    assert qs.rewrite_with_history(_LLM(), "and which interface?", [("What are xApps?", "RIC apps")]).startswith(
        "What interface")
    with pytest.raises(ValueError):
        qs.retrieve("nope", _LLM(), store, "q")


def test_reranker_scores_against_original_question(store):
    class Ranker:
        top_n = 3

        def __init__(self):
            self.seen = None

        def compress_documents(self, docs, query):
            self.seen = (len(docs), query, self.top_n)
            return list(reversed(docs))[: self.top_n]

    rk = Ranker()
    r = qs.retrieve("multi_query", _LLM(), store, "What does the near-RT RIC host?", k=2, top_n=2, ranker=rk)
    assert rk.seen[1] == "What does the near-RT RIC host?" and rk.seen[2] == 2 and len(r.documents) == 2
    assert rk.top_n == 3  # restored


def test_framework_ranker_takes_top_n_per_call_concurrently():
    """Concurrent requests with different top_n never see each other's value (the shared ranker is not mutated)."""
    import threading

    from generativeaiexamples_amd.chain_server.connectors import Ranker, rerank
    from generativeaiexamples_amd.index.hbm_index import Document

    gate = threading.Barrier(8)

    class Slow(Ranker):
        def rank(self, query, passages):
            gate.wait(timeout=10)  # every call is inside compress_documents at once
            return [(i, 1.0 / (i + 1)) for i in range(len(passages))]

    rk, docs, got = Slow(top_n=4), [Document(f"d{i}", {}) for i in range(10)], {}

    def call(n):
        got[n] = len(rerank(rk, docs, "q", n))

    ts = [threading.Thread(target=call, args=(n,)) for n in range(1, 9)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert got == {n: n for n in range(1, 9)} and rk.top_n == 4


def test_fact_check_and_assistant_turn(store):
    assert qs.parse_fact_check("TRUE. fine").verdict is True
    assert qs.parse_fact_check("**FALSE** the context does not say").verdict is False
    assert qs.parse_fact_check("cannot tell").verdict is None
    assert qs.fact_check(_LLM("FALSE - unsupported"), "ctx", "q", "a").verdict is False
    chain = qs.AssistantChain(_LLM(), store, strategy="plain", describe_image=lambda b: f"a diagram of {len(b)} bytes")
    out = "".join(chain.turn("What do xApps use?", image=b"1234"))
    assert out.startswith("They use E2.") and "Fact check: TRUE" in out
    assert chain.history[0][0].startswith("I have uploaded an image with the following description: a diagram of 4")
    out2 = "".join(chain.turn("and which interface?"))  # second turn: rewritten against the history
    assert chain.history[1][0] == "What interface do xApps on the near-RT RIC use?" and "Fact check" in out2
