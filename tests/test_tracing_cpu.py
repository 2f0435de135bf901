"""Tracing (C6, T5/T6): component spans for retriever / reranker / LLM stream carry scores, TTFT and
process metrics, nest under the request span, and export as OTLP JSON."""
import json

import torch

from generativeaiexamples_amd.chain_server import tracing
from generativeaiexamples_amd.chain_server.connectors import ChatLLM, Embeddings, Ranker
from generativeaiexamples_amd.chain_server.vectorstore import VectorStore
from generativeaiexamples_amd.index.hbm_index import Document


class _Emb(Embeddings):
    dim = 16

    def embed_tensor(self, texts, input_type):
        g = torch.Generator().manual_seed(len(texts))
        return torch.nn.functional.normalize(torch.randn(len(texts), self.dim, generator=g), dim=-1)


class _Rank(Ranker):
    def rank(self, query, passages):
        return sorted(((i, float(len(p))) for i, p in enumerate(passages)), key=lambda x: -x[1])


class _LLM(ChatLLM):
    model = "fake"

    def stream(self, messages, **override):
        yield from ["a", "b", "c"]


def test_component_spans_exported(tmp_path, monkeypatch):
    out = tmp_path / "spans.jsonl"
    monkeypatch.setattr(tracing, "ENABLED", True)
    monkeypatch.setattr(tracing.EXPORTER, "file", str(out))
    vs = VectorStore("t", _Emb(), device="cpu")
    vs.add_documents([Document(f"doc {i}", {"filename": "f"}) for i in range(10)])
    with tracing.span("generate", None) as root:
        hits = vs.similarity_search_with_relevance_scores("q", k=3)
        _Rank(top_n=2).compress_documents([d for d, _ in hits], "q")
        assert "".join(_LLM().traced_stream([{"role": "user", "content": "hi"}])) == "abc"
    tracing.EXPORTER.flush()
    spans = [s for line in out.read_text().splitlines()
             for s in json.loads(line)["resourceSpans"][0]["scopeSpans"][0]["spans"]]
    by = {s["name"]: s for s in spans}
    assert {"generate", "retriever.similarity_search_with_relevance_scores", "reranker.compress_documents",
            "llm.stream"} <= set(by)
    attrs = {a["key"] for a in by["llm.stream"]["attributes"]}
    assert {"first_token_time_ms", "llm.model", "process.memory.rss_bytes"} <= attrs
    assert "retriever.scores" in {a["key"] for a in by["retriever.similarity_search_with_relevance_scores"]["attributes"]}
    root_id = by["generate"]["spanId"]
    assert by["llm.stream"]["parentSpanId"] == root_id and by["reranker.compress_documents"]["parentSpanId"] == root_id
