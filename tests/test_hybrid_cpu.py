"""BM25 sparse index, reciprocal-rank fusion and the hybrid / ranked_hybrid retrieval pipelines (S7)."""
import zlib

import torch

from generativeaiexamples_amd.chain_server.connectors import Embeddings
from generativeaiexamples_amd.chain_server.vectorstore import VectorStore
from generativeaiexamples_amd.index.bm25 import BM25Index, rrf
from generativeaiexamples_amd.index.hbm_index import Document


def test_bm25_ranks_exact_term_matches():
    ix = BM25Index()
    docs = ["the infusion pump occlusion alarm E3", "cooking pasta in salted water", "pump priming procedure",
            "occlusion occlusion occlusion downstream alarm"]
    ix.add(range(len(docs)), docs)
    top = [r for r, _ in ix.search("occlusion alarm", 3)]
    assert top[0] in (0, 3) and set(top[:2]) == {0, 3} and 1 not in top
    ix.delete([3])
    assert [r for r, _ in ix.search("occlusion", 3)] == [0]


def test_rrf_prefers_items_in_both_lists():
    fused = [r for r, _ in rrf([[1, 2, 3], [3, 4, 1]], 3)]
    assert fused[:2] == [1, 3] or fused[:2] == [3, 1]
    assert 4 in fused or 2 in fused


class _HashEmb(Embeddings):
    """Deterministic bag-of-words hashing embedder (dense side without a model)."""
    dim = 64

    def embed_tensor(self, texts, input_type):
        out = torch.zeros(len(texts), self.dim)
        for i, t in enumerate(texts):
            for w in t.lower().split():
                out[i, zlib.crc32(w.encode()) % self.dim] += 1.0
        return torch.nn.functional.normalize(out + 1e-3, dim=-1)


def test_vectorstore_hybrid_search_and_delete(tmp_path):
    vs = VectorStore("h", _HashEmb(), device="cpu", hybrid=True)
    docs = [Document(f"manual page {i} about topic{i % 5} with serial SN{i:04d}", {"filename": f"f{i % 3}.txt"})
            for i in range(60)]
    vs.add_documents(docs)
    hits = vs.hybrid_search("serial SN0042", 4)
    assert any(d.page_content.endswith("SN0042") for d, _ in hits)  # exact-token match surfaced by BM25
    assert vs.bm25.search("SN0042", 1)[0][0] == 42
    assert vs.delete_filename("f0.txt")
    assert all(d.metadata["filename"] != "f0.txt" for d, _ in vs.hybrid_search("manual page", 20))
    hits = vs.hybrid_search("serial SN0041", 4)
    assert any(d.page_content.endswith("SN0041") for d, _ in hits)
