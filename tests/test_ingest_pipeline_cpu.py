"""Stage-pipelined streaming ingest (P6): files + documents flow through load/split -> embed -> write
concurrently; every chunk lands in the store once, bad inputs are reported, not fatal."""
import torch

from generativeaiexamples_amd.chain_server.connectors import Embeddings
from generativeaiexamples_amd.chain_server.vectorstore import VectorStore
from generativeaiexamples_amd.index.hbm_index import Document
from generativeaiexamples_amd.rag.ingest_pipeline import IngestPipeline, directory_source, jsonl_source
from generativeaiexamples_amd.rag.text_splitter import RecursiveCharacterTextSplitter


class _Emb(Embeddings):
    dim = 32

    def __init__(self):
        self.calls = 0

    def embed_tensor(self, texts, input_type):
        self.calls += 1
        g = torch.Generator().manual_seed(len(texts))
        return torch.nn.functional.normalize(torch.randn(len(texts), self.dim, generator=g), dim=-1)


def test_pipeline_ingests_directory_and_stream(tmp_path):
    d = tmp_path / "docs"
    d.mkdir()
    for i in range(12):
        (d / f"doc{i}.txt").write_text(f"Document {i}. " + "Paragraph text about MI355X accelerators. " * 40)
    js = tmp_path / "stream.jsonl"
    js.write_text("\n".join('{"text": "streamed record %d about HBM3E", "filename": "s.jsonl"}' % i for i in range(50)))
    store = VectorStore("ingest", _Emb(), device="cpu", hybrid=True)
    pipe = IngestPipeline(store, RecursiveCharacterTextSplitter(chunk_size=300, chunk_overlap=30), embed_batch=16,
                          write_batch=40)
    pipe.start()
    for p in directory_source(str(d)):
        pipe.submit(p)
    for doc in jsonl_source(str(js)):
        pipe.submit(doc)
    pipe.submit(str(tmp_path / "missing.txt"))  # unreadable input: reported, stream continues
    stats = pipe.close()
    n_chunks = stats.load.items
    assert n_chunks == len(store) == stats.write.items and n_chunks > 60
    assert stats.docs == 12 + 50 and len(stats.errors) == 1  # the missing file
    assert store.emb.calls == (n_chunks + 15) // 16
    assert "doc3.txt" in store.filenames() and len(store.bm25) == n_chunks
    r = pipe.rates()
    assert r["chunks_per_s"] > 0 and r["embeddings_per_s"] > 0 and r["rows_written_per_s"] > 0
    assert store.hybrid_search("streamed record 7", 3)
