"""Chain-server API client (the reference's RAG_Chain_Server_API_Client notebook uploads a
folder of PDFs and streams /generate, printing tokens/s - its counter was never incremented, §7.7).

    python RAG/src/chain_server/api_client.py --url http://localhost:8081 --docs ./pdfs \\
        --question "What is the MI355X memory size?"
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", "..")))
from generativeaiexamples_amd.playground.chat_client import ChatClient  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--url", default="http://localhost:8081")
    ap.add_argument("--docs", default=None, help="folder of documents to upload first")
    ap.add_argument("--question", default="Summarise the uploaded documents.")
    ap.add_argument("--max-tokens", type=int, default=256)
    ap.add_argument("--no-kb", action="store_true")
    a = ap.parse_args()
    c = ChatClient(a.url)
    if a.docs:
        files = [os.path.join(a.docs, f) for f in sorted(os.listdir(a.docs)) if os.path.isfile(os.path.join(a.docs, f))]
        t0 = time.perf_counter()
        c.upload_documents(files)
        print(f"uploaded {len(files)} files in {time.perf_counter() - t0:.1f}s; server has {len(c.get_uploaded_documents())}")
    t0 = time.perf_counter()
    first, chunks = None, 0
    for piece in c.predict(a.question, not a.no_kb, a.max_tokens):
        if first is None:
            first = time.perf_counter() - t0
        chunks += 1
        print(piece, end="", flush=True)
    dt = time.perf_counter() - t0
    print(f"\n\nTTFT {first or dt:.3f}s, {chunks} streamed chunks in {dt:.2f}s = {chunks / dt:.1f} chunks/s")


if __name__ == "__main__":
    main()
