"""``python -m generativeaiexamples_amd.chain_server --host 0.0.0.0 --port 8081`` (the reference image's
entrypoint runs uvicorn on RAG/src/chain_server/server.py with the same flags)."""
import argparse

import uvicorn


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8081)
    ap.add_argument("--workers", type=int, default=1)
    a = ap.parse_args()
    uvicorn.run("generativeaiexamples_amd.chain_server.server:app", host=a.host, port=a.port, workers=a.workers)


if __name__ == "__main__":
    main()
