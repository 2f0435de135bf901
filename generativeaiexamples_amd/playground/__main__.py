"""``python -m generativeaiexamples_amd.playground --port 8090`` (reference: rag_playground/default/__main__.py)."""
import argparse

import uvicorn

from .app import create_app


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8090)
    ap.add_argument("--server-url", default=None, help="chain server URL (default: APP_SERVERURL:APP_SERVERPORT)")
    ap.add_argument("--model", default=None)
    a = ap.parse_args()
    uvicorn.run(create_app(a.server_url, a.model), host=a.host, port=a.port)


if __name__ == "__main__":
    main()
