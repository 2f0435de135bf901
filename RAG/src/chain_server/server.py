"""Drop-in entrypoint: ``uvicorn RAG.src.chain_server.server:app`` (reference Dockerfile ENTRYPOINT)."""
from generativeaiexamples_amd.chain_server.server import app  # noqa: F401
