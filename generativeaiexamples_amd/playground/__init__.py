"""RAG Playground: browser UI + Python client for the chain server."""
from .chat_client import ChatClient

__all__ = ["ChatClient", "create_app"]


def create_app(*a, **kw):
    from .app import create_app as _c
    return _c(*a, **kw)
