"""multi-turn RAG with reranking and per-conversation memory."""
from generativeaiexamples_amd.examples.multi_turn import MultiTurnRAG  # noqa: F401
