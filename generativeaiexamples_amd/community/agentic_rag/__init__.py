"""Agentic RAG flows of the community projects: ``graph`` (a bounded state-graph runner, the LangGraph role),
``corrective`` (self-corrective log-analysis RAG: hybrid retrieval, rerank, concurrent document grading, query
rewriting, grounded / useful answer grading), ``routing`` (routed multi-source RAG with concurrent sources and a
token-budgeted context)."""
from .corrective import CorrectiveRag, HybridLogRetriever  # noqa: F401
from .graph import END, START, GraphRecursionError, StateGraph  # noqa: F401
from .routing import RoutedRag, llm_source, parse_route, vector_source  # noqa: F401
