"""query-decomposition agent (Search / Math tools)."""
from generativeaiexamples_amd.examples.query_decomposition import QueryDecompositionRAG  # noqa: F401
