"""basic_rag (LlamaIndex flavour) on the MI355X engines."""
from generativeaiexamples_amd.examples.basic_rag import LlamaIndexRAG  # noqa: F401
