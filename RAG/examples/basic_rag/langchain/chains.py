"""basic_rag (LangChain flavour) on the MI355X engines."""
from generativeaiexamples_amd.examples.basic_rag import BasicRAG  # noqa: F401
