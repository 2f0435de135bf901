"""CSV question answering with sandboxed pandas expressions."""
from generativeaiexamples_amd.examples.structured_data import StructuredDataRAG  # noqa: F401
