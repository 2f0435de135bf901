"""multimodal ingest (PDF / PPTX / images) + RAG."""
from generativeaiexamples_amd.examples.multimodal import MultimodalRAG  # noqa: F401
