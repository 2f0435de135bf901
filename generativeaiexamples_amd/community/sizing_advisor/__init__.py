"""MI355X sizing advisor on the RAG-Blueprint-2.x API (reference: /root/reference/community/vgpu-sizing-advisor):
``store`` (named HBM collections, background ingestion tasks), ``ingestor`` (documents / status / collections API),
``rag_server`` (streaming generate with citations and usage, search, structured deployment recommendations, GPU
detection, measured test runs and server launch via ``deploy``). The analytic planner is
``generativeaiexamples_amd.sizing``.

  python -m generativeaiexamples_amd.community.sizing_advisor.rag_server --port 8081 --ingestor-port 8082
"""
from .ingestor import create_ingestor_app  # noqa: F401
from .rag_server import BlueprintRag, create_rag_app  # noqa: F401
from .store import CollectionManager, TaskHandler  # noqa: F401
