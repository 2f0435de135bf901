"""Knowledge-graph RAG (reference: /root/reference/community/knowledge_graph_rag): ``graph`` (typed triple graph,
k-hop entity knowledge, GraphML / CSV), ``extract`` (LLM triple extraction, document ingest, QA-pair generation,
judge), ``rag`` (text / graph / combined answers), ``server`` (FastAPI backend of the reference's UI)."""
from .extract import extract_triples, parse_triples, process_documents  # noqa: F401
from .graph import KnowledgeGraph  # noqa: F401
from .rag import KGRag, parse_entities  # noqa: F401
