"""Event-driven CVE triage agent (reference: /root/reference/community/event-driven-rag-cve-analysis): ``checklist``
(CVE -> exploitability checklist), ``tools`` (SBOM lookup, PEP 440 / Debian version ranges, code search), ``agent``
(text-protocol ReAct loop), ``pipeline`` (concurrent per-CVE / per-item engine, ``POST /scan`` service)."""
from .agent import ReActAgent, parse_step  # noqa: F401
from .checklist import generate_checklist, parse_checklist  # noqa: F401
from .pipeline import CVEEngine, CVEResult, create_app  # noqa: F401
from .tools import CodeSearch, SBOMChecker, debian_compare, version_comparison  # noqa: F401
