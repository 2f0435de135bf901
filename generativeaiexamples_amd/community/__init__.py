"""Community projects of the reference re-built on this framework (README.md here lists how to run them):
``fm_asr`` (FM-radio streaming RAG: SDR signal chain on HIP kernels, transcript accumulator, time-aware retrieval, chain
server), ``dfp`` (digital-fingerprinting autoencoder), ``kg_rag`` (knowledge-graph RAG), ``cve_agent`` (event-driven
CVE triage), ``sizing_advisor`` (RAG Blueprint 2.x API with MI355X sizing), ``agentic_rag`` (self-corrective and
routed RAG flows), ``text_to_sql`` (retrieval-augmented SQL generation) and ``data_analysis`` (pandas analysis
agent)."""
