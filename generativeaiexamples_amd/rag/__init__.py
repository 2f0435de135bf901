"""RAG building blocks: prompts, text splitting, document loading, synthetic corpora."""
