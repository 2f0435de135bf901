"""Example pipelines (BaseExample implementations) - the reference's RAG/examples/* chains."""
