"""Retrieval-augmented text-to-SQL (reference: /root/reference/community/Vanna_with_NVIDIA_AI_Endpoints,
SQLServer_AI_with_NVIDIA_NIM): train on DDL / documentation / question-SQL pairs in an HBM collection, generate SQL from
the retrieved context, run it on a read-only sqlite connection with one self-correction round."""
from .agent import SqlAgent, extract_sql  # noqa: F401
