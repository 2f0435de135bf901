"""Exact HBM-resident vector index (fused similarity + top-k kernel), DP sharding, persistence."""
from .hbm_index import Document, HBMIndex, SearchHit  # noqa: F401
