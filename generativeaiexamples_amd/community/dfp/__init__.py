"""Digital-fingerprinting (DFP) per-user tabular autoencoder (reference: community/digital-human-security-analyst)."""
from .autoencoder import AEConfig, TabularAutoEncoder, train_per_user  # noqa: F401
