"""Cross-cutting utilities: metrics, tracing, logging."""
