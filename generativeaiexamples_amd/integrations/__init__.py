"""Adapters that let third-party agent frameworks call this framework's LLMs."""
