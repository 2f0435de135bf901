"""Agent examples consuming the /v1 tool-calling API (SURVEY W11 bash agent, W12 thinking toggle)."""
