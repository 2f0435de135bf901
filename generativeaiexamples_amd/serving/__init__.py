"""HTTP serving: NIM/OpenAI-compatible /v1 API, async engine front-end, model hub."""
