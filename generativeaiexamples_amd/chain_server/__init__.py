"""Chain server: REST API (/health /documents /generate /search), config wizard, factories, tracing."""
