"""HTTP serving layer (FastAPI conformance app, upstream transport, tick scheduler)."""
