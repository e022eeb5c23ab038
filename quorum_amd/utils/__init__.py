"""Config, metrics, logging and tracing utilities."""
