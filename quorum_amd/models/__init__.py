"""Merge strategies ("model families" of the proxy): concatenate, aggregate, passthrough."""
from .strategies import aggregate_responses, build_aggregator_prompt, combine_finals  # noqa: F401
