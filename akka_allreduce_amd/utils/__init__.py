"""Utilities: logging, metrics, tracing."""
