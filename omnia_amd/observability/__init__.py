"""Metrics, tracing and logging."""
