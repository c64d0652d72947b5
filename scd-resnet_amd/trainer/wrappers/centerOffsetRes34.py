"""Wrapper for centerOffsetRes34 (the reference ships one wrapper per architecture name, trace.py:62)."""
from trainer.wrappers.centerOffsetResidual import Wrapper  # noqa: F401
