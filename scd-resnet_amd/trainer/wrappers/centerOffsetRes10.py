"""Wrapper for centerOffsetRes10 (the reference ships one wrapper per architecture name, trace.py:62)."""
from trainer.wrappers.centerOffsetResidual import Wrapper  # noqa: F401
