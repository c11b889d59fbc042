"""Utilities: storage, config, tracing, logging."""
from .storage import Storage

__all__ = ["Storage"]
