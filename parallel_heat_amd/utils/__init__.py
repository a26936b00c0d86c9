"""I/O, timing and reporting utilities."""
from . import io, report

__all__ = ["io", "report"]
