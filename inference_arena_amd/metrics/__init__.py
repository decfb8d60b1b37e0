"""Prometheus metrics of the arena services."""
from .prom import ArenaMetrics

__all__ = ["ArenaMetrics"]
