"""Closed-loop load generator (the reference specifies Locust but ships none:
experiment.yaml load_testing)."""
from .runner import LoadConfig, PhaseResult, run_level, run_sweep, summarize  # noqa: F401
