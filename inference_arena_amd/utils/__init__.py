"""Shared utilities: structured logging, settings, timing."""
