"""Structured JSON logging with a per-request context id.

Same record shape as the reference's service loggers
(architectures/monolithic/app/logger.py:17-88): timestamp, level, logger,
message, the request id from a ContextVar, a whitelist of extra fields and
the formatted exception.  The classification-service variant's extra fields
(class_name, confidence; architectures/microservices/classification/app/
logger.py:53-54) and the arena's batching fields are included.
"""
from __future__ import annotations

import json
import logging
import sys
from contextvars import ContextVar
from typing import Any

request_id_var: ContextVar[str | None] = ContextVar("request_id", default=None)

EXTRA_FIELDS = ("endpoint", "latency_ms", "status_code", "detections", "port", "class_name", "confidence",
                "batch_size", "queue_ms", "gpu", "replica", "model", "error")


class JSONFormatter(logging.Formatter):
    def format(self, record: logging.LogRecord) -> str:
        data: dict[str, Any] = {
            "timestamp": self.formatTime(record, self.datefmt),
            "level": record.levelname,
            "logger": record.name,
            "message": record.getMessage(),
        }
        rid = request_id_var.get()
        if rid:
            data["request_id"] = rid
        for key in EXTRA_FIELDS:
            if hasattr(record, key):
                data[key] = getattr(record, key)
        if record.exc_info:
            data["exception"] = self.formatException(record.exc_info)
        return json.dumps(data, default=str)


def setup_logging(log_level: str = "INFO", stream=None) -> None:
    handler = logging.StreamHandler(stream or sys.stdout)
    handler.setFormatter(JSONFormatter())
    root = logging.getLogger()
    root.setLevel(getattr(logging, str(log_level).upper(), logging.INFO))
    root.handlers.clear()
    root.addHandler(handler)
