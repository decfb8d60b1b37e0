"""Minimal multipart/form-data parser for ``POST /predict``.

FastAPI's ``UploadFile = File(...)`` needs the python-multipart package,
which is not installed here; the endpoints read the raw body and extract
the ``file`` field with this parser (RFC 7578 subset: boundary-delimited
parts with Content-Disposition headers; no nested multipart).
"""
from __future__ import annotations

import re

_BOUNDARY = re.compile(r'boundary="?([^";]+)"?', re.I)
_NAME = re.compile(rb'\bname="([^"]*)"', re.I)
_FILENAME = re.compile(rb'\bfilename="([^"]*)"', re.I)


class MultipartError(ValueError):
    pass


def parse_multipart(body: bytes, content_type: str) -> dict[str, tuple[bytes, str | None]]:
    """Return {field name: (payload bytes, filename or None)}."""
    m = _BOUNDARY.search(content_type or "")
    if not m or not content_type.lower().startswith("multipart/form-data"):
        raise MultipartError("Content-Type must be multipart/form-data with a boundary")
    delim = b"--" + m.group(1).encode("latin-1")
    parts = body.split(delim)
    if len(parts) < 3:
        raise MultipartError("no multipart parts found")
    out: dict[str, tuple[bytes, str | None]] = {}
    for part in parts[1:]:
        if part.startswith(b"--"):
            break
        if part.startswith(b"\r\n"):
            part = part[2:]
        head, sep, payload = part.partition(b"\r\n\r\n")
        if not sep:
            raise MultipartError("malformed part (no header terminator)")
        if payload.endswith(b"\r\n"):
            payload = payload[:-2]
        disp = None
        for line in head.split(b"\r\n"):
            if line.lower().startswith(b"content-disposition:"):
                disp = line
        if disp is None:
            continue
        nm = _NAME.search(disp)
        if not nm:
            continue
        fn = _FILENAME.search(disp)
        out[nm.group(1).decode("utf-8", "replace")] = (payload, fn.group(1).decode("utf-8", "replace") if fn else None)
    return out


def encode_multipart(field: str, data: bytes, filename: str = "image.jpg",
                     content_type: str = "image/jpeg", boundary: str = "arena-boundary-7d1f") -> tuple[bytes, str]:
    """Build a multipart body (used by the load generator and tests)."""
    head = (f"--{boundary}\r\nContent-Disposition: form-data; name=\"{field}\"; filename=\"{filename}\"\r\n"
            f"Content-Type: {content_type}\r\n\r\n").encode()
    body = head + data + f"\r\n--{boundary}--\r\n".encode()
    return body, f"multipart/form-data; boundary={boundary}"
