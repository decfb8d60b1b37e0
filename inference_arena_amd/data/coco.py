"""COCO val2017 utilities (reference: src/shared/data/coco_dataset.py:34-314).

``download_coco_val2017`` fetches ``val2017.zip`` over HTTP(S) (or any urllib URL, e.g. ``file://`` or a local
mirror) with a progress callback, resumes a partial ``.part`` file with a Range request when the server allows
it, and extracts it; it is idempotent like the reference's (coco_dataset.py:141-217).  A locally provided archive
is extracted without any network access.  Everything else — presence check, image listing, loading and
iteration — works on an existing ``<data_dir>/val2017`` directory.  When no COCO images exist (this environment
has no network), the synthetic COCO-shaped stream (``synthetic.py``) is the source.
"""
from __future__ import annotations

import logging
import os
import sys
import urllib.request
import zipfile
from pathlib import Path
from typing import Callable, Iterator

import numpy as np

COCO_VAL_IMAGES = 5000
COCO_VAL_DIR = "val2017"
COCO_VAL2017_URL = "http://images.cocodataset.org/zips/val2017.zip"
COCO_ZIP_BYTES = 815_585_330  # approximate size of val2017.zip (~778 MiB), for progress without Content-Length

log = logging.getLogger(__name__)

ProgressFn = Callable[[int, int], None]  # (bytes so far, total bytes or -1)


class DownloadProgress:
    """Console progress for ``fetch_url`` (reference DownloadProgressBar, coco_dataset.py:49-97): a 40-cell
    bar with percent and MiB, redrawn only when the percentage changes."""

    def __init__(self, expected_bytes: int = COCO_ZIP_BYTES, stream=None) -> None:
        self.expected = expected_bytes
        self.stream = stream or sys.stderr
        self.last = -1

    def __call__(self, done: int, total: int) -> None:
        tot = total if total > 0 else self.expected
        pct = min(100 if total > 0 else 99, int(100 * done / max(1, tot)))
        if pct == self.last:
            return
        self.last = pct
        fill = 40 * pct // 100
        self.stream.write(f"\r  [{'#' * fill}{'.' * (40 - fill)}] {pct}% - {done / 2**20:.1f} / {tot / 2**20:.1f} MiB")
        self.stream.flush()


def fetch_url(url: str, dest: str | Path, progress: ProgressFn | None = None, chunk: int = 1 << 20,
              timeout: float = 60.0) -> Path:
    """Stream ``url`` to ``dest``.  Bytes land in ``dest.part`` first; a ``.part`` left by an interrupted run is
    resumed with ``Range: bytes=<size>-`` when the server answers 206 (restarted from zero on 200).  ``dest``
    appears only once complete, so a crash never leaves a truncated archive behind."""
    dest = Path(dest)
    dest.parent.mkdir(parents=True, exist_ok=True)
    part = dest.with_name(dest.name + ".part")
    have = part.stat().st_size if part.exists() else 0
    req = urllib.request.Request(url)
    if have and url.startswith(("http://", "https://")):
        req.add_header("Range", f"bytes={have}-")
    try:
        resp = urllib.request.urlopen(req, timeout=timeout)  # noqa: S310 - caller-chosen dataset URL
    except Exception as e:  # noqa: BLE001
        raise RuntimeError(f"Download failed: {e}") from e
    with resp:
        status = getattr(resp, "status", 200)
        length = int(resp.headers.get("Content-Length") or -1)
        if status == 206:
            total = have + length if length >= 0 else -1
            mode = "ab"
        else:
            have, total, mode = 0, length, "wb"
        done = have
        with open(part, mode) as f:
            while True:
                buf = resp.read(chunk)
                if not buf:
                    break
                f.write(buf)
                done += len(buf)
                if progress:
                    progress(done, total)
    if total >= 0 and done != total:
        raise RuntimeError(f"Download failed: got {done} of {total} bytes from {url}")
    os.replace(part, dest)
    return dest


def is_coco_downloaded(data_dir: str | Path, expected: int = COCO_VAL_IMAGES) -> tuple[bool, str]:
    d = Path(data_dir) / COCO_VAL_DIR
    if not d.is_dir():
        return False, f"{d} does not exist"
    n = sum(1 for _ in d.glob("*.jpg"))
    if n < expected:
        return False, f"{d} has {n} of {expected} images"
    return True, f"{d} has {n} images"


def download_coco_val2017(data_dir: str | Path, archive: str | Path | None = None, force: bool = False,
                          url: str | None = COCO_VAL2017_URL, progress: ProgressFn | None = None,
                          cleanup_zip: bool = True, expected_images: int = COCO_VAL_IMAGES) -> Path:
    """Make ``<data_dir>/val2017`` hold the COCO val2017 images; idempotent (reference coco_dataset.py:141-217).

    1. already complete (``is_coco_downloaded``) and not ``force``: nothing to do;
    2. ``archive`` (default ``<data_dir>/val2017.zip``) exists: extract it, no network;
    3. otherwise fetch ``url`` into that archive (``fetch_url``: progress, resumable ``.part``) and extract.
    ``url=None`` forbids the network step.  ``expected_images`` is the completeness check after extraction
    (5000 for the real archive; tests pass a small mirror).  A downloaded archive is removed after a successful
    extraction when ``cleanup_zip``; a caller-provided one is kept."""
    data_dir = Path(data_dir)
    ok, _ = is_coco_downloaded(data_dir, expected_images)
    if ok and not force:
        return data_dir / COCO_VAL_DIR
    provided = archive is not None
    archive = Path(archive) if archive else data_dir / "val2017.zip"
    fetched = False
    if not archive.exists():
        if url is None:
            raise FileNotFoundError(
                f"{archive} not found and downloads are disabled: place the COCO val2017 archive there, or use the "
                "synthetic COCO-shaped stream (inference_arena_amd.data.synthetic)")
        log.info("downloading COCO val2017 from %s to %s", url, archive)
        fetch_url(url, archive, progress=progress if progress is not None else DownloadProgress())
        fetched = True
    data_dir.mkdir(parents=True, exist_ok=True)
    try:
        with zipfile.ZipFile(archive) as z:
            z.extractall(data_dir)
    except (zipfile.BadZipFile, OSError) as e:
        raise RuntimeError(f"Extraction failed: {e}") from e
    ok, msg = is_coco_downloaded(data_dir, expected_images)
    if not ok:
        raise RuntimeError(f"Extraction incomplete: {msg}")
    if cleanup_zip and fetched and not provided:
        archive.unlink(missing_ok=True)
    return data_dir / COCO_VAL_DIR


def load_coco_image(image_path: str | Path) -> np.ndarray:
    from ..processing import load_image

    return load_image(str(image_path))


def get_coco_image_paths(data_dir: str | Path) -> list[Path]:
    return sorted((Path(data_dir) / COCO_VAL_DIR).glob("*.jpg"))


def iter_coco_images(data_dir: str | Path, limit: int | None = None) -> Iterator[tuple[Path, np.ndarray]]:
    for i, p in enumerate(get_coco_image_paths(data_dir)):
        if limit is not None and i >= limit:
            return
        yield p, load_coco_image(p)
