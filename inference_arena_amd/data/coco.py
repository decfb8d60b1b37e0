"""COCO val2017 utilities (reference: src/shared/data/coco_dataset.py:105-314).

The arena runs without network access, so ``download_coco_val2017`` only
extracts a locally provided ``val2017.zip`` (the reference downloads it);
everything else — presence check, image listing, loading and iteration —
works on an existing ``<data_dir>/val2017`` directory.  When no COCO images
exist, the synthetic COCO-shaped stream (``synthetic.py``) is the source.
"""
from __future__ import annotations

import zipfile
from pathlib import Path
from typing import Iterator

import numpy as np

COCO_VAL_IMAGES = 5000
COCO_VAL_DIR = "val2017"


def is_coco_downloaded(data_dir: str | Path) -> tuple[bool, str]:
    d = Path(data_dir) / COCO_VAL_DIR
    if not d.is_dir():
        return False, f"{d} does not exist"
    n = sum(1 for _ in d.glob("*.jpg"))
    if n < COCO_VAL_IMAGES:
        return False, f"{d} has {n} of {COCO_VAL_IMAGES} images"
    return True, f"{d} has {n} images"


def download_coco_val2017(data_dir: str | Path, archive: str | Path | None = None, force: bool = False) -> Path:
    """Extract ``archive`` (default ``<data_dir>/val2017.zip``) into ``<data_dir>``; idempotent."""
    data_dir = Path(data_dir)
    ok, _ = is_coco_downloaded(data_dir)
    if ok and not force:
        return data_dir / COCO_VAL_DIR
    archive = Path(archive) if archive else data_dir / "val2017.zip"
    if not archive.exists():
        raise FileNotFoundError(
            f"{archive} not found: this environment has no network access; place the COCO val2017 archive "
            "there, or use the synthetic COCO-shaped stream (inference_arena_amd.data.synthetic)")
    data_dir.mkdir(parents=True, exist_ok=True)
    with zipfile.ZipFile(archive) as z:
        z.extractall(data_dir)
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
