"""Classifier label names.

The reference ships the 1000 ImageNet class names
(src/shared/data/imagenet_labels.txt) and refuses to start unless exactly
1000 lines load (architectures/monolithic/app/inference.py:96-125).  The same
constant table ships here (``inference_arena_amd/data/imagenet_labels.txt``,
the standard ImageNet-1k class names) and is the default; ``LABELS_FILE`` (or
a model repository's ``labels.txt``) overrides it.  ``placeholder_labels``
remains for tests that want synthetic names.
"""
from __future__ import annotations

from pathlib import Path

NUM_CLASSES = 1000


def placeholder_labels(n: int = NUM_CLASSES) -> list[str]:
    return [f"imagenet_class_{i:03d}" for i in range(n)]


DEFAULT_LABELS = Path(__file__).resolve().parent / "data" / "imagenet_labels.txt"


def load_labels(path: str | Path | None = None, n: int = NUM_CLASSES) -> list[str]:
    """The configured label file, else the shipped ImageNet table; exactly ``n`` names (reference check)."""
    p = Path(path) if path else DEFAULT_LABELS
    if not p.exists():
        raise FileNotFoundError(f"labels file not found: {p}")
    labels = [ln.strip() for ln in p.read_text(encoding="utf-8").splitlines()]
    while labels and labels[-1] == "":
        labels.pop()
    if len(labels) != n:
        raise ValueError(f"Expected {n} labels, got {len(labels)} in {p}")
    return labels
