"""Classifier label names.

The reference ships the 1000 ImageNet class names
(src/shared/data/imagenet_labels.txt) and refuses to start unless exactly
1000 lines load (architectures/monolithic/app/inference.py:96-125).  The arena
uses random-init weights, so the label *names* carry no meaning; it loads a
real 1000-line label file when one is configured (``LABELS_FILE`` or the
model repository's ``labels.txt``) and otherwise generates stable
placeholder names ``imagenet_class_XXX``.
"""
from __future__ import annotations

from pathlib import Path

NUM_CLASSES = 1000


def placeholder_labels(n: int = NUM_CLASSES) -> list[str]:
    return [f"imagenet_class_{i:03d}" for i in range(n)]


def load_labels(path: str | Path | None = None, n: int = NUM_CLASSES) -> list[str]:
    if not path:
        return placeholder_labels(n)
    p = Path(path)
    if not p.exists():
        raise FileNotFoundError(f"labels file not found: {p}")
    labels = [ln.strip() for ln in p.read_text(encoding="utf-8").splitlines()]
    while labels and labels[-1] == "":
        labels.pop()
    if len(labels) != n:
        raise ValueError(f"Expected {n} labels, got {len(labels)} in {p}")
    return labels
