"""Dataset curation: keep images whose detection count lies in a range.

Re-implements the reference's DatasetCurator (src/shared/data/curator.py:
CurationConfig :69-87, curate :480-599, _sample_balanced :601-678,
_generate_manifest :680-724) over any image source and any detection
counter (the GPU pipeline, or the fp32 reference).  Sampling weights are
1 / (1 + |d - mid|) per detection count, the remainder goes to the middle
bucket, and numpy's legacy seeded ``choice`` picks the members, as upstream.

The arena's default source is the synthetic COCO-shaped stream
(``synthetic.py``): image ``i`` of stream ``seed`` is regenerated from
``default_rng([seed, i])``, so a manifest of indices is enough to rebuild
the curated set bit-exactly without storing pixels.
"""
from __future__ import annotations

import json
import time
from dataclasses import asdict, dataclass, field
from datetime import datetime, timezone
from pathlib import Path
from typing import Callable, Iterable

import numpy as np

from .synthetic import synthetic_image

DEFAULT_TARGET_COUNT = 100
DEFAULT_MIN_DETECTIONS = 3
DEFAULT_MAX_DETECTIONS = 5


@dataclass
class CurationConfig:
    target_count: int = DEFAULT_TARGET_COUNT
    min_detections: int = DEFAULT_MIN_DETECTIONS
    max_detections: int = DEFAULT_MAX_DETECTIONS
    confidence_threshold: float = 0.5
    iou_threshold: float = 0.45
    random_seed: int = 42


@dataclass
class ImageRecord:
    filename: str
    detection_count: int
    original_path: str | None = None


@dataclass
class CurationResult:
    images: list[ImageRecord] = field(default_factory=list)
    total_scanned: int = 0
    total_selected: int = 0
    skipped_low: int = 0
    skipped_high: int = 0
    errors: int = 0


@dataclass
class DatasetManifest:
    version: str = "1.0"
    created: str = ""
    source: str = "synthetic"
    config: dict = field(default_factory=dict)
    statistics: dict = field(default_factory=dict)
    distribution: dict = field(default_factory=dict)
    images: list[dict] = field(default_factory=list)

    def to_dict(self) -> dict:
        return asdict(self)

    def save(self, path: Path) -> None:
        Path(path).parent.mkdir(parents=True, exist_ok=True)
        with open(path, "w", encoding="utf-8") as f:
            json.dump(self.to_dict(), f, indent=2)

    @classmethod
    def load(cls, path: Path) -> "DatasetManifest":
        with open(path, encoding="utf-8") as f:
            return cls(**json.load(f))


def sampling_targets(cfg: CurationConfig) -> dict[int, int]:
    rng_d = list(range(cfg.min_detections, cfg.max_detections + 1))
    mid = (cfg.min_detections + cfg.max_detections) / 2
    w = [1.0 / (1.0 + abs(d - mid)) for d in rng_d]
    tw = sum(w)
    targets = {d: int(cfg.target_count * wi / tw) for d, wi in zip(rng_d, w)}
    short = cfg.target_count - sum(targets.values())
    if short > 0:
        targets[rng_d[len(rng_d) // 2]] += short
    return targets


def sample_balanced(candidates: dict[int, list[ImageRecord]], cfg: CurationConfig) -> list[ImageRecord]:
    np.random.seed(cfg.random_seed)
    selected: list[ImageRecord] = []
    for d, target in sampling_targets(cfg).items():
        avail = candidates.get(d, [])
        if not avail:
            continue
        k = min(target, len(avail))
        idx = np.random.choice(len(avail), size=k, replace=False)
        selected.extend(avail[i] for i in idx)
    if len(selected) < cfg.target_count:
        taken = {r.filename for r in selected}
        for d in range(cfg.min_detections, cfg.max_detections + 1):
            for r in candidates.get(d, []):
                if len(selected) >= cfg.target_count:
                    break
                if r.filename not in taken:
                    selected.append(r)
                    taken.add(r.filename)
    return selected[: cfg.target_count]


def make_manifest(result: CurationResult, cfg: CurationConfig, source: str, extra: dict | None = None) -> DatasetManifest:
    counts = [r.detection_count for r in result.images]
    if counts:
        mean = sum(counts) / len(counts)
        std = (sum((c - mean) ** 2 for c in counts) / len(counts)) ** 0.5
        lo, hi = min(counts), max(counts)
    else:
        mean = std = lo = hi = 0
    dist: dict[int, int] = {}
    for c in counts:
        dist[c] = dist.get(c, 0) + 1
    conf = asdict(cfg)
    conf.update(extra or {})
    return DatasetManifest(
        version="1.0",
        created=datetime.now(timezone.utc).isoformat(),
        source=source,
        config=conf,
        statistics={"total_images": len(counts), "mean_detections": round(mean, 2),
                    "std_detections": round(std, 2), "min_detections": lo, "max_detections": hi,
                    "total_scanned": result.total_scanned, "skipped_low": result.skipped_low,
                    "skipped_high": result.skipped_high},
        distribution={str(k): v for k, v in sorted(dist.items())},
        images=[{"filename": r.filename, "detections": r.detection_count} for r in result.images],
    )


def stream_image(seed: int, index: int) -> np.ndarray:
    return synthetic_image(np.random.default_rng([int(seed), int(index)]))


def curate(counter: Callable[[list[np.ndarray]], Iterable[int]], cfg: CurationConfig | None = None, *,
           stream_seed: int = 7, batch: int = 32, max_scan: int = 20000, log: Callable[[str], None] | None = None
           ) -> tuple[CurationResult, DatasetManifest]:
    """Scan the synthetic stream until every detection-count bucket can meet its target."""
    cfg = cfg or CurationConfig()
    targets = sampling_targets(cfg)
    cands: dict[int, list[ImageRecord]] = {d: [] for d in targets}
    res = CurationResult()
    t0 = time.time()
    i = 0
    while i < max_scan and any(len(cands[d]) < t for d, t in targets.items()):
        imgs = [stream_image(stream_seed, i + k) for k in range(batch)]
        for k, c in enumerate(counter(imgs)):
            res.total_scanned += 1
            c = int(c)
            if c < cfg.min_detections:
                res.skipped_low += 1
            elif c > cfg.max_detections:
                res.skipped_high += 1
            else:
                cands[c].append(ImageRecord(f"synthetic_{stream_seed}_{i + k:06d}", c))
        i += batch
        if log and (i // batch) % 20 == 0:
            log(f"curate: scanned {i}, candidates {({d: len(v) for d, v in cands.items()})}, {time.time() - t0:.1f}s")
    sel = sample_balanced(cands, cfg)
    res.images = sel
    res.total_selected = len(sel)
    man = make_manifest(res, cfg, source=f"synthetic stream seed={stream_seed}", extra={"stream_seed": stream_seed})
    return res, man


def curate_paths(counter: Callable[[list[np.ndarray]], Iterable[int]], paths, cfg: CurationConfig | None = None, *,
                 loader: Callable | None = None, batch: int = 32, log: Callable[[str], None] | None = None
                 ) -> tuple[CurationResult, DatasetManifest]:
    """Curate a local image collection (COCO val2017, reference src/shared/data/curator.py:480-599): count
    the detections of every file, keep those with min..max detections, sample the 25/50/25 mix."""
    from ..processing.transforms import load_image

    cfg = cfg or CurationConfig()
    loader = loader or load_image
    targets = sampling_targets(cfg)
    cands: dict[int, list[ImageRecord]] = {d: [] for d in targets}
    res = CurationResult()
    t0 = time.time()
    paths = list(paths)
    for s in range(0, len(paths), batch):
        chunk = paths[s: s + batch]
        for p, c in zip(chunk, counter([loader(p) for p in chunk])):
            res.total_scanned += 1
            c = int(c)
            if c < cfg.min_detections:
                res.skipped_low += 1
            elif c > cfg.max_detections:
                res.skipped_high += 1
            else:
                cands[c].append(ImageRecord(str(p), c))
        if log and (s // batch) % 20 == 0:
            log(f"curate: scanned {res.total_scanned}/{len(paths)}, {time.time() - t0:.1f}s")
    res.images = sample_balanced(cands, cfg)
    res.total_selected = len(res.images)
    return res, make_manifest(res, cfg, source="local image collection")


def load_manifest_images(man: DatasetManifest) -> list[np.ndarray]:
    seed = int(man.config.get("stream_seed", 7))
    return [stream_image(seed, int(r["filename"].rsplit("_", 1)[1])) for r in man.images]


def workload_images(n: int | None = None, weight_seed: int = 0, n_images: int = 100) -> list[np.ndarray]:
    """Images of the committed curated workload (``data/synthetic_set/manifest_w<seed>_n<N>.json``)."""
    root = Path(__file__).resolve().parents[2] / "data" / "synthetic_set"
    man = DatasetManifest.load(root / f"manifest_w{weight_seed}_n{n_images}.json")
    if n is not None:
        man.images = man.images[:n]
    return load_manifest_images(man)


class DetectionCounter:
    """Count detections in a raw detector output, accepting the three layouts the
    reference's counter understands (src/shared/data/curator.py:226-321):

    * YOLOv8/v5u head ``[1, 84, N]`` (or ``[84, N]``): 4 box + 80 class scores;
    * classic YOLOv5 ``[1, N, 85]``: 4 box + objectness + 80 class scores
      (confidence = objectness x class score);
    * post-NMS ``[1, N, 6]`` / ``[N, 6]``: x1, y1, x2, y2, conf, cls.

    Raw layouts go through the reference's class-aware NMS (``postprocess``).
    """

    def __init__(self, confidence_threshold: float = 0.5, iou_threshold: float = 0.45):
        self.conf = confidence_threshold
        self.iou = iou_threshold

    def count(self, output: np.ndarray) -> int:
        a = np.asarray(output, dtype=np.float32)
        if a.ndim == 3:
            a = a[0]
        if a.ndim != 2:
            raise ValueError(f"unsupported detector output shape {np.shape(output)}")
        if a.shape[1] == 6 and a.shape[0] != 84:
            return int((a[:, 4] >= self.conf).sum())
        if a.shape[0] == 84:
            return self._raw(a[:4].T, a[4:].T)
        if a.shape[1] == 85:
            return self._raw(a[:, :4], a[:, 5:] * a[:, 4:5])
        if a.shape[1] == 84:
            return self._raw(a[:, :4], a[:, 4:])
        raise ValueError(f"unsupported detector output shape {np.shape(output)}")

    def _raw(self, xywh: np.ndarray, cls_scores: np.ndarray) -> int:
        from ..postprocess import apply_nms

        conf = cls_scores.max(axis=1)
        cls = cls_scores.argmax(axis=1)
        return len(apply_nms(xywh, conf, cls, self.conf, self.iou))
