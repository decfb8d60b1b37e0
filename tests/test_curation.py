"""Dataset curation semantics (reference: src/shared/data/curator.py —
CurationConfig :69-87, _sample_balanced :601-678, _generate_manifest
:680-724; tests/shared/test_data.py) and the synthetic workload it feeds."""
from __future__ import annotations

import json

import numpy as np
import pytest

from inference_arena_amd.data.curator import (
    CurationConfig,
    CurationResult,
    DatasetManifest,
    ImageRecord,
    curate,
    load_manifest_images,
    make_manifest,
    sample_balanced,
    sampling_targets,
    stream_image,
    workload_images,
)
from inference_arena_amd.data.synthetic import encode_png, synthetic_image, synthetic_images
from inference_arena_amd.processing import load_image_from_bytes


def test_sampling_targets_reference_split():
    # weights 1/(1+|d-4|) for d = 3, 4, 5 -> 0.5 : 1 : 0.5 -> 25 / 50 / 25 (thesis_test_set/manifest.json:12-23)
    assert sampling_targets(CurationConfig()) == {3: 25, 4: 50, 5: 25}


@pytest.mark.parametrize("n", [1, 7, 10, 99, 101, 1000])
def test_sampling_targets_sum_to_target(n):
    t = sampling_targets(CurationConfig(target_count=n))
    assert sum(t.values()) == n
    assert t[4] >= t[3] == t[5]


def test_sampling_targets_other_ranges():
    t = sampling_targets(CurationConfig(target_count=60, min_detections=1, max_detections=4))
    assert sum(t.values()) == 60 and set(t) == {1, 2, 3, 4}
    assert t[1] == t[4] and min(t[2], t[3]) > t[1]  # the rounding remainder goes to the middle bucket


def _cands(per_bucket: dict[int, int]):
    return {d: [ImageRecord(f"img_{d}_{i}", d) for i in range(n)] for d, n in per_bucket.items()}


def test_sample_balanced_hits_targets_and_is_seeded():
    cands = _cands({3: 80, 4: 120, 5: 60})
    a = sample_balanced(cands, CurationConfig())
    b = sample_balanced(cands, CurationConfig())
    c = sample_balanced(cands, CurationConfig(random_seed=7))
    assert [r.filename for r in a] == [r.filename for r in b]
    assert [r.filename for r in a] != [r.filename for r in c]
    counts = {d: sum(1 for r in a if r.detection_count == d) for d in (3, 4, 5)}
    assert counts == {3: 25, 4: 50, 5: 25}
    assert len({r.filename for r in a}) == 100


def test_sample_balanced_backfills_short_buckets():
    cands = _cands({3: 5, 4: 200, 5: 10})
    sel = sample_balanced(cands, CurationConfig())
    assert len(sel) == 100 and len({r.filename for r in sel}) == 100
    assert sum(1 for r in sel if r.detection_count == 3) == 5


def test_sample_balanced_with_too_few_candidates():
    sel = sample_balanced(_cands({3: 2, 4: 3, 5: 1}), CurationConfig())
    assert len(sel) == 6


def test_manifest_schema_and_statistics(tmp_path):
    res = CurationResult(images=[ImageRecord("a", 3), ImageRecord("b", 4), ImageRecord("c", 4), ImageRecord("d", 5)],
                         total_scanned=10, skipped_low=4, skipped_high=2)
    man = make_manifest(res, CurationConfig(), source="unit")
    d = man.to_dict()
    assert set(d) == {"version", "created", "source", "config", "statistics", "distribution", "images"}
    assert d["statistics"]["total_images"] == 4 and d["statistics"]["mean_detections"] == 4.0
    assert d["statistics"]["std_detections"] == pytest.approx(0.71, abs=0.01)
    assert d["distribution"] == {"3": 1, "4": 2, "5": 1}
    assert d["images"][0] == {"filename": "a", "detections": 3}
    assert d["config"]["random_seed"] == 42 and d["config"]["iou_threshold"] == 0.45
    p = tmp_path / "m" / "manifest.json"
    man.save(p)
    assert json.loads(p.read_text())["source"] == "unit"
    assert DatasetManifest.load(p) == man


def test_empty_manifest():
    man = make_manifest(CurationResult(), CurationConfig(), source="none")
    assert man.statistics["total_images"] == 0 and man.distribution == {} and man.images == []


def test_curate_with_a_deterministic_counter():
    def counter(imgs):  # detection count from the pixel content (stable per image)
        return [int(im[::97, ::89].sum()) % 7 for im in imgs]

    res, man = curate(counter, CurationConfig(target_count=20), batch=16, max_scan=2000)
    assert len(res.images) == 20
    assert all(3 <= r.detection_count <= 5 for r in res.images)
    assert man.distribution == {"3": 5, "4": 10, "5": 5}
    assert res.total_scanned >= 20 and res.skipped_low + res.skipped_high > 0
    # the manifest alone regenerates the exact images
    imgs = load_manifest_images(man)
    assert [counter([im])[0] for im in imgs] == [r["detections"] for r in man.images]


def test_stream_images_are_reproducible():
    a, b = stream_image(7, 123), stream_image(7, 123)
    assert np.array_equal(a, b) and a.dtype == np.uint8 and a.ndim == 3 and a.shape[2] == 3
    assert not np.array_equal(a, stream_image(7, 124))


def test_synthetic_images_shapes_and_determinism():
    imgs = synthetic_images(4, 3)
    assert all(i.dtype == np.uint8 and i.ndim == 3 and i.shape[2] == 3 for i in imgs)
    assert all(np.array_equal(x, y) for x, y in zip(imgs, synthetic_images(4, 3)))
    fixed = synthetic_images(2, 5, hw=(333, 500))
    assert all(i.shape == (333, 500, 3) for i in fixed)
    im = synthetic_image(np.random.default_rng(0))
    assert np.array_equal(load_image_from_bytes(encode_png(im)), im)


def test_committed_workload_manifest_matches_reference_protocol():
    imgs = workload_images()
    from pathlib import Path

    root = Path(__file__).resolve().parents[1] / "data" / "synthetic_set"
    man = DatasetManifest.load(root / "manifest_w0_n100.json")
    assert len(imgs) == len(man.images) == 100
    assert man.distribution == {"3": 25, "4": 50, "5": 25}
    assert man.statistics["mean_detections"] == 4.0
    assert man.config["min_detections"] == 3 and man.config["max_detections"] == 5
