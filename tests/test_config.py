"""experiment.yaml loader / accessors / validator (reference contract:
src/shared/config.py:57-475; invariants asserted by tests/shared/test_config.py:
bs = 1, 3 channels, ordered user levels, Triton threads == ORT threads as
strings, locust tool)."""
from __future__ import annotations

import textwrap

import pytest
import yaml

from inference_arena_amd import config as C


@pytest.fixture(autouse=True)
def _fresh_config():
    C.reload_config()
    yield
    C.reload_config()


def test_config_loads_and_is_cached():
    a = C.get_config()
    b = C.get_config()
    assert a is b
    assert isinstance(a, dict)
    c = C.reload_config()
    assert c is not a and c == a


def test_required_top_level_sections():
    cfg = C.get_config()
    for sec in ("metadata", "research_questions", "hypotheses", "independent_variables", "controlled_variables",
                "infrastructure", "triton", "changelog"):
        assert sec in cfg, sec


def test_validate_config_clean():
    assert C.validate_config() == []


def test_model_names_and_configs():
    assert C.get_model_names() == ["yolov5n", "mobilenetv2"]
    y = C.get_model_config("yolov5n")
    m = C.get_model_config("mobilenetv2")
    assert y["input"]["shape"] == [1, 3, 640, 640]
    assert y["output"]["shape"] == [1, 84, 8400]
    assert m["input"]["shape"] == [1, 3, 224, 224]
    assert m["output"]["shape"] == [1, 1000]
    assert y["confidence_threshold"] == 0.5 and y["iou_threshold"] == 0.45


@pytest.mark.parametrize("name", ["yolov5n", "mobilenetv2"])
def test_model_input_invariants(name):
    shape = C.get_model_config(name)["input"]["shape"]
    assert shape[0] == 1, "batch dimension stays 1 in models.* (batching lives in the gpu: section)"
    assert shape[1] == 3
    assert shape[2] == shape[3]


def test_yolo_output_matches_anchor_count():
    out = C.get_model_config("yolov5n")["output"]["shape"]
    size = C.get_controlled_variable("preprocessing", "yolo")["target_size"]
    anchors = sum((size // s) ** 2 for s in (8, 16, 32))
    assert out == [1, 4 + 80, anchors]


def test_unknown_model_raises():
    with pytest.raises(KeyError, match="nope"):
        C.get_model_config("nope")


def test_preprocessing_sizes_match_model_inputs():
    yp = C.get_controlled_variable("preprocessing", "yolo")
    mp = C.get_controlled_variable("preprocessing", "mobilenet")
    assert yp["target_size"] == C.get_model_config("yolov5n")["input"]["shape"][2]
    assert mp["target_size"] == C.get_model_config("mobilenetv2")["input"]["shape"][2]
    assert yp["normalization_scale"] == 255.0
    assert mp["mean"] == pytest.approx([0.485, 0.456, 0.406])
    assert mp["std"] == pytest.approx([0.229, 0.224, 0.225])


def test_controlled_variable_errors():
    with pytest.raises(KeyError):
        C.get_controlled_variables("no_such_section")
    with pytest.raises(KeyError):
        C.get_controlled_variable("preprocessing", "no_such_key")


def test_onnx_runtime_threads_and_triton_parameters_agree():
    ort = C.get_controlled_variables("onnx_runtime")
    tr = C.get_triton_config()["parameters"]
    assert tr["intra_op_thread_count"] == str(ort["intra_op_num_threads"])
    assert tr["inter_op_thread_count"] == str(ort["inter_op_num_threads"])
    assert isinstance(tr["intra_op_thread_count"], str)


def test_triton_section_has_gpu_instance_group_and_dynamic_batching():
    tr = C.get_triton_config()
    assert tr["instance_group"]["kind"] in ("KIND_GPU", "KIND_CPU")
    assert tr["instance_group"]["count"] >= 1
    db = tr["dynamic_batching"]
    assert db["preferred_batch_size"] == sorted(db["preferred_batch_size"])
    assert max(db["preferred_batch_size"]) <= db["max_batch_size"]
    assert db["max_queue_delay_microseconds"] > 0


def test_concurrent_user_levels_ordered():
    levels = C.get_concurrent_user_levels()
    assert levels == sorted(levels)
    assert levels[0] == 1 and levels[-1] == 100
    assert len(set(levels)) == len(levels)


def test_architecture_levels():
    iv = C.get_config()["independent_variables"]
    assert iv["architecture"]["levels"] == ["monolithic", "microservices", "triton"]


def test_load_testing_protocol():
    lt = C.get_load_testing_config()
    assert lt["tool"] == "locust"
    ph = lt["phases"]
    assert ph["warmup"]["duration_seconds"] == 60
    assert ph["measurement"]["duration_seconds"] == 180
    assert ph["cooldown"]["duration_seconds"] == 30
    assert lt["runs_per_configuration"] == 3


def test_hypotheses_accessors():
    h = C.get_hypothesis("H1a")
    assert h["category"] == "performance"
    perf = C.get_hypotheses_by_category("performance")
    assert set(perf) >= {"H1a", "H1b", "H1c", "H1d"}
    assert all(v["category"] == "performance" for v in perf.values())
    assert C.get_hypotheses_by_category("does_not_exist") == {}
    with pytest.raises(KeyError):
        C.get_hypothesis("H9z")


def test_every_hypothesis_has_required_fields():
    for hid, h in C.get_config()["hypotheses"].items():
        for f in ("category", "statement", "rationale"):
            assert f in h, (hid, f)
        assert "testable_prediction" in h or "prediction" in h, hid


def test_dataset_spec():
    ds = C.get_controlled_variables("dataset")
    assert ds["detection_range"] == {"min": 3, "max": 5}
    assert ds["random_seed"] == 42
    assert ds["sample_size"] == 100
    assert ds["target_distribution"]["mean"] == 4.0


def test_resources_per_architecture():
    r = C.get_controlled_variables("resources")
    assert r["monolithic"]["containers"] == 1
    for arch in ("microservices", "triton"):
        assert r[arch]["containers"] == 2
        assert r[arch]["total_vcpu"] == 2 * r["vcpu_per_container"]


def test_infrastructure_accessors():
    infra = C.get_infrastructure_config()
    assert "minio" in infra
    assert C.get_minio_config() == infra["minio"]
    with pytest.raises(KeyError):
        C.get_infrastructure_config("nonexistent_service")


def test_metadata_and_version():
    md = C.get_metadata()
    assert "title" in md
    assert C.get_spec_version() == str(md["spec_version"])


def test_gpu_section_defaults_and_values():
    g = C.get_gpu_config()
    assert g["arch"] == "gfx950"
    assert g["batch_buckets"] == sorted(g["batch_buckets"])
    assert g["batch_buckets"][-1] == C.get_triton_config()["dynamic_batching"]["max_batch_size"]
    assert g["replicas"] == [1, 2, 4, 8]
    assert g["dtype"] == "fp32"  # the reference's precision (ONNX Runtime fp32); bf16 is opt-in
    ports = g["ports"]
    assert (ports["monolithic"], ports["detection"], ports["classification"], ports["gateway"]) == (8100, 8200, 8201,
                                                                                                      8300)
    assert (ports["model_http"], ports["model_grpc"], ports["metrics"]) == (8000, 8001, 8002)


def _write(tmp_path, text: str):
    p = tmp_path / "experiment.yaml"
    p.write_text(textwrap.dedent(text))
    return p


def test_env_override_and_validation_errors(tmp_path, monkeypatch):
    p = _write(tmp_path, """
        metadata: {title: t, spec_version: 9.9}
        hypotheses:
          H1: {category: performance, statement: s}
        controlled_variables:
          models:
            yolov5n: {opset_version: 17, input: {}, output: {}}
          onnx_runtime: {intra_op_num_threads: 2}
        gpu: {batch_buckets: [4, 2]}
    """)
    monkeypatch.setenv("ARENA_EXPERIMENT_YAML", str(p))
    C.reload_config()
    assert C.config_path() == p
    assert C.get_spec_version() == "9.9"
    errs = C.validate_config()
    joined = "\n".join(errs)
    assert "Missing required section: research_questions" in joined
    assert "Missing model configuration: mobilenetv2" in joined
    assert "Missing onnx_runtime field: inter_op_num_threads" in joined
    assert "Hypothesis H1 missing required field: rationale" in joined
    assert "testable_prediction" in joined
    assert "gpu.batch_buckets" in joined


def test_missing_file_reported(tmp_path, monkeypatch):
    monkeypatch.setenv("ARENA_EXPERIMENT_YAML", str(tmp_path / "absent.yaml"))
    with pytest.raises(FileNotFoundError):
        C.reload_config()
    errs = C.validate_config()
    assert errs and errs[0].startswith("Failed to load config")


def test_non_mapping_file_rejected(tmp_path, monkeypatch):
    p = tmp_path / "experiment.yaml"
    p.write_text("- just\n- a list\n")
    monkeypatch.setenv("ARENA_EXPERIMENT_YAML", str(p))
    with pytest.raises(ValueError, match="mapping"):
        C.reload_config()


def test_yaml_is_parsed_safely(tmp_path, monkeypatch):
    p = tmp_path / "experiment.yaml"
    p.write_text("metadata: !!python/object/apply:os.system ['true']\n")
    monkeypatch.setenv("ARENA_EXPERIMENT_YAML", str(p))
    with pytest.raises(yaml.YAMLError):
        C.reload_config()


def test_gpu_defaults_when_section_absent(tmp_path, monkeypatch):
    p = _write(tmp_path, "metadata: {spec_version: 1}\n")
    monkeypatch.setenv("ARENA_EXPERIMENT_YAML", str(p))
    C.reload_config()
    g = C.get_gpu_config()
    assert g["batch_buckets"] == [1, 2, 4, 8, 16, 32] and g["max_det"] == 300


def test_monitoring_metrics_listed():
    mon = C.get_controlled_variables("monitoring")
    assert mon
