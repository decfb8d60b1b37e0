"""``config.pbtxt`` — model configuration of the arena model server.

The reference generates Triton configs with string templates
(infrastructure/minio/triton_config.py:49-131: name, platform
``onnxruntime_onnx``, ``max_batch_size: 0``, full-rank dims, one
``instance_group`` of KIND_CPU, ORT thread ``parameters``) and validates them
by substring search (:193-221).  Here the configuration schema is a protobuf
message (a subset of Triton's ModelConfig, same field names), so configs are
parsed and emitted with ``google.protobuf.text_format`` — any Triton-style
``config.pbtxt`` using these fields round-trips, and a typo is a parse error
instead of a silently ignored line.

Fields: name, platform, backend, max_batch_size, input/output (name,
data_type, dims, reshape, optional, label_filename), instance_group (name,
kind, count, gpus), dynamic_batching (preferred_batch_size,
max_queue_delay_microseconds, preserve_ordering), parameters
(map<string,{string_value}>), ensemble_scheduling (step: model_name,
model_version, input_map, output_map), version_policy (latest/all/specific),
default_model_filename.
"""
from __future__ import annotations

from google.protobuf import text_format

from ..proto.builder import ProtoFile

_f = ProtoFile("arena/model_config.proto", "arena.config")
N = ProtoFile.nested
DATA_TYPES = ["TYPE_INVALID", "TYPE_BOOL", "TYPE_UINT8", "TYPE_UINT16", "TYPE_UINT32", "TYPE_UINT64", "TYPE_INT8",
              "TYPE_INT16", "TYPE_INT32", "TYPE_INT64", "TYPE_FP16", "TYPE_FP32", "TYPE_FP64", "TYPE_STRING",
              "TYPE_BF16"]
_f.message("DataTypeHolder", [], enums=[("DataType", [(n, i) for i, n in enumerate(DATA_TYPES)])])
_f.message("ModelTensorReshape", [("shape", 1, "int64", "repeated")])
_f.message("ModelInput", [("name", 1, "string"), ("data_type", 2, "enum:DataTypeHolder.DataType"),
                          ("dims", 4, "int64", "repeated"), ("reshape", 5, "ModelTensorReshape"),
                          ("optional", 9, "bool")])
_f.message("ModelOutput", [("name", 1, "string"), ("data_type", 2, "enum:DataTypeHolder.DataType"),
                           ("dims", 3, "int64", "repeated"), ("reshape", 5, "ModelTensorReshape"),
                           ("label_filename", 4, "string")])
_f.message("ModelInstanceGroup", [("name", 1, "string"), ("kind", 4, "enum:ModelInstanceGroup.Kind"),
                                  ("count", 2, "int32"), ("gpus", 3, "int32", "repeated")],
           enums=[("Kind", [("KIND_AUTO", 0), ("KIND_GPU", 1), ("KIND_CPU", 2), ("KIND_MODEL", 3)])])
_f.message("ModelDynamicBatching", [("preferred_batch_size", 1, "int32", "repeated"),
                                    ("max_queue_delay_microseconds", 2, "uint64"),
                                    ("preserve_ordering", 3, "bool")])
_f.message("ModelParameter", [("string_value", 1, "string")])
_f.message("ModelVersionPolicy",
           [("latest", 1, "ModelVersionPolicy.Latest"), ("all", 2, "ModelVersionPolicy.All"),
            ("specific", 3, "ModelVersionPolicy.Specific")],
           nested=[N("Latest", [("num_versions", 1, "uint32")]), N("All", []),
                   N("Specific", [("versions", 1, "int64", "repeated")])],
           oneofs={"latest": "policy_choice", "all": "policy_choice", "specific": "policy_choice"})
_f.message("ModelEnsembling",
           [("step", 1, "ModelEnsembling.Step", "repeated")],
           nested=[N("Step", [("model_name", 1, "string"), ("model_version", 2, "int64"),
                              ("input_map", 3, "map<string, string>"), ("output_map", 4, "map<string, string>")])])
_f.message("ModelConfig", [
    ("name", 1, "string"), ("platform", 2, "string"), ("backend", 17, "string"),
    ("version_policy", 3, "ModelVersionPolicy"), ("max_batch_size", 4, "int32"),
    ("input", 5, "ModelInput", "repeated"), ("output", 6, "ModelOutput", "repeated"),
    ("instance_group", 7, "ModelInstanceGroup", "repeated"), ("default_model_filename", 8, "string"),
    ("dynamic_batching", 11, "ModelDynamicBatching"), ("parameters", 14, "map<string, ModelParameter>"),
    ("ensemble_scheduling", 15, "ModelEnsembling"),
])
pb = _f.build()
ModelConfig = pb.ModelConfig
DataType = pb.DataTypeHolder.DataType
Kind = pb.ModelInstanceGroup.Kind

NP_TO_TYPE = {"float32": "TYPE_FP32", "float16": "TYPE_FP16", "uint8": "TYPE_UINT8", "int32": "TYPE_INT32",
              "int64": "TYPE_INT64", "bool": "TYPE_BOOL", "float64": "TYPE_FP64"}
TYPE_TO_KSERVE = {"TYPE_FP32": "FP32", "TYPE_FP16": "FP16", "TYPE_UINT8": "UINT8", "TYPE_INT32": "INT32",
                  "TYPE_INT64": "INT64", "TYPE_BOOL": "BOOL", "TYPE_FP64": "FP64", "TYPE_BF16": "BF16",
                  "TYPE_STRING": "BYTES", "TYPE_INT8": "INT8", "TYPE_INT16": "INT16", "TYPE_UINT16": "UINT16",
                  "TYPE_UINT32": "UINT32", "TYPE_UINT64": "UINT64"}

PLATFORM = "arena_hip"  # executor programs compiled from the repository weights
ENSEMBLE = "ensemble"


class ConfigError(ValueError):
    pass


def parse(text: str):
    """config.pbtxt text -> ModelConfig (ConfigError on syntax / unknown field)."""
    cfg = ModelConfig()
    try:
        text_format.Parse(text, cfg)
    except text_format.ParseError as e:
        raise ConfigError(str(e)) from e
    return cfg


def dump(cfg, header: str = "") -> str:
    body = text_format.MessageToString(cfg, use_short_repeated_primitives=True)
    return (header.rstrip() + "\n\n" if header else "") + body


def data_type_name(v: int) -> str:
    return DataType.Name(v)


def validate(cfg) -> list[str]:
    """Structural checks (reference validator: required name/platform/input/output/instance_group)."""
    errs = []
    if not cfg.name:
        errs.append("missing name")
    if not cfg.platform and not cfg.backend:
        errs.append("missing platform/backend")
    if cfg.platform != ENSEMBLE and not len(cfg.instance_group):
        errs.append("missing instance_group")
    if not len(cfg.input):
        errs.append("missing input")
    if not len(cfg.output):
        errs.append("missing output")
    for t in list(cfg.input) + list(cfg.output):
        if not t.name:
            errs.append("tensor without name")
        if t.data_type == 0:
            errs.append(f"tensor '{t.name}' has no data_type")
        if not len(t.dims):
            errs.append(f"tensor '{t.name}' has no dims")
        if any(d == 0 or d < -1 for d in t.dims):
            errs.append(f"tensor '{t.name}' has invalid dims {list(t.dims)}")
    if cfg.max_batch_size < 0:
        errs.append("max_batch_size must be >= 0")
    if cfg.HasField("dynamic_batching"):
        if cfg.max_batch_size == 0:
            errs.append("dynamic_batching requires max_batch_size > 0")
        for p in cfg.dynamic_batching.preferred_batch_size:
            if p <= 0 or (cfg.max_batch_size and p > cfg.max_batch_size):
                errs.append(f"preferred_batch_size {p} outside (0, max_batch_size]")
    for g in cfg.instance_group:
        if g.count < 0:
            errs.append("instance_group count must be >= 0")
    if cfg.platform == ENSEMBLE and not len(cfg.ensemble_scheduling.step):
        errs.append("ensemble without ensemble_scheduling steps")
    return errs


def generate(model_name: str, *, reference_compat: bool = False, gpus: list[int] | None = None) -> object:
    """ModelConfig for a model of experiment.yaml.

    ``reference_compat=True`` reproduces the reference's config exactly in
    content (max_batch_size 0, full-rank dims incl. the batch 1, no
    dynamic_batching); the default enables the server-side dynamic batcher
    (``triton.dynamic_batching``) with batch-less dims.  Instance kind/count
    and the thread parameters come from the ``triton`` section; ``gpus`` (or
    ``triton.instance_group.gpus``) lists the devices of a KIND_GPU group —
    ``count`` instances on each (Triton semantics, parallel/placement.py).
    """
    from ..config import get_model_config, get_triton_config

    mc = get_model_config(model_name)
    tc = get_triton_config()
    cfg = ModelConfig(name=model_name, platform=PLATFORM)
    db = tc.get("dynamic_batching") or {}
    batched = bool(db) and not reference_compat
    cfg.max_batch_size = int(db.get("max_batch_size", 32)) if batched else 0
    for spec, coll in ((mc["input"], cfg.input), (mc["output"], cfg.output)):
        t = coll.add(name=spec["name"], data_type=DataType.Value(NP_TO_TYPE[spec.get("dtype", "float32")]))
        dims = list(spec["shape"])
        t.dims.extend(dims[1:] if batched else dims)
    ig = tc.get("instance_group", {}) or {}
    kind = str(ig.get("kind", "KIND_GPU"))
    g = cfg.instance_group.add(count=int(ig.get("count", 1)), kind=Kind.Value(kind))
    dev = gpus if gpus is not None else ig.get("gpus")
    if dev and kind != "KIND_CPU" and not reference_compat:
        g.gpus.extend(int(x) for x in dev)
    for k, v in (tc.get("parameters") or {}).items():
        cfg.parameters[k].string_value = str(v)
    if batched:
        cfg.dynamic_batching.preferred_batch_size.extend(int(p) for p in db.get("preferred_batch_size", []))
        cfg.dynamic_batching.max_queue_delay_microseconds = int(db.get("max_queue_delay_microseconds", 500))
    return cfg


def generate_pipeline(name: str = "arena_pipeline", detector: str = "yolov5n", classifier: str = "mobilenetv2"):
    """Ensemble: one image -> detections + top-5 classifications of every crop.

    Inputs (one of): ``IMAGE`` RGB uint8 [H, W, 3] or ``IMAGE_BYTES`` (the
    encoded JPEG/PNG, decoded by the server — ships ~100 KB instead of the
    4.9 MB FP32 tensor the reference gateway sends per request).

    The server compiles this ensemble into ONE fused device program
    (letterbox -> YOLO -> decode/NMS -> crop-gather -> MobileNetV2 -> top-5)
    instead of running the steps as separate models.
    """
    from ..config import get_triton_config

    tc = get_triton_config()
    cfg = ModelConfig(name=name, platform=ENSEMBLE, max_batch_size=0)
    cfg.input.add(name="IMAGE", data_type=DataType.Value("TYPE_UINT8"), dims=[-1, -1, 3], optional=True)
    cfg.input.add(name="IMAGE_BYTES", data_type=DataType.Value("TYPE_STRING"), dims=[1], optional=True)
    cfg.output.add(name="DETECTIONS", data_type=DataType.Value("TYPE_FP32"), dims=[-1, 6])
    cfg.output.add(name="CLASS_IDS", data_type=DataType.Value("TYPE_INT32"), dims=[-1, 5])
    cfg.output.add(name="CLASS_LOGITS", data_type=DataType.Value("TYPE_FP32"), dims=[-1, 5])
    cfg.output.add(name="CLASS_PROBS", data_type=DataType.Value("TYPE_FP32"), dims=[-1, 5])
    cfg.output.add(name="STAGE_MS", data_type=DataType.Value("TYPE_FP32"), dims=[4])
    s1 = cfg.ensemble_scheduling.step.add(model_name=detector, model_version=-1)
    s1.input_map["images"] = "IMAGE"
    s1.output_map["output0"] = "DETECTIONS"
    s2 = cfg.ensemble_scheduling.step.add(model_name=classifier, model_version=-1)
    s2.input_map["input"] = "DETECTIONS"
    s2.output_map["output"] = "CLASS_LOGITS"
    db = tc.get("dynamic_batching") or {}
    cfg.parameters["max_batch"].string_value = str(int(db.get("max_batch_size", 32)))
    cfg.parameters["max_queue_delay_microseconds"].string_value = str(int(db.get("max_queue_delay_microseconds",
                                                                                 500)))
    ig = tc.get("instance_group", {}) or {}
    cfg.parameters["instance_count"].string_value = str(int(ig.get("count", 1)))
    return cfg
