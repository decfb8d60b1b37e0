"""Wire contract of the code-built protobufs (protoc is absent here, so the
descriptors are built in inference_arena_amd/proto/builder.py) against the
reference's own ``src/shared/proto/inference.proto`` text, read as a fixture
(reference tests/shared/test_proto.py checks the same file's syntax,
messages, fields and services).  When the reference checkout is absent, an
embedded copy of its field table is used instead."""
from __future__ import annotations

import re
from pathlib import Path

import pytest
from google.protobuf import descriptor_pb2
from google.protobuf.descriptor import FieldDescriptor

from inference_arena_amd.proto import inference_api as pb
from inference_arena_amd.proto import kserve as kv

REF_PROTO = Path("/root/reference/src/shared/proto/inference.proto")

# message -> {field: (number, type, repeated)} of the reference contract (inference.proto:30-152)
EMBEDDED = {
    "BoundingBox": {"x1": (1, "float", False), "y1": (2, "float", False), "x2": (3, "float", False),
                    "y2": (4, "float", False), "confidence": (5, "float", False), "class_id": (6, "int32", False)},
    "ClassificationResult": {"class_id": (1, "int32", False), "class_name": (2, "string", False),
                             "confidence": (3, "float", False)},
    "TimingInfo": {"preprocessing_ms": (1, "double", False), "inference_ms": (2, "double", False),
                   "postprocessing_ms": (3, "double", False), "total_ms": (4, "double", False)},
    "ClassificationRequest": {"request_id": (1, "string", False), "image_crop": (2, "bytes", False),
                              "source_box": (3, "BoundingBox", False)},
    "ClassificationResponse": {"request_id": (1, "string", False), "result": (2, "ClassificationResult", False),
                               "top_k": (3, "ClassificationResult", True), "timing": (4, "TimingInfo", False),
                               "error": (5, "string", False)},
    "BatchClassificationRequest": {"requests": (1, "ClassificationRequest", True)},
    "BatchClassificationResponse": {"responses": (1, "ClassificationResponse", True),
                                    "batch_timing": (2, "TimingInfo", False)},
    "InferenceRequest": {"request_id": (1, "string", False), "image": (2, "bytes", False),
                         "detection_threshold": (3, "float", False), "max_detections": (4, "int32", False),
                         "top_k": (5, "int32", False)},
    "DetectionWithClassification": {"detection": (1, "BoundingBox", False),
                                    "classification": (2, "ClassificationResult", False)},
    "InferenceResponse": {"request_id": (1, "string", False), "results": (2, "DetectionWithClassification", True),
                          "timing": (3, "TimingInfo", False), "error": (4, "string", False)},
    "HealthCheckRequest": {"service": (1, "string", False)},
    "HealthCheckResponse": {"status": (1, "ServingStatus", False)},
}
SERVICES = {
    "ClassificationService": {"Classify": ("ClassificationRequest", "ClassificationResponse"),
                              "ClassifyBatch": ("BatchClassificationRequest", "BatchClassificationResponse")},
    "InferenceService": {"Infer": ("InferenceRequest", "InferenceResponse")},
    "Health": {"Check": ("HealthCheckRequest", "HealthCheckResponse")},
}


def _parse_reference(text: str):
    """Minimal proto3 parser for the reference file: messages (one nesting level), services."""
    text = re.sub(r"//[^\n]*", "", text)
    msgs: dict[str, dict] = {}
    for m in re.finditer(r"message\s+(\w+)\s*\{", text):
        name, depth, i = m.group(1), 1, m.end()
        while depth:
            depth += {"{": 1, "}": -1}.get(text[i], 0)
            i += 1
        body = text[m.end():i - 1]
        body = re.sub(r"enum\s+\w+\s*\{[^}]*\}", "", body)  # nested enum values are not fields
        fields = {}
        for f in re.finditer(r"(repeated\s+)?([\w.]+)\s+(\w+)\s*=\s*(\d+)\s*;", body):
            fields[f.group(3)] = (int(f.group(4)), f.group(2).split(".")[-1], bool(f.group(1)))
        msgs[name] = fields
    svcs: dict[str, dict] = {}
    for s in re.finditer(r"service\s+(\w+)\s*\{([^}]*)\}", text):
        svcs[s.group(1)] = {r.group(1): (r.group(2), r.group(3)) for r in
                            re.finditer(r"rpc\s+(\w+)\s*\(\s*(\w+)\s*\)\s*returns\s*\(\s*(\w+)\s*\)", s.group(2))}
    pkg = re.search(r"package\s+([\w.]+)\s*;", text).group(1)
    return pkg, msgs, svcs


@pytest.fixture(scope="module")
def reference():
    if REF_PROTO.exists():
        return _parse_reference(REF_PROTO.read_text())
    return "inference", EMBEDDED, SERVICES


_SCALAR = {FieldDescriptor.TYPE_FLOAT: "float", FieldDescriptor.TYPE_DOUBLE: "double",
           FieldDescriptor.TYPE_INT32: "int32", FieldDescriptor.TYPE_INT64: "int64",
           FieldDescriptor.TYPE_STRING: "string", FieldDescriptor.TYPE_BYTES: "bytes",
           FieldDescriptor.TYPE_BOOL: "bool", FieldDescriptor.TYPE_UINT32: "uint32",
           FieldDescriptor.TYPE_UINT64: "uint64"}


def _ours(msg_cls):
    out = {}
    for f in msg_cls.DESCRIPTOR.fields:
        if f.type == FieldDescriptor.TYPE_MESSAGE:
            t = f.message_type.name
        elif f.type == FieldDescriptor.TYPE_ENUM:
            t = f.enum_type.name
        else:
            t = _SCALAR[f.type]
        out[f.name] = (f.number, t, bool(f.is_repeated))
    return out


def test_reference_parse_matches_embedded_table(reference):
    pkg, msgs, svcs = reference
    assert pkg == "inference"
    assert msgs == EMBEDDED
    assert svcs == SERVICES


# arena extensions: additive fields with numbers far from the reference's (a reference peer skips them)
EXTENSIONS = {"ClassificationRequest": {"device_image": (100, "DeviceImageRef", False)}}


@pytest.mark.parametrize("name", sorted(EMBEDDED))
def test_message_fields_match_reference(reference, name):
    _, msgs, _ = reference
    ours = _ours(getattr(pb, name))
    ext = EXTENSIONS.get(name, {})
    assert {k: v for k, v in ours.items() if k not in ext} == msgs[name]
    assert {k: ours[k] for k in ext} == ext
    assert all(n >= 100 for n, _, _ in ext.values())


def test_health_enum_values():
    e = pb.HealthCheckResponse.DESCRIPTOR.enum_types_by_name["ServingStatus"]
    assert {v.name: v.number for v in e.values} == {"UNKNOWN": 0, "SERVING": 1, "NOT_SERVING": 2}


@pytest.mark.parametrize("service", sorted(SERVICES))
def test_services_and_paths(reference, service):
    _, _, svcs = reference
    svc = getattr(pb, service)
    assert set(svc.methods) == set(svcs[service])
    for method, (req, resp) in svcs[service].items():
        r, s = svc.methods[method]
        assert (r.DESCRIPTOR.name, s.DESCRIPTOR.name) == (req, resp)
        assert svc.path(method) == f"/inference.{service}/{method}"


def test_full_names_are_in_the_reference_package():
    for name in EMBEDDED:
        assert getattr(pb, name).DESCRIPTOR.full_name == f"inference.{name}"


def test_roundtrip_nested_and_repeated():
    r = pb.ClassificationResponse(request_id="a_1")
    r.result.class_id, r.result.class_name, r.result.confidence = 7, "cat", 0.5
    for k in range(5):
        r.top_k.add(class_id=k, class_name=str(k), confidence=1.0 / (k + 1))
    r.timing.total_ms = 3.25
    back = pb.ClassificationResponse.FromString(r.SerializeToString())
    assert back == r and len(back.top_k) == 5 and back.top_k[4].confidence == pytest.approx(0.2)
    batch = pb.BatchClassificationResponse(responses=[r, r])
    assert pb.BatchClassificationResponse.FromString(batch.SerializeToString()).responses[1].result.class_name == "cat"


def test_unknown_fields_survive_roundtrip():
    """A newer peer's extra field is kept (proto3 unknown-field preservation)."""
    extra = pb.BoundingBox(x1=1.0).SerializeToString() + bytes([0x38, 0x2A])  # field 7 varint 42
    b = pb.BoundingBox.FromString(extra)
    assert b.x1 == 1.0 and b.SerializeToString().endswith(bytes([0x38, 0x2A]))


def test_file_descriptor_is_proto3_and_serializable():
    fd = descriptor_pb2.FileDescriptorProto()
    pb.BoundingBox.DESCRIPTOR.file.CopyToProto(fd)
    assert fd.package == "inference" and fd.syntax == "proto3"
    assert {m.name for m in fd.message_type} >= set(EMBEDDED)
    assert {s.name for s in fd.service} == set(SERVICES)


def test_kserve_contract_fields():
    """KServe v2 (Triton) messages used by the reference gateway (tritonclient.grpc: ServerReady,
    ModelMetadata, ModelInfer with InferInput / InferRequestedOutput)."""
    f = lambda m: {x.name: x.number for x in m.DESCRIPTOR.fields}  # noqa: E731
    assert f(kv.ModelInferRequest)["model_name"] == 1
    assert f(kv.ModelInferRequest)["inputs"] == 5 and f(kv.ModelInferRequest)["outputs"] == 6
    assert f(kv.ModelInferRequest)["raw_input_contents"] == 7
    assert f(kv.ModelInferResponse)["raw_output_contents"] == 6
    assert f(kv.ServerReadyResponse) == {"ready": 1}
    assert f(kv.ModelMetadataRequest) == {"name": 1, "version": 2}
    assert kv.GRPCInferenceService.path("ModelInfer") == "/inference.GRPCInferenceService/ModelInfer"
    t = kv.ModelInferRequest.InferInputTensor(name="images", datatype="FP32", shape=[1, 3, 640, 640])
    req = kv.ModelInferRequest(model_name="yolov5n", inputs=[t], raw_input_contents=[b"\0" * 16])
    back = kv.ModelInferRequest.FromString(req.SerializeToString())
    assert list(back.inputs[0].shape) == [1, 3, 640, 640] and back.raw_input_contents[0] == b"\0" * 16
