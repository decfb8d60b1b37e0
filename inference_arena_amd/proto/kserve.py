"""KServe-v2 / Triton ``inference.GRPCInferenceService`` predict protocol.

The reference's gateway talks to Triton through ``tritonclient.grpc``
(architectures/triton/gateway/app/triton_client.py:39-179: ServerReady,
ModelMetadata, ModelInfer with FP32 tensors).  The arena's model server
(server/model_server.py) implements the same service so that a stock
KServe-v2 client works against it; the message layouts follow the public
KServe-v2 specification (field numbers included), with Triton's extra
parameter kinds and the repository/statistics extensions the server uses.
"""
from __future__ import annotations

import numpy as np

from .builder import ProtoFile

_f = ProtoFile("arena/kserve_v2.proto", "inference")
N = ProtoFile.nested

_f.message("ServerLiveRequest", [])
_f.message("ServerLiveResponse", [("live", 1, "bool")])
_f.message("ServerReadyRequest", [])
_f.message("ServerReadyResponse", [("ready", 1, "bool")])
_f.message("ModelReadyRequest", [("name", 1, "string"), ("version", 2, "string")])
_f.message("ModelReadyResponse", [("ready", 1, "bool")])
_f.message("ServerMetadataRequest", [])
_f.message("ServerMetadataResponse", [("name", 1, "string"), ("version", 2, "string"),
                                      ("extensions", 3, "string", "repeated")])
_f.message("ModelMetadataRequest", [("name", 1, "string"), ("version", 2, "string")])
_f.message("ModelMetadataResponse",
           [("name", 1, "string"), ("versions", 2, "string", "repeated"), ("platform", 3, "string"),
            ("inputs", 4, "ModelMetadataResponse.TensorMetadata", "repeated"),
            ("outputs", 5, "ModelMetadataResponse.TensorMetadata", "repeated")],
           nested=[N("TensorMetadata", [("name", 1, "string"), ("datatype", 2, "string"),
                                        ("shape", 3, "int64", "repeated")])])
_f.message("InferParameter",
           [("bool_param", 1, "bool"), ("int64_param", 2, "int64"), ("string_param", 3, "string"),
            ("double_param", 4, "double"), ("uint64_param", 5, "uint64")],
           oneofs={k: "parameter_choice" for k in ("bool_param", "int64_param", "string_param", "double_param",
                                                   "uint64_param")})
_f.message("InferTensorContents",
           [("bool_contents", 1, "bool", "repeated"), ("int_contents", 2, "int32", "repeated"),
            ("int64_contents", 3, "int64", "repeated"), ("uint_contents", 4, "uint32", "repeated"),
            ("uint64_contents", 5, "uint64", "repeated"), ("fp32_contents", 6, "float", "repeated"),
            ("fp64_contents", 7, "double", "repeated"), ("bytes_contents", 8, "bytes", "repeated")])
_f.message("ModelInferRequest",
           [("model_name", 1, "string"), ("model_version", 2, "string"), ("id", 3, "string"),
            ("parameters", 4, "map<string, InferParameter>"),
            ("inputs", 5, "ModelInferRequest.InferInputTensor", "repeated"),
            ("outputs", 6, "ModelInferRequest.InferRequestedOutputTensor", "repeated"),
            ("raw_input_contents", 7, "bytes", "repeated")],
           nested=[N("InferInputTensor", [("name", 1, "string"), ("datatype", 2, "string"),
                                          ("shape", 3, "int64", "repeated"),
                                          ("parameters", 4, "map<string, InferParameter>"),
                                          ("contents", 5, "InferTensorContents")]),
                   N("InferRequestedOutputTensor", [("name", 1, "string"),
                                                    ("parameters", 2, "map<string, InferParameter>")])])
_f.message("ModelInferResponse",
           [("model_name", 1, "string"), ("model_version", 2, "string"), ("id", 3, "string"),
            ("parameters", 4, "map<string, InferParameter>"),
            ("outputs", 5, "ModelInferResponse.InferOutputTensor", "repeated"),
            ("raw_output_contents", 6, "bytes", "repeated")],
           nested=[N("InferOutputTensor", [("name", 1, "string"), ("datatype", 2, "string"),
                                           ("shape", 3, "int64", "repeated"),
                                           ("parameters", 4, "map<string, InferParameter>"),
                                           ("contents", 5, "InferTensorContents")])])
# repository / statistics extensions (subset)
_f.message("RepositoryIndexRequest", [("repository_name", 1, "string"), ("ready", 2, "bool")])
_f.message("RepositoryIndexResponse",
           [("models", 1, "RepositoryIndexResponse.ModelIndex", "repeated")],
           nested=[N("ModelIndex", [("name", 1, "string"), ("version", 2, "string"), ("state", 3, "string"),
                                    ("reason", 4, "string")])])
_f.message("ModelStatisticsRequest", [("name", 1, "string"), ("version", 2, "string")])
_f.message("ModelStatisticsResponse", [("model_stats", 1, "ModelStatisticsResponse.ModelStatistics", "repeated")],
           nested=[N("ModelStatistics", [("name", 1, "string"), ("version", 2, "string"),
                                         ("last_inference", 3, "uint64"), ("inference_count", 4, "uint64"),
                                         ("execution_count", 5, "uint64")])])
_f.service("GRPCInferenceService", [
    ("ServerLive", "ServerLiveRequest", "ServerLiveResponse"),
    ("ServerReady", "ServerReadyRequest", "ServerReadyResponse"),
    ("ModelReady", "ModelReadyRequest", "ModelReadyResponse"),
    ("ServerMetadata", "ServerMetadataRequest", "ServerMetadataResponse"),
    ("ModelMetadata", "ModelMetadataRequest", "ModelMetadataResponse"),
    ("ModelInfer", "ModelInferRequest", "ModelInferResponse"),
    ("RepositoryIndex", "RepositoryIndexRequest", "RepositoryIndexResponse"),
    ("ModelStatistics", "ModelStatisticsRequest", "ModelStatisticsResponse"),
])

pb = _f.build()
GRPCInferenceService = pb.services["GRPCInferenceService"]
for _n in dir(pb):
    if not _n.startswith("_") and _n not in ("services", "DESCRIPTOR"):
        globals()[_n] = getattr(pb, _n)

# ----------------------------------------------------------------- tensors
DTYPES = {"FP32": np.float32, "FP16": np.float16, "FP64": np.float64, "INT8": np.int8, "INT16": np.int16,
          "INT32": np.int32, "INT64": np.int64, "UINT8": np.uint8, "UINT16": np.uint16, "UINT32": np.uint32,
          "UINT64": np.uint64, "BOOL": np.bool_}
_CONTENTS = {"FP32": "fp32_contents", "FP64": "fp64_contents", "INT32": "int_contents", "INT16": "int_contents",
             "INT8": "int_contents", "INT64": "int64_contents", "UINT8": "uint_contents", "UINT16": "uint_contents",
             "UINT32": "uint_contents", "UINT64": "uint64_contents", "BOOL": "bool_contents"}


def serialize_bytes(items) -> bytes:
    """BYTES tensor wire form (Triton/KServe raw contents): 4-byte LE length + payload per element."""
    out = bytearray()
    for it in items:
        b = it if isinstance(it, (bytes, bytearray)) else str(it).encode()
        out += len(b).to_bytes(4, "little") + b
    return bytes(out)


def deserialize_bytes(buf: bytes) -> list[bytes]:
    out, i = [], 0
    while i < len(buf):
        if i + 4 > len(buf):
            raise ValueError("truncated BYTES tensor")
        n = int.from_bytes(buf[i:i + 4], "little")
        if i + 4 + n > len(buf):
            raise ValueError("truncated BYTES element")
        out.append(bytes(buf[i + 4:i + 4 + n]))
        i += 4 + n
    return out


def datatype_of(arr: np.ndarray) -> str:
    if arr.dtype == np.object_:
        return "BYTES"
    for k, v in DTYPES.items():
        if arr.dtype == v:
            return k
    raise ValueError(f"unsupported dtype {arr.dtype}")


def decode_input(req, i: int) -> np.ndarray:
    """Tensor ``i`` of a ModelInferRequest (raw_input_contents or typed contents)."""
    t = req.inputs[i]
    shape = tuple(int(s) for s in t.shape)
    if t.datatype == "BYTES":
        items = (deserialize_bytes(req.raw_input_contents[i]) if len(req.raw_input_contents) > i
                 else list(t.contents.bytes_contents))
        if len(items) != int(np.prod(shape)):
            raise ValueError(f"input '{t.name}': {len(items)} elements for shape {list(shape)}")
        arr = np.empty(len(items), dtype=object)
        arr[:] = items
        return arr.reshape(shape)
    dt = DTYPES.get(t.datatype)
    if dt is None:
        raise ValueError(f"unsupported datatype {t.datatype}")
    if len(req.raw_input_contents) > i:
        raw = req.raw_input_contents[i]
        a = np.frombuffer(raw, dtype=dt)
    else:
        a = np.asarray(getattr(t.contents, _CONTENTS[t.datatype]), dtype=dt)
    if a.size != int(np.prod(shape)):
        raise ValueError(f"input '{t.name}': {a.size} elements for shape {list(shape)}")
    return a.reshape(shape)


def encode_output(resp, name: str, arr: np.ndarray) -> None:
    arr = np.ascontiguousarray(arr)
    o = resp.outputs.add(name=name, datatype=datatype_of(arr))
    o.shape.extend(int(s) for s in arr.shape)
    resp.raw_output_contents.append(arr.tobytes())


def make_infer_request(model: str, inputs: dict[str, np.ndarray], outputs: list[str] | None = None,
                       request_id: str = "", version: str = ""):
    req = ModelInferRequest(model_name=model, model_version=version, id=request_id)  # noqa: F821
    for name, arr in inputs.items():
        arr = np.asarray(arr) if isinstance(arr, np.ndarray) and arr.dtype == np.object_ else np.ascontiguousarray(arr)
        t = req.inputs.add(name=name, datatype=datatype_of(arr))
        t.shape.extend(int(s) for s in arr.shape)
        req.raw_input_contents.append(serialize_bytes(arr.ravel()) if arr.dtype == np.object_ else arr.tobytes())
    for name in outputs or []:
        req.outputs.add(name=name)
    return req


def decode_outputs(resp) -> dict[str, np.ndarray]:
    out = {}
    for i, o in enumerate(resp.outputs):
        dt = DTYPES[o.datatype]
        shape = tuple(int(s) for s in o.shape)
        if len(resp.raw_output_contents) > i:
            a = np.frombuffer(resp.raw_output_contents[i], dtype=dt)
        else:
            a = np.asarray(getattr(o.contents, _CONTENTS[o.datatype]), dtype=dt)
        out[o.name] = a.reshape(shape)
    return out
