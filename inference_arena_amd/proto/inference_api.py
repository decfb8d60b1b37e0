"""The arena's own ``inference`` gRPC contract (wire-compatible with the
reference's src/shared/proto/inference.proto:30-152).

Services
  inference.ClassificationService  Classify, ClassifyBatch
      (implemented by server/classification_service.py — arm B, :8201)
  inference.InferenceService       Infer
      (declared but never implemented upstream; implemented here over the
       fused GPU pipeline by the same server)
  inference.Health                 Check
"""
from __future__ import annotations

from .builder import ProtoFile

_f = ProtoFile("arena/inference.proto", "inference")
_f.message("BoundingBox", [("x1", 1, "float"), ("y1", 2, "float"), ("x2", 3, "float"), ("y2", 4, "float"),
                           ("confidence", 5, "float"), ("class_id", 6, "int32")])
_f.message("ClassificationResult", [("class_id", 1, "int32"), ("class_name", 2, "string"),
                                    ("confidence", 3, "float")])
_f.message("TimingInfo", [("preprocessing_ms", 1, "double"), ("inference_ms", 2, "double"),
                          ("postprocessing_ms", 3, "double"), ("total_ms", 4, "double")])
# Arena extension (field 100, ignored by reference peers): the crop is named by a frame resident in device
# memory that the sender exported over IPC, cut at ``source_box`` on the receiver (server/device_transport.py).
_f.message("DeviceImageRef", [("handle", 1, "bytes"), ("device", 2, "int32"), ("offset", 3, "int64"),
                              ("height", 4, "int32"), ("width", 5, "int32")])
_f.message("ClassificationRequest", [("request_id", 1, "string"), ("image_crop", 2, "bytes"),
                                     ("source_box", 3, "BoundingBox"), ("device_image", 100, "DeviceImageRef")])
_f.message("ClassificationResponse", [("request_id", 1, "string"), ("result", 2, "ClassificationResult"),
                                      ("top_k", 3, "ClassificationResult", "repeated"), ("timing", 4, "TimingInfo"),
                                      ("error", 5, "string")])
_f.message("BatchClassificationRequest", [("requests", 1, "ClassificationRequest", "repeated")])
_f.message("BatchClassificationResponse", [("responses", 1, "ClassificationResponse", "repeated"),
                                           ("batch_timing", 2, "TimingInfo")])
_f.message("InferenceRequest", [("request_id", 1, "string"), ("image", 2, "bytes"),
                                ("detection_threshold", 3, "float"), ("max_detections", 4, "int32"),
                                ("top_k", 5, "int32")])
_f.message("DetectionWithClassification", [("detection", 1, "BoundingBox"),
                                           ("classification", 2, "ClassificationResult")])
_f.message("InferenceResponse", [("request_id", 1, "string"),
                                 ("results", 2, "DetectionWithClassification", "repeated"),
                                 ("timing", 3, "TimingInfo"), ("error", 4, "string")])
_f.message("HealthCheckRequest", [("service", 1, "string")])
_f.message("HealthCheckResponse", [("status", 1, "enum:HealthCheckResponse.ServingStatus")],
           enums=[("ServingStatus", [("UNKNOWN", 0), ("SERVING", 1), ("NOT_SERVING", 2)])])
_f.service("ClassificationService", [("Classify", "ClassificationRequest", "ClassificationResponse"),
                                     ("ClassifyBatch", "BatchClassificationRequest", "BatchClassificationResponse")])
_f.service("InferenceService", [("Infer", "InferenceRequest", "InferenceResponse")])
_f.service("Health", [("Check", "HealthCheckRequest", "HealthCheckResponse")])

pb = _f.build()
BoundingBox = pb.BoundingBox
ClassificationResult = pb.ClassificationResult
TimingInfo = pb.TimingInfo
DeviceImageRef = pb.DeviceImageRef
ClassificationRequest = pb.ClassificationRequest
ClassificationResponse = pb.ClassificationResponse
BatchClassificationRequest = pb.BatchClassificationRequest
BatchClassificationResponse = pb.BatchClassificationResponse
InferenceRequest = pb.InferenceRequest
InferenceResponse = pb.InferenceResponse
DetectionWithClassification = pb.DetectionWithClassification
HealthCheckRequest = pb.HealthCheckRequest
HealthCheckResponse = pb.HealthCheckResponse
ClassificationService = pb.services["ClassificationService"]
InferenceService = pb.services["InferenceService"]
Health = pb.services["Health"]
SERVING = HealthCheckResponse.SERVING
NOT_SERVING = HealthCheckResponse.NOT_SERVING
