"""Run one batch through the executor eagerly, syncing after every op."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("ARENA_DEBUG_SYNC", "1")
import torch
from inference_arena_amd.models.zoo import make_yolo, make_mobilenet
from inference_arena_amd.engine.pipeline import GpuPipeline
from inference_arena_amd.data.synthetic import synthetic_images
pipe = GpuPipeline(make_yolo(0, cls_shift=-20.0), make_mobilenet(1), device=0, buckets=[int(sys.argv[1]) if len(sys.argv) > 1 else 4])
res = pipe.infer(synthetic_images(3, 21))
print("ok", [len(r) for r in res])
