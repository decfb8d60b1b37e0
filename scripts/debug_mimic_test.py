"""Mimic tests/test_pipeline_gpu.py step by step (copy mode 0), printing detections."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("OMP_NUM_THREADS", "4")
import numpy as np, torch
from inference_arena_amd.models.zoo import make_yolo, make_mobilenet
from inference_arena_amd.engine.pipeline import GpuPipeline
from inference_arena_amd.engine.reference import ReferencePipeline
from inference_arena_amd.data.synthetic import synthetic_images
print("cuda", torch.cuda.is_available(), flush=True)
dm = make_yolo(0, cls_shift=-20.0), make_mobilenet(1)
pipe = GpuPipeline(*dm, device=0, buckets=[1, 4, 8])
imgs = synthetic_images(6, 21)
def show(tag):
    res = pipe.infer(imgs)
    print(tag, [(len(r), r.det_count, round(float(r.scores.min()), 3) if len(r) else None) for r in res], flush=True)
show("first")
show("second")
ref = ReferencePipeline(*dm, device="cuda:0")
show("after ref init")
r = ref(imgs[0]); print("ref img0", len(r), flush=True)
show("after ref run")
