"""Diagnostic: executor behaviour around large torch allocations.

argv[1] mode: eager | recapture | torch_first
"""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mode = sys.argv[1]
if mode == "eager":
    os.environ["ARENA_DEBUG_SYNC"] = "1"
import numpy as np, torch
from inference_arena_amd.models.zoo import make_yolo, make_mobilenet
from inference_arena_amd.engine.pipeline import GpuPipeline
from inference_arena_amd.engine.planner import layout
from inference_arena_amd.data.synthetic import synthetic_images
dm = make_yolo(0, cls_shift=-20.0), make_mobilenet(1)
big = []
def torch_big():
    big.append(torch.randn(64, 1024, 1024, device="cuda:0"))   # 256 MB
    big.append(torch.nn.functional.conv2d(torch.randn(8, 64, 128, 128, device="cuda:0"), torch.randn(64, 64, 3, 3, device="cuda:0")))
    torch.cuda.synchronize()
if mode == "torch_first":
    torch_big()
pipe = GpuPipeline(*dm, device=0, buckets=[1, 4, 8])
imgs = synthetic_images(6, 21)
def show(tag):
    res = pipe.infer(imgs)
    print(mode, tag, [r.det_count for r in res], flush=True)
show("before")
torch_big()
if mode == "recapture":
    for B in pipe.buckets:
        offs, total = layout(pipe.program.buffers, B, pipe.ex.crop_cap_for(B))
        pipe.ex.add_bucket(B, offs, total)
show("after")
torch_big()
show("after2")
