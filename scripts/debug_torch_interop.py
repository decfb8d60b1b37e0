"""Diagnostic: does torch CUDA work after executor creation corrupt the captured graphs?"""
import os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
code = r'''
import sys, json; sys.path.insert(0, %r)
import numpy as np, torch
MODE = %r
if MODE == "torch_first":
    torch.zeros(1, device="cuda:0"); torch.nn.functional.conv2d(torch.randn(1,3,32,32,device="cuda:0"), torch.randn(4,3,3,3,device="cuda:0"))
from inference_arena_amd.models.zoo import make_yolo, make_mobilenet
from inference_arena_amd.engine.pipeline import GpuPipeline
from inference_arena_amd.data.synthetic import synthetic_images
pipe = GpuPipeline(make_yolo(0, cls_shift=-20.0), make_mobilenet(1), device=0, buckets=[1, 4, 8])
if MODE == "torch_after":
    torch.zeros(1, device="cuda:0"); torch.nn.functional.conv2d(torch.randn(1,3,32,32,device="cuda:0"), torch.randn(4,3,3,3,device="cuda:0"))
if MODE == "alloc_after":
    x = torch.zeros(1, device="cuda:0")
res = pipe.infer(synthetic_images(3, 21))
print(json.dumps([[len(r), r.det_count] for r in res]))
''' 
for mode in ("none", "alloc_after", "torch_after", "torch_first"):
    r = subprocess.run([sys.executable, "-c", code % (ROOT, mode)], capture_output=True, text=True, timeout=200)
    print(mode, r.returncode, r.stdout.strip()[-300:], r.stderr.strip().splitlines()[-1:] if r.returncode else "")
