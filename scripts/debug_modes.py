"""Compare executor execution modes on the same batch (diagnostic)."""
import os, subprocess, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
code = r'''
import sys, json; sys.path.insert(0, %r)
import numpy as np, torch
from inference_arena_amd.models.zoo import make_yolo, make_mobilenet
from inference_arena_amd.engine.pipeline import GpuPipeline
from inference_arena_amd.data.synthetic import synthetic_images
pipe = GpuPipeline(make_yolo(0, cls_shift=-20.0), make_mobilenet(1), device=0, buckets=[1, 4, 8])
out = []
for n in (3, 6, 1):
    res = pipe.infer(synthetic_images(n, 21))
    out.append([[len(r), float(r.boxes.sum()) if len(r) else 0.0] for r in res])
print(json.dumps(out))
''' % ROOT
for env in ({"ARENA_DEBUG_SYNC": "1"}, {}, {"ARENA_COPY_MODE": "1"}, {"ARENA_COPY_MODE": "2"}):
    e = dict(os.environ, **env)
    r = subprocess.run([sys.executable, "-c", code], env=e, capture_output=True, text=True, timeout=200)
    print(env, r.returncode, r.stdout.strip()[-600:], r.stderr.strip().splitlines()[-1:] if r.returncode else "")
