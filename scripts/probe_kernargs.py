"""Does other GPU work clobber a captured graph's kernel arguments? (fault-free probe)"""
import os, sys, copy
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from inference_arena_amd.ops import native
C = native()
h = C.probe_create(1000)
print("fresh", C.probe_launch(h)[:4], flush=True)
x = torch.zeros(1, device="cuda:0")
for i in range(200):
    x += 1
torch.cuda.synchronize()
print("after 200 torch launches", C.probe_launch(h)[:4], flush=True)
for i in range(20000):
    x += 1
torch.cuda.synchronize()
print("after 20k torch launches", C.probe_launch(h)[:4], flush=True)
from inference_arena_amd.models.zoo import make_yolo
m = copy.deepcopy(make_yolo(0)).to("cuda:0")
torch.cuda.synchronize()
print("after model.to(cuda)", C.probe_launch(h)[:4], flush=True)
h2 = C.probe_create(5000)
for i in range(20000):
    x += 1
torch.cuda.synchronize()
print("second probe after 20k", C.probe_launch(h2)[:4], "first", C.probe_launch(h)[:4], flush=True)
