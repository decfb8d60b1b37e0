"""Compare every executor buffer (no sharing) against the fp32 torch oracle's intermediates."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from inference_arena_amd.models.zoo import make_yolo, make_mobilenet
from inference_arena_amd.engine.pipeline import GpuPipeline
from inference_arena_amd.data.synthetic import synthetic_images
from inference_arena_amd.processing import YOLOPreprocessor
y, m = make_yolo(0, cls_shift=-20.0), make_mobilenet(1)
pipe = GpuPipeline(y, m, device=0, buckets=[1], share_buffers=False)
img = synthetic_images(1, 21)[0]
res = pipe.infer([img])
x = torch.from_numpy(YOLOPreprocessor()(img).tensor)
acts = {}
def hook(name):
    def f(mod, i, o):
        acts[name] = o.detach()
    return f
for n in ["b0", "b1", "b2", "b3", "b4", "b5", "b6", "b7", "b8", "b9", "h10", "h13", "h14", "h17", "h18", "h20", "h21", "h23"]:
    getattr(y, n).register_forward_hook(hook(n))
with torch.no_grad():
    maps = y.head_maps(x)
def cmp(name, buf, coff=0, C=None, ref=None):
    g = pipe.read_buffer(buf, 1)
    C = C or g.shape[-1]
    g = g[..., coff:coff + C]
    r = ref[0].permute(1, 2, 0).numpy()
    err = np.abs(g - r)
    rel = err.mean() / (np.abs(r).mean() + 1e-9)
    print(f"{name:6s} buf={buf:12s} shape={g.shape} rel_mean_err={rel:.4f} max_err={err.max():.3f} ref_absmean={np.abs(r).mean():.3f}", flush=True)
cmp("b0", "b0", ref=acts["b0"]); cmp("b1", "b1", ref=acts["b1"]); cmp("b2", "b2", ref=acts["b2"]); cmp("b3", "b3", ref=acts["b3"])
cmp("b4", "cat16", 64, 64, acts["b4"]); cmp("b5", "b5", ref=acts["b5"]); cmp("b6", "cat12", 128, 128, acts["b6"])
cmp("b7", "b7", ref=acts["b7"]); cmp("b8", "b8", ref=acts["b8"]); cmp("b9", "b9", ref=acts["b9"])
cmp("h10", "cat22", 128, 128, acts["h10"]); cmp("h13", "h13", ref=acts["h13"]); cmp("h14", "cat19", 64, 64, acts["h14"])
cmp("h17", "p3", ref=acts["h17"]); cmp("h18", "cat19", 0, 64, acts["h18"]); cmp("h20", "p4", ref=acts["h20"])
cmp("h21", "cat22", 0, 128, acts["h21"]); cmp("h23", "p5", ref=acts["h23"])
for l in range(3):
    cmp(f"head{l}", f"det{l}.out", ref=maps[l])
print("gpu dets", len(res[0]), res[0].boxes[:3].tolist(), res[0].classes[:3].tolist())
