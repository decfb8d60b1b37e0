#!/usr/bin/env python3
"""Build the native extension ``inference_arena_amd/_C*.so`` in-tree.

Every HIP kernel and the C++ runtime (executor, dynamic batcher, pybind11
bindings) are compiled by ``hipcc --offload-arch=gfx950`` into object files
under ``build/obj`` (rebuilt only when a source or header is newer), then
linked into one shared library next to the Python package so that the GPU
box loads it from the snapshot of the repository.

The HIP runtime is resolved at import time from the one PyTorch already
loaded (``libamdhip64.so.7`` is matched by SONAME), so tensors allocated by
torch and buffers used by the kernels live in the same HIP runtime.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "csrc"
OBJ = ROOT / "build" / "obj"
PKG = ROOT / "inference_arena_amd"
ARCH = os.environ.get("ARENA_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

SOURCES = [
    "kernels/conv_mfma.hip",
    "kernels/conv_f32.hip",
    "kernels/gemm_x3.hip",
    "kernels/halo_x3g.hip",
    "kernels/stem_x3.hip",
    "kernels/ir_f32.hip",
    "kernels/ir_crop_f32.hip",
    "kernels/ir_tile_x3.hip",
    "kernels/dwconv.hip",
    "kernels/ir_block.hip",
    "kernels/ir_block_wave.hip",
    "kernels/ir_crop.hip",
    "kernels/conv_igemm.hip",
    "kernels/conv_pw.hip",
    "kernels/conv3x3_v3.hip",
    "kernels/c3_fused.hip",
    "kernels/c3_x3.hip",
    "kernels/preprocess.hip",
    "kernels/stem_fused.hip",
    "kernels/detect.hip",
    "kernels/classify_head.hip",
    "kernels/head_pool.hip",
    "kernels/fc_splitk.hip",
    "kernels/jpeg_idct.hip",
    "runtime/executor.cpp",
    "runtime/batcher.cpp",
    "runtime/http_front.cpp",
    "runtime/http_loadgen.cpp",
    "runtime/ipc_buffer.cpp",
    "runtime/trace.cpp",
    "runtime/jpeg_decode.cpp",
    "runtime/jpeg_ingest.cpp",
    "runtime/kserve.cpp",
    "runtime/crash_trace.cpp",
    "bindings_jpeg.cpp",
    "bindings.cpp",
]


PER_FILE_FLAGS: dict[str, list[str]] = {}


def ext_path() -> Path:
    return PKG / ("_C" + sysconfig.get_config_var("EXT_SUFFIX"))


def _includes() -> list[str]:
    import pybind11

    return ["-I" + str(CSRC), "-I" + pybind11.get_include(), "-I" + sysconfig.get_paths()["include"]]


def _torch_lib() -> str | None:
    try:
        import importlib.util

        spec = importlib.util.find_spec("torch")
        if spec and spec.origin:
            return str(Path(spec.origin).parent / "lib")
    except Exception:  # pragma: no cover - torch is optional for the build
        pass
    return None


def _newest_header() -> float:
    hs = list(CSRC.rglob("*.h"))
    return max((h.stat().st_mtime for h in hs), default=0.0)


def compile_one(src: Path, obj: Path, extra: list[str], verbose: bool) -> str:
    obj.parent.mkdir(parents=True, exist_ok=True)
    cmd = [HIPCC, "-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-c", str(src), "-o", str(obj)]
    cmd += _includes() + extra
    if src.name in PER_FILE_FLAGS:
        cmd += PER_FILE_FLAGS[src.name]
    if src.suffix == ".cpp":
        # host-only translation units still go through hipcc (HIP runtime headers)
        cmd += ["-x", "hip"] if "bindings" not in src.name else []
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    return str(obj)


def build(force: bool = False, verbose: bool = False, jobs: int | None = None) -> Path:
    out = ext_path()
    newest_h = _newest_header()
    work = []
    objs = []
    for rel in SOURCES:
        src = CSRC / rel
        obj = OBJ / (rel.replace("/", "__") + ".o")
        objs.append(obj)
        if force or not obj.exists() or obj.stat().st_mtime < max(src.stat().st_mtime, newest_h):
            work.append((src, obj))
    extra = ["-Wno-unused-result"]
    jobs = jobs or min(8, os.cpu_count() or 4)
    if work:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            futs = [ex.submit(compile_one, s, o, extra, verbose) for s, o in work]
            for f in futs:
                f.result()
    if work or force or not out.exists() or out.stat().st_mtime < max(o.stat().st_mtime for o in objs):
        link = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", str(out)] + [str(o) for o in objs] + ["-ldl"]
        tl = _torch_lib()
        if tl:
            link += [f"-Wl,-rpath,{tl}"]
        if verbose:
            print(" ".join(link), flush=True)
        r = subprocess.run(link, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    a = ap.parse_args(argv)
    p = build(force=a.force, verbose=a.verbose, jobs=a.jobs)
    print(p)
    return 0


if __name__ == "__main__":
    sys.exit(main())
