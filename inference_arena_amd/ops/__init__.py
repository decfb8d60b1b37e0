"""Loader for the native extension ``inference_arena_amd._C`` (HIP/gfx950).

torch is imported first on purpose: PyTorch-ROCm ships its own
``libamdhip64.so.7`` and the extension resolves the HIP runtime by SONAME, so
both share one runtime (and one device allocator view).  ``native()`` raises
loudly when the extension is missing so GPU code paths never fall back to an
eager PyTorch implementation silently.
"""
from __future__ import annotations

import importlib
import os
from types import ModuleType

import torch  # noqa: F401  (must precede the extension import)

_mod: ModuleType | None = None
_err: Exception | None = None


def build_ext(force: bool = False):
    """Compile the extension in-tree with hipcc (tools/build_ext.py)."""
    import importlib.util
    from pathlib import Path

    path = Path(__file__).resolve().parents[2] / "tools" / "build_ext.py"
    spec = importlib.util.spec_from_file_location("_arena_build_ext", path)
    mod = importlib.util.module_from_spec(spec)
    assert spec.loader is not None
    spec.loader.exec_module(mod)
    return mod.build(force=force)


def native() -> ModuleType:
    global _mod, _err
    if _mod is not None:
        return _mod
    try:
        _mod = importlib.import_module("inference_arena_amd._C")
    except ImportError as e:
        if os.environ.get("ARENA_AUTOBUILD", "1") == "1":
            build_ext()
            _mod = importlib.import_module("inference_arena_amd._C")
        else:
            _err = e
            raise RuntimeError(
                "inference_arena_amd native extension is not built; run `python tools/build_ext.py` "
                f"(import error: {e})"
            ) from e
    return _mod


def available() -> bool:
    try:
        native()
        return True
    except Exception:  # noqa: BLE001
        return False
