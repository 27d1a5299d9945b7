"""Loader for the in-tree native extension ``_C.so`` (HIP kernels, torch.ops.tdc.*).

On a GPU host the native path is mandatory unless the caller explicitly asks for
``backend="torch"``: :func:`require` raises instead of silently falling back to
PyTorch ops, so a missing/stale build shows up as an error, not as a slow run.
"""
from __future__ import annotations

import os
import threading
from pathlib import Path

import torch

_LIB = Path(__file__).resolve().parent / "_C.so"
_lock = threading.Lock()
_state = {"loaded": False, "error": None}


def lib_path() -> Path:
    return _LIB


def load(build_if_missing: bool = False) -> bool:
    """Load ``_C.so`` once; returns True on success."""
    with _lock:
        if _state["loaded"]:
            return True
        if not _LIB.exists() and build_if_missing:
            try:
                from .runtime.build import build
                build(verbose=False)
            except Exception as e:  # pragma: no cover - build env specific
                _state["error"] = f"build failed: {e}"
                return False
        if not _LIB.exists():
            _state["error"] = f"{_LIB} not built (run python -m tensorflow_distributed_clustering_amd.runtime.build)"
            return False
        try:
            torch.ops.load_library(str(_LIB))
            _state["loaded"] = True
            _state["error"] = None
        except Exception as e:
            _state["error"] = f"failed to load {_LIB}: {e}"
            return False
        return True


def available() -> bool:
    return load(build_if_missing=os.environ.get("TDC_AUTOBUILD", "0") == "1")


def error() -> str:
    return _state["error"] or ""


def require():
    """Return ``torch.ops.tdc`` or raise (fail loudly on a GPU box with no extension)."""
    if not available():
        raise RuntimeError("tdc native extension unavailable: " + error())
    return torch.ops.tdc


def ops():
    return require()
