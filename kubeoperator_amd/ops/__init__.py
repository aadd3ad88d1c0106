"""gfx950 HIP kernels of kubeoperator_amd and their autograd wrappers.

``load()`` returns the compiled extension module (``kubeoperator_amd/_C.so``). On a machine with a GPU the
extension is REQUIRED: if it is missing it is built in-tree with hipcc, and if that fails the error
propagates -- there is deliberately no silent eager-PyTorch fallback on the GPU path. The pure-PyTorch
fp32 references in :mod:`kubeoperator_amd.ops.reference` exist for numerics tests and for CPU-only
plumbing tests (``KOP_ALLOW_REFERENCE=1`` or no GPU present).
"""
from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_lib = None


def load():
    """Import (building first if needed) the gfx950 extension module."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        import torch  # noqa: F401  (loads libc10/libtorch/libamdhip64 before our .so)

        from . import _build

        alt = os.environ.get("KOP_EXT_MODULE")  # A/B runs: a second build of the kernels (tools/build_ab.py)
        if alt:
            _lib = importlib.import_module(f"kubeoperator_amd.{alt}")
            return _lib
        if not os.path.exists(_build.SO_PATH) or os.environ.get("KOP_REBUILD") == "1":
            _build.build()
        _lib = importlib.import_module("kubeoperator_amd._C")
        return _lib


def native_available() -> bool:
    try:
        load()
        return True
    except Exception:
        return False


def use_native(t=None) -> bool:
    """True when an op on tensor ``t`` must run the HIP kernel (i.e. it lives on the GPU)."""
    if t is not None and not t.is_cuda:
        return False
    return True


from .functional import (  # noqa: E402
    cross_entropy_lmhead,
    embedding,
    flash_attention,
    gelu,
    layer_norm,
    linear,
    rms_norm,
    rope_attention,
    swiglu,
)
from .optim import FusedAdamW  # noqa: E402

__all__ = [
    "load",
    "native_available",
    "rms_norm",
    "layer_norm",
    "linear",
    "embedding",
    "swiglu",
    "gelu",
    "flash_attention",
    "rope_attention",
    "cross_entropy_lmhead",
    "FusedAdamW",
]
