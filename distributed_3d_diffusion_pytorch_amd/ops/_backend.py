"""Backend selection and native-library loading.

The native library (``libd3d_hip.so``) is built in-tree by ``tools/build_native.py``
with ``hipcc --offload-arch=gfx950``.  It is a plain HIP shared object with a C
ABI (no torch headers, no hipify): Python passes raw device pointers, shapes and
the current HIP stream handle through ctypes.

Policy:
  * ``D3D_BACKEND=hip|torch|auto`` (default auto).
  * auto -> ``hip`` for GPU tensors when the library loads, ``torch`` on CPU.
  * On a machine with a GPU, a missing/unloadable library is an ERROR unless
    ``D3D_ALLOW_TORCH_FALLBACK=1`` -- GPU runs must never silently fall back.
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

import torch

_LIB: Optional[ctypes.CDLL] = None
_LIB_ERR: Optional[str] = None
_LOCK = threading.Lock()
_FORCED: Optional[str] = None

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("D3D_LIB_PATH") or os.path.join(PKG_DIR, "ops", "libd3d_hip.so")   # override: A/B builds


def lib_path() -> str:
    return LIB_PATH


def load_library(required: bool = False) -> Optional[ctypes.CDLL]:
    """Load the in-tree HIP library once (torch must already be imported so
    its HIP runtime -- SONAME libamdhip64.so.7 -- is the one we bind to)."""
    global _LIB, _LIB_ERR
    if _LIB is not None:
        return _LIB
    with _LOCK:
        if _LIB is not None:
            return _LIB
        if not os.path.exists(LIB_PATH):
            _LIB_ERR = f"native library not built: {LIB_PATH} (run python tools/build_native.py)"
        else:
            try:
                lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
                from . import _abi
                _abi.declare(lib)
                _LIB = lib
            except OSError as e:  # pragma: no cover - depends on the box
                _LIB_ERR = f"failed to load {LIB_PATH}: {e}"
    if _LIB is None and required:
        raise RuntimeError(_LIB_ERR)
    return _LIB


def library_error() -> Optional[str]:
    return _LIB_ERR


def set_backend(name: Optional[str]) -> None:
    """Force a backend for subsequent ops ('hip', 'torch' or None=auto)."""
    global _FORCED
    if name not in (None, "auto", "hip", "torch"):
        raise ValueError(name)
    _FORCED = None if name in (None, "auto") else name


def get_forced() -> Optional[str]:
    if _FORCED is not None:
        return _FORCED
    env = os.environ.get("D3D_BACKEND", "auto").lower()
    return None if env == "auto" else env


def use_hip(t: torch.Tensor, any_dtype: bool = False) -> bool:
    """Decide the backend for an op whose main input is ``t``.  The HIP
    activation kernels are bf16-only (the MI355X compute dtype); fp32 GPU
    runs use the torch composition unless ``any_dtype`` (fp32 buffers such as
    the optimizer state or camera matrices)."""
    forced = get_forced()
    if t.is_cuda and not any_dtype and t.dtype != torch.bfloat16:
        return False
    if forced == "torch" or not t.is_cuda:
        if forced == "hip" and not t.is_cuda:
            raise RuntimeError("D3D_BACKEND=hip but tensor is on CPU")
        return False
    lib = load_library(required=False)
    if lib is None:
        if forced == "hip" or os.environ.get("D3D_ALLOW_TORCH_FALLBACK", "0") != "1":
            raise RuntimeError(
                "HIP backend requested/required on a GPU but the native library is "
                f"unavailable: {_LIB_ERR}. Set D3D_ALLOW_TORCH_FALLBACK=1 to use torch ops.")
        return False
    return True


def stream_handle(device: Optional[torch.device] = None) -> int:
    return torch.cuda.current_stream(device).cuda_stream
