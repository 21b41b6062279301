"""Observability: rank-0 JSONL metrics, step timer with examples/s and
achieved TFLOP/s, roctx ranges, NaN/Inf guards.

Reference: ``print("Loss:", loss.item())`` every 50 steps and tqdm bars
(`train.py:264,284-285`); tensorboardX imported but unused (U1)."""
from __future__ import annotations

import contextlib
import json
import math
import os
import time
from typing import Any, Dict, Optional

import torch

# fwd+bwd FLOPs per training example (one 2-view pair), measured from the
# reference model definition: 707.6 GF @64^2, 2907.8 @128^2.
_FLOPS_FB = {64: 707.6e9, 128: 2907.8e9}


def train_flops_per_example(imgsize: int) -> float:
    if imgsize in _FLOPS_FB:
        return _FLOPS_FB[imgsize]
    return _FLOPS_FB[64] * (imgsize / 64.0) ** 2


class MetricsLogger:
    def __init__(self, path: Optional[str], enabled: bool = True):
        self.enabled = enabled and bool(path)
        self.f = None
        if self.enabled:
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
            self.f = open(path, "a", buffering=1)

    def log(self, **kw: Any) -> None:
        if not self.enabled:
            return
        kw.setdefault("time", time.time())
        self.f.write(json.dumps(kw, default=float) + "\n")

    def close(self) -> None:
        if self.f:
            self.f.close()
            self.f = None


class StepTimer:
    """Wall-clock throughput over a window of steps (device-synchronised at
    window boundaries only)."""

    def __init__(self, examples_per_step: int, flops_per_example: float, device=None):
        self.eps = examples_per_step
        self.fpe = flops_per_example
        self.device = device
        self.t0 = None
        self.n = 0

    def _sync(self):
        if self.device is not None and torch.device(self.device).type == "cuda":
            torch.cuda.synchronize(self.device)

    def start(self):
        self._sync()
        self.t0 = time.perf_counter()
        self.n = 0

    def tick(self):
        self.n += 1

    def report(self) -> Dict[str, float]:
        self._sync()
        dt = time.perf_counter() - self.t0
        ex = self.n * self.eps
        out = {"steps": self.n, "seconds": dt, "examples_per_s": ex / dt if dt > 0 else float("nan"),
               "ms_per_step": 1e3 * dt / max(self.n, 1)}
        out["tflops"] = out["examples_per_s"] * self.fpe / 1e12
        return out


@contextlib.contextmanager
def range_push(name: str):
    """roctx range (shows in rocprofv3 --marker-trace) when available."""
    pushed = False
    try:
        if torch.cuda.is_available():
            torch.cuda.nvtx.range_push(name)
            pushed = True
    except Exception:
        pushed = False
    try:
        yield
    finally:
        if pushed:
            torch.cuda.nvtx.range_pop()


def check_finite(loss: torch.Tensor, step: int) -> None:
    v = float(loss)
    if not math.isfinite(v):
        raise FloatingPointError(f"non-finite loss {v} at step {step}")
