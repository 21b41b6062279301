"""Checkpoint I/O compatible with the reference layout.

Reference format: ``torch.save({'optim': Adam.state_dict(), 'model':
model.state_dict(), 'step': int[, 'epoch': int]})`` into ``<dir>/after_warmup.pt``
(every 50 steps) and ``<dir>/latest.pt`` (`train.py:288-298`); resume reads
``<transfer>/latest.pt`` (`train.py:238-251`).  Published weights carry a
``module.`` prefix (DataParallel, `sampling.py:52-56`) while ``train.py`` saves
without it (D5).

Here: same file names and top-level keys (plus optional ``ema``, ``rng``,
``config``, ``world_size``); writes are rank-0, atomic (tmp + fsync + rename);
loads use ``weights_only=True`` (no code execution) and accept either prefix
convention; parameters stay in the reference OIHW / [out,in] shapes on disk.
"""
from __future__ import annotations

import os
import tempfile
from typing import Any, Dict, Optional

import torch


def strip_prefix(sd: Dict[str, torch.Tensor], prefix: str = "module.") -> Dict[str, torch.Tensor]:
    if sd and all(k.startswith(prefix) for k in sd):
        return {k[len(prefix):]: v for k, v in sd.items()}
    return dict(sd)


def add_prefix(sd: Dict[str, torch.Tensor], prefix: str = "module.") -> Dict[str, torch.Tensor]:
    return {(k if k.startswith(prefix) else prefix + k): v for k, v in sd.items()}


def atomic_save(obj: Any, path: str) -> None:
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    fd, tmp = tempfile.mkstemp(prefix=".tmp_ckpt_", dir=d)
    try:
        with os.fdopen(fd, "wb") as f:
            torch.save(obj, f)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, path)
    except BaseException:
        if os.path.exists(tmp):
            os.unlink(tmp)
        raise


def model_state_cpu(model: torch.nn.Module) -> Dict[str, torch.Tensor]:
    # clone: parameters are views of the flat buffer; saving a view would
    # serialise the whole underlying storage
    return {k: v.detach().to("cpu", copy=True) for k, v in model.state_dict().items()}


def save_checkpoint(path: str, model: torch.nn.Module, optimizer=None, step: int = 0,
                    epoch: Optional[int] = None, extra: Optional[Dict[str, Any]] = None) -> None:
    ck: Dict[str, Any] = {"model": model_state_cpu(model), "step": int(step)}
    if optimizer is not None:
        osd = optimizer.state_dict()
        for s in osd.get("state", {}).values():
            for k, v in list(s.items()):
                if torch.is_tensor(v):
                    s[k] = v.detach().cpu()
        ck["optim"] = osd
    if epoch is not None:
        ck["epoch"] = int(epoch)
    if extra:
        ck.update(extra)
    atomic_save(ck, path)


def load_checkpoint(path: str, map_location="cpu") -> Dict[str, Any]:
    return torch.load(path, map_location=map_location, weights_only=True)


def load_model_weights(model: torch.nn.Module, sd: Dict[str, torch.Tensor], strict: bool = True):
    """Load a (possibly ``module.``-prefixed) state dict IN PLACE, preserving
    the flat-buffer views the parameters live in."""
    sd = strip_prefix(sd)
    own = model.state_dict()
    missing = [k for k in own if k not in sd]
    unexpected = [k for k in sd if k not in own]
    if strict and (missing or unexpected):
        raise KeyError(f"state_dict mismatch: missing={missing[:5]} unexpected={unexpected[:5]}")
    with torch.no_grad():
        for k, v in own.items():
            if k in sd:
                if tuple(sd[k].shape) != tuple(v.shape):
                    raise ValueError(f"shape mismatch for {k}: {tuple(sd[k].shape)} vs {tuple(v.shape)}")
                v.copy_(sd[k])
    return missing, unexpected


def find_resume(transfer: str) -> Optional[str]:
    """``--transfer DIR`` resumes from ``DIR/latest.pt`` (reference), else the
    newest valid of ``latest.pt`` / ``after_warmup.pt``; a file path is used as is."""
    if not transfer:
        return None
    if os.path.isfile(transfer):
        return transfer
    cands = [os.path.join(transfer, n) for n in ("latest.pt", "after_warmup.pt")]
    cands = [c for c in cands if os.path.isfile(c)]
    if not cands:
        return None
    best, best_step = None, -1
    for c in cands:
        try:
            s = int(load_checkpoint(c).get("step", -1))
        except Exception:
            continue
        if s > best_step:
            best, best_step = c, s
    return best
