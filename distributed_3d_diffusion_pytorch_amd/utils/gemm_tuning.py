"""Tuned library GEMMs (PyTorch TunableOp over hipBLASLt / rocBLAS).

The per-pixel dense layers that stay plain library GEMMs (the level-batched
FiLM projections, the attention in / out projections and NIN skips at large
per-GPU batch; ops/hip_impl.py) are dispatched by hipBLASLt's heuristic,
which does not always pick its fastest solution for these tall-skinny
shapes.  ``tools/tune_gemms.py`` benchmarks every candidate solution for
every GEMM shape of the training step on an MI355X and stores the winners in
``tuning/tunableop_mi355x.csv``; at start-up the trainer / bench load that
table read-only (TunableOp dispatches the recorded solution, no tuning at run
time, graph-capture safe).  The table carries TunableOp's validators (ROCm,
hipBLASLt and PyTorch versions, gfx arch): on any other stack it is ignored.
``D3D_TUNED_GEMMS=0`` turns the table off.
"""
from __future__ import annotations

import os
import shutil
import tempfile

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
TABLE = os.path.join(ROOT, "tuning", "tunableop_mi355x.csv")
_DONE = [False]


def enable_tuned_gemms(path: str = None) -> bool:
    """Load the tuned-solution table (once per process; ``path`` overrides
    the repository table).  Returns True when TunableOp is active with it."""
    path = path or TABLE
    if _DONE[0]:
        return torch.cuda.tunable.is_enabled()
    _DONE[0] = True
    if os.environ.get("D3D_TUNED_GEMMS", "1") == "0" or not torch.cuda.is_available() or not os.path.exists(path):
        return False
    tun = torch.cuda.tunable
    try:
        # work on a private copy: TunableOp may rewrite its results file at
        # exit, and the repository copy must stay what the tuning run produced
        tmp = os.path.join(tempfile.gettempdir(), f"d3d_tunableop_{os.getpid()}.csv")
        shutil.copyfile(path, tmp)
        tun.enable(True)
        tun.tuning_enable(False)
        tun.record_untuned_enable(False)
        tun.set_filename(tmp)
        ok = bool(tun.read_file(tmp))
    except Exception:                       # noqa: BLE001 -- a table problem must never stop training
        ok = False
    if not ok:
        tun.enable(False)
    return ok
