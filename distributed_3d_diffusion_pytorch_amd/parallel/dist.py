"""Process-group bootstrap: one process per GPU, RCCL over xGMI.

Reference: `train.py:181-196,307-319` hard-codes ``localhost:12355``, the
``gloo`` backend and ``mp.spawn`` (so torchrun's env is ignored and each
torchrun worker would spawn its own children, P2).  Here:

* torchrun / any launcher that exports ``RANK, WORLD_SIZE, LOCAL_RANK,
  MASTER_ADDR, MASTER_PORT`` is honoured;
* otherwise :func:`spawn` self-launches ``nprocs`` workers on 127.0.0.1;
* backend ``nccl`` (= RCCL on ROCm) for GPU tensors, ``gloo`` on CPU, with a
  finite timeout so a dead rank surfaces as an error instead of a hang;
* ``torch.cuda.set_device(local_rank)`` before anything touches the GPU (D4);
* RCCL hardening (:func:`rccl_env_defaults`): asynchronous error handling
  tears a rank down when a collective fails or exceeds the timeout (so the
  launcher's "one rank died" path ends the job instead of a silent hang), and
  the watchdog's heartbeat monitor dumps the flight recorder of a stuck rank.
"""
from __future__ import annotations

import datetime
import os
import socket
from dataclasses import dataclass
from typing import Callable, Optional

import torch
import torch.distributed as dist


@dataclass
class DistContext:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str = "none"

    @property
    def is_dist(self) -> bool:
        return self.world > 1

    @property
    def is_main(self) -> bool:
        return self.rank == 0


_CTX: Optional[DistContext] = None


def get_context() -> DistContext:
    return _CTX if _CTX is not None else DistContext()


def env_world() -> int:
    return int(os.environ.get("WORLD_SIZE", "1"))


def rccl_env_defaults() -> None:
    """Defaults for the ``nccl`` (= RCCL) process group, set before it is
    created; an explicit setting in the environment always wins.

    * ``TORCH_NCCL_ASYNC_ERROR_HANDLING=1``: a failed / timed-out collective
      aborts the communicator and raises in the rank instead of leaving the
      other ranks blocked inside RCCL kernels;
    * ``TORCH_NCCL_ENABLE_MONITORING=1`` with a heartbeat timeout above the
      collective timeout: a rank whose watchdog itself hangs is killed;
    * ``TORCH_NCCL_DUMP_ON_TIMEOUT=0``: no flight-recorder files in the repo;
    * ``TORCH_NCCL_CUDA_EVENT_CACHE=0``: every collective gets fresh events.
      With the cache, an event recorded by a collective CAPTURED into the graph
      step could be one the watchdog thread still queries for an eager work
      (warm-up / probe), and the query fails ("operation not permitted on an
      event last recorded in a capturing stream"), aborting the rank.
    """
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    os.environ.setdefault("TORCH_NCCL_ENABLE_MONITORING", "1")
    os.environ.setdefault("TORCH_NCCL_HEARTBEAT_TIMEOUT_SEC", "1200")
    os.environ.setdefault("TORCH_NCCL_DUMP_ON_TIMEOUT", "0")
    os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC (the only mode the host driver has)


def init_distributed(backend: str = "auto", timeout_s: float = 600.0, use_gpu: Optional[bool] = None
                     ) -> DistContext:
    """Initialise from the environment (torchrun-compatible).  Single-process
    runs (no WORLD_SIZE or WORLD_SIZE=1) get a trivial context and no group."""
    global _CTX
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    if use_gpu is None:
        use_gpu = torch.cuda.device_count() > 0
    if use_gpu:
        ndev = torch.cuda.device_count()
        torch.cuda.set_device(local_rank % max(ndev, 1))
        device = torch.device("cuda", torch.cuda.current_device())
    else:
        device = torch.device("cpu")
    if backend == "auto":
        backend = "nccl" if use_gpu else "gloo"
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29512")
        kw = dict(backend=backend, rank=rank, world_size=world,
                  timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            rccl_env_defaults()
            kw["device_id"] = device        # eager communicator creation (no lazy init inside graph capture)
        dist.init_process_group(**kw)
    _CTX = DistContext(rank, world, local_rank, device, backend if world > 1 else "none")
    return _CTX


def cleanup() -> None:
    global _CTX
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
    _CTX = None


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawn_entry(local_rank: int, fn: Callable, world: int, port: int, args: tuple) -> None:
    os.environ.update(RANK=str(local_rank), LOCAL_RANK=str(local_rank), WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    fn(*args)


def spawn(fn: Callable, nprocs: int, args: tuple = ()) -> None:
    """Self-launch ``nprocs`` ranks on this node (reference ``run``,
    `train.py:189-193`), rendezvous on 127.0.0.1.  ``fn(*args)`` reads its rank
    from the environment like a torchrun worker."""
    import torch.multiprocessing as mp
    port = free_port()
    mp.spawn(_spawn_entry, args=(fn, nprocs, port, args), nprocs=nprocs, join=True)


def barrier() -> None:
    if dist.is_available() and dist.is_initialized():
        dist.barrier()


def all_reduce_max(value: float, device=None) -> float:
    if not (dist.is_available() and dist.is_initialized()):
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
