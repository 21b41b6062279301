"""Data-parallel gradient engine: bucketed RCCL all-reduce overlapped with
backward.

Reference behaviour: ``DDP(model)`` is constructed (`train.py:230-233`) but the
loss is computed through the raw module (`train.py:275`), so the gradient
all-reduce never fires and replicas diverge (D2); comm is ``gloo`` through host
memory, and every step ends in a barrier (D8).

Design here (MI355X, 8 GPUs on xGMI, 7 point-to-point links per GPU):

* gradients are views of one flat fp32 buffer laid out in backward order
  (:class:`.flat.FlatParams`), so a bucket is a contiguous slice that RCCL
  reduces in place -- no flatten copies;
* buckets default to 64 MiB with a small first bucket: big enough that RCCL's
  rings over the 7 links each carry >=0.5 MiB chunks, few enough (≈9 over the
  521 MiB model) that per-collective latency is negligible, and the small first
  bucket starts communication early in backward;
* each bucket is launched from a post-accumulate-grad hook the moment its last
  gradient lands, on RCCL's own stream (``async_op``), so reduction overlaps the
  rest of backward; ``finish()`` makes the compute stream wait on the handles;
* averaging is folded into the optimizer (``grad_scale = 1/world``) -- no
  separate divide pass;
* optional bf16 payload halves link traffic: each bucket is narrowed into a
  persistent bf16 mirror on the collective's stream, reduced there, and
  widened back by ``finish()`` -- no allocation per step, so the same code
  runs eagerly and captured in the graph step (engine/graphs.py).
"""
from __future__ import annotations

import contextlib
import os
from typing import List, Optional

import torch
import torch.distributed as dist

from .flat import FlatParams


# diagnostic (tools/diag_flush_nan.py): the race probe snapshots each bucket but
# the collective reduces the bucket in place, as without the probe
_PROBE_COPY_ONLY = os.environ.get("D3D_DIAG_PROBE_COPY_ONLY", "0") == "1"


class GradReducer:
    def __init__(self, flat: FlatParams, bucket_mb: float = 64.0, first_bucket_mb: float = 4.0,
                 grad_dtype: str = "fp32", group=None, force: bool = False):
        self.flat = flat
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        # collectives run at world > 1, or when forced (tests: a 1-rank RCCL
        # group runs the full multi-GPU step topology on one GPU)
        self.active = self.world > 1 or (force and dist.is_initialized())
        self.grad_dtype = torch.bfloat16 if grad_dtype == "bf16" else torch.float32
        self.mirror = (torch.empty(flat.grad.numel(), dtype=torch.bfloat16, device=flat.grad.device)
                       if self.grad_dtype != torch.float32 and self.active else None)
        self.enabled = True
        # buckets over the backward-ordered layout
        self.buckets: List[dict] = []
        cur: Optional[dict] = None
        limit = first_bucket_mb * 2 ** 20
        for i in flat.order:
            s, e = flat.span(i)
            if cur is None:
                cur = {"start": s, "end": e, "params": [i]}
            else:
                cur["end"] = e
                cur["params"].append(i)
            if (cur["end"] - cur["start"]) * 4 >= limit:
                self.buckets.append(cur)
                cur = None
                limit = bucket_mb * 2 ** 20
        if cur is not None:
            self.buckets.append(cur)
        self.param_bucket = {}
        for b, bk in enumerate(self.buckets):
            for i in bk["params"]:
                self.param_bucket[i] = b
        self.sink = None            # ops.gradsink.GradSink delivering kernel-deposited grads
        # segmented graph capture (engine/graphs.py comm_mode "seg"): a ready
        # bucket is handed to seg_cut(b, cut) instead of being reduced here --
        # the capture is split at that point and the bucket's collective is
        # issued eagerly between the segment replays
        self.seg_cut = None
        self._pending = [0] * len(self.buckets)
        self._launched = [False] * len(self.buckets)
        self._works: List = []
        self._tmp = {}
        # bucket issue order of the last step (captured mode: compared over the
        # group after the capture, engine/graphs.py)
        self.issue_log: List[int] = []
        # test-only race probe (1-rank groups, enable_race_probe): (snapshots, final)
        self.race_probe = None
        self._hooks = []
        for i, p in enumerate(flat.params):
            if p.requires_grad:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(i)))
        self.reset()

    # ------------------------------------------------------------------
    def reset(self) -> None:
        # the stream this step's backward runs its trunk on (the capture stream inside a graph capture)
        self.main_stream = torch.cuda.current_stream() if self.flat.grad.is_cuda else None
        for b, bk in enumerate(self.buckets):
            self._pending[b] = sum(1 for i in bk["params"] if self.flat.params[i].requires_grad)
            self._launched[b] = False
        self._works = []
        self.issue_log = []

    def enable_race_probe(self) -> None:
        """Test-only (1-rank group): every collective reduces a SNAPSHOT of its
        bucket taken on the collective's stream at issue time, and its result
        is discarded (a 1-rank sum is the identity), so the real gradient is
        never overwritten by the collective.  ``finish()`` copies the complete
        gradient into ``race_probe[1]``: a collective issued before a deposit
        into its bucket landed shows as a snapshot that differs from it, for
        fp32 and bf16 payloads alike (with the in-place reduction a premature
        read is invisible on one rank: the write-back restores what was read)."""
        assert self.world == 1, "race probe: 1-rank groups only"
        n = self.flat.grad.numel()
        self.race_probe = (torch.zeros(n, device=self.flat.grad.device),
                           torch.zeros(n, device=self.flat.grad.device))

    def probe_src(self, b: int, view: torch.Tensor) -> torch.Tensor:
        """The tensor bucket b's collective reduces: the bucket itself, or its
        race-probe snapshot (copied on the current stream)."""
        if self.race_probe is None:
            return view
        bk = self.buckets[b]
        snap = self.race_probe[0][bk["start"]: bk["end"]]
        snap.copy_(view)
        if _PROBE_COPY_ONLY:
            return view         # diagnostic: snapshot taken, the collective still reduces in place
        return snap

    def probe_final(self) -> None:
        if self.race_probe is not None:
            self.race_probe[1].copy_(self.flat.grad)

    def _make_hook(self, i: int):
        def hook(p):
            if self.sink is not None and self.sink.was_used(p):
                return          # the sink reports this parameter itself
            self.mark_ready(i)
        return hook

    def mark_ready(self, i: int) -> None:
        """Parameter i's gradient is complete in the flat buffer (called by the
        autograd hook, or by the HIP gradient sink for kernel-deposited grads)."""
        if not self.enabled or not self.active:
            return
        b = self.param_bucket[i]
        self._pending[b] -= 1
        if self._pending[b] == 0:
            self._launch(b)

    def completes_bucket(self, params) -> bool:
        """True when reporting parameters ``params`` (indices) would complete
        a bucket not yet launched (the sink's bucket-aware flush)."""
        if not self.enabled or not self.active:
            return False
        cnt = {}
        for i in params:
            b = self.param_bucket[i]
            cnt[b] = cnt.get(b, 0) + 1
        return any(not self._launched[b] and self._pending[b] <= c for b, c in cnt.items())

    def _launch(self, b: int) -> None:
        if self._launched[b]:
            return
        self._launched[b] = True
        if self.seg_cut is not None:
            self.seg_cut(b, True)
            return
        self.issue_log.append(b)
        bk = self.buckets[b]
        view = self.flat.grad[bk["start"]: bk["end"]]
        ctx = self.sink.collective(self.main_stream) if self.sink is not None else contextlib.nullcontext()
        with ctx:       # behind the sink's weight-gradient stream (ops/gradsink.py)
            src = self.probe_src(b, view)
            back = view if src is view else None                    # probe: the result is discarded
            if self.mirror is None:
                self._works.append((dist.all_reduce(src, group=self.group, async_op=True), None, None))
            else:
                tmp = self.mirror[bk["start"]: bk["end"]]
                tmp.copy_(src)                                      # narrow on the collective's stream
                self._works.append((dist.all_reduce(tmp, group=self.group, async_op=True), tmp, back))

    def finish(self) -> None:
        """Launch any bucket whose gradients never arrived (unused params) and
        make the current stream wait for every reduction."""
        if self.sink is not None:
            self.sink.join()
        if not self.active or not self.enabled:
            self.reset()
            return
        if self.seg_cut is not None:
            # the remaining buckets belong to the last segment (no cut after it)
            for b in range(len(self.buckets)):
                if not self._launched[b]:
                    self._launched[b] = True
                    self.seg_cut(b, False)
            self.reset()
            return
        for b in range(len(self.buckets)):
            if not self._launched[b]:
                self._launch(b)
        if self.sink is not None:
            # collectives issued above from behind the weight-gradient stream:
            # rejoin it (also a graph capture's end-of-capture join)
            self.sink.join()
        for w, tmp, view in self._works:
            w.wait()
            if tmp is not None and view is not None:
                view.copy_(tmp)                                     # widen (persistent mirror: no recycling)
        self.probe_final()
        log = self.issue_log
        self.reset()
        self.issue_log = log

    def describe(self) -> dict:
        """Bucket layout and payload, for benchmark / metrics records."""
        sizes = [(bk["end"] - bk["start"]) * 4 / 2 ** 20 for bk in self.buckets]
        return {"active": bool(self.active), "world_pg": int(self.world), "buckets": len(self.buckets),
                "bucket_mib": [round(x, 2) for x in sizes], "total_mib": round(sum(sizes), 2),
                "payload": "bf16" if self.grad_dtype == torch.bfloat16 else "fp32"}

    @contextlib.contextmanager
    def no_sync(self):
        """Gradient accumulation: skip communication inside the block."""
        prev = self.enabled
        self.enabled = False
        try:
            yield
        finally:
            self.enabled = prev

    def broadcast_params(self, src: int = 0) -> None:
        if self.active:
            dist.broadcast(self.flat.data, src, group=self.group)

    def remove_hooks(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []


def param_checksum(flat: FlatParams) -> torch.Tensor:
    """Order-sensitive fp64 fingerprint of the flat parameters."""
    d = flat.data.double()
    w = torch.linspace(1.0, 2.0, d.numel(), dtype=torch.float64, device=d.device)
    return torch.stack([d.sum(), (d * w).sum(), d.abs().max()])


def check_replicas_in_sync(flat: FlatParams, group=None, rtol: float = 0.0) -> bool:
    """Divergence detector (catches D2-class bugs): compares every rank's
    fingerprint against rank 0's.  Returns True when all ranks agree."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return True
    c = param_checksum(flat)
    hi, lo = c.clone(), c.clone()
    dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=group)
    dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=group)
    tol = rtol * hi.abs().clamp_min(1e-30)
    return bool(((hi - lo).abs() <= tol).all().item())
