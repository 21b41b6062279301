"""Direct parameter-gradient sink.

With the flat gradient buffer (parallel/flat.py) every parameter gradient has
a fixed home.  When the sink is enabled, the weight-gradient kernels deposit
(accumulate) straight into that home and the autograd Function returns
``None`` for the parameter, so PyTorch runs no AccumulateGrad add kernel and
allocates no temporary gradient tensor.  Because autograd then never sees
those gradients, the sink tracks how many uses of each parameter the current
forward made and tells the data-parallel reducer when the last one has been
deposited (a parameter can be used more than once, e.g. the conditioning
convs run on the rays and on the learned-embedding image).

Weight-gradient stream.  A deposited weight gradient has no consumer until the
all-reduce / optimizer, so :meth:`GradSink.producer` runs it on a second HIP
stream: the compute stream goes straight on to the next layer's input
gradient (the critical path of backward) while the weight-gradient GEMMs and
their split-K reductions fill the CUs it leaves idle -- at 16 examples per GPU
most backward launches cover well under the 256 CUs.  The side stream first
waits for the compute stream (its operands are ready), the operands are
``record_stream``-ed so the caching allocator cannot hand their memory to the
compute stream early (during graph capture such frees are deferred to the end
of the capture), and an end-of-backward autograd callback joins the side
stream back into the caller's stream, so optimizers, graph capture and tests
see the same ordering as a single stream.  Collectives over the deposited
gradients are issued from behind the side stream (:meth:`collective`).
Per-parameter accumulation order is unchanged (one side stream, launch
order), so results stay bitwise reproducible.  ``D3D_WGRAD_STREAM=0`` runs
everything on the compute stream.

Inside HIP-graph capture (:meth:`submit`): a fork
per weight gradient cost ~7 us of graph dependency latency per edge -- ~1,600
edges ate the concurrency (busy 88.7 %, profiles/busy_bs16_side_stream.txt).
There the weight-gradient jobs are DEFERRED instead: queued as closures and
flushed onto the side stream 8 at a time (4 measured 1.5 % slower at bs16)
behind ONE fork each, and joined once at the end of backward, so the graph
holds a few dozen cross-stream edges while the weight-gradient branch runs
concurrently with the input-gradient chain.  Deferred operands stay alive in
the closures; the allocator defers frees of side-stream-recorded blocks to
the end of the capture.
"""
from __future__ import annotations

import contextlib
import os
from typing import Callable, Dict, Optional

import torch


_PRIO = 0          # HIP stream priority of the weight-gradient stream (higher measured slower)
# diagnostic switch (never set in training): collectives wait only for the
# issuing stream, as before the round-5 / round-6 ordering fixes -- used to
# confirm what the race probe catches (tools/diag_bucket_flush_race.py)
_DIAG_NO_STREAM_WAITS = os.environ.get("D3D_DIAG_SINK_NO_STREAM_WAITS", "0") == "1"


class GradSink:
    def __init__(self) -> None:
        self.enabled = False
        self.owners: Dict[int, torch.Tensor] = {}
        self.views: Dict[int, torch.Tensor] = {}
        self.index: Dict[int, int] = {}
        self.uses: Dict[int, int] = {}
        self.seen = set()
        self.notify: Optional[Callable[[int], None]] = None
        self.stream_enabled = os.environ.get("D3D_WGRAD_STREAM", "1") != "0"
        self.graph_defer = True      # weight gradients on the side stream inside graph capture too
        # jobs per fork (4 measured 1.5 % slower at bs16; D3D_WGRAD_DEFER_BATCH for A/B)
        self.defer_batch = int(os.environ.get("D3D_WGRAD_DEFER_BATCH", "8"))
        # eager steps: queue the grouped-kernel jobs too and flush them 8 at a
        # time (one grouped launch each) instead of one launch pair per job
        # (default "2": eager jobs run immediately, each as a one-job grouped
        # launch -- the 128x128 grouped tile with its planner beat the per-job
        # split-K kernels at bs128, 965 -> 973 examples/s; "1" (deferred
        # batches of 8 in eager steps) measured 940, "0" keeps the per-job
        # kernels: profiles/r4/b128_eager_ab.txt)
        mode = os.environ.get("D3D_WGRAD_EAGER_GROUP", "2")
        self.eager_group = mode == "1"
        self.eager_single = mode == "2"
        self._queue = []
        self._compute = []
        self._streams: Dict[int, "torch.cuda.Stream"] = {}
        self._forked = set()
        self._cb_queued = False
        # grouped weight-gradient launcher (set by ops.hip_impl): runs a
        # flush's job descriptors as one launch + one slab reduce
        self.group_fn: Optional[Callable[[list], None]] = None
        # bucket-aware flushing (set by the trainer, D3D_WGRAD_BUCKET_FLUSH):
        # called with the parameter indices a flush of the queue would
        # complete; True = that completes an all-reduce bucket, flush now
        # instead of waiting for defer_batch jobs
        self.bucket_flush: Optional[Callable[[list], bool]] = None
        self._qcount: Dict[int, int] = {}
        # work-based flushing: a queue holding at least this many weight-
        # gradient FLOPs is flushed at once (0: by job count only), so a few
        # big jobs (the 64x64 level's convs) start early while the many small
        # ones still share forks and grouped launches
        self.defer_work = float(os.environ.get("D3D_WGRAD_DEFER_GFLOP", "0")) * 1e9
        self._qwork = 0.0

    def attach(self, params, views, notify: Optional[Callable[[int], None]] = None) -> None:
        # the parameter objects themselves are kept: a key is only trusted
        # when it still names the same object (ids are reused once a model
        # that attached earlier is gone)
        self.owners = {id(p): p for p in params}
        self.views = {id(p): v for p, v in zip(params, views)}
        self.index = {id(p): i for i, p in enumerate(params)}
        self.uses = {}
        self.notify = notify
        self.enabled = True

    def detach(self) -> None:
        self.enabled = False
        self.views, self.index, self.uses, self.notify, self.owners = {}, {}, {}, None, {}

    def managed(self, p) -> bool:
        return self.enabled and p is not None and self.owners.get(id(p)) is p

    def target(self, p) -> Optional[torch.Tensor]:
        if not self.managed(p):
            return None
        return self.views[id(p)]

    def use(self, p, needed: bool = True) -> None:
        """Count one forward use of p.  Call from autograd.Function.forward
        with ``needed = ctx.needs_input_grad[...]`` (grad mode is always off
        inside Function.forward, so it cannot be queried there)."""
        if needed and self.managed(p) and p.requires_grad:
            k = id(p)
            self.uses[k] = self.uses.get(k, 0) + 1
            self.seen.add(k)

    def was_used(self, p) -> bool:
        """True when this step's gradient of p is delivered by the sink."""
        return self.enabled and id(p) in self.seen and self.owners.get(id(p)) is p

    def done(self, p) -> None:
        if not self.managed(p):
            return
        k = id(p)
        n = self.uses.get(k, 1) - 1
        self.uses[k] = n
        if n == 0 and self.notify is not None:
            self.notify(self.index[k])

    # ------------------------------------------------ weight-gradient stream
    def _side(self, idx: int):
        st = self._streams.get(idx)
        if st is None:
            # (a higher-priority queue, to keep the weight-gradient work in
            # pace with the input-gradient chain, measured slower)
            st = self._streams[idx] = torch.cuda.Stream(device=idx, priority=_PRIO)
        return st

    @contextlib.contextmanager
    def producer(self, dev: torch.device, *keep):
        """Run the enclosed sink-depositing work on the side stream (see the
        module doc).  ``keep``: tensors the work reads that autograd may free
        right after the enclosing backward returns."""
        if not (self.stream_enabled and dev.type == "cuda") or torch.cuda.is_current_stream_capturing():
            if self._compute and dev.type == "cuda":
                # no side stream, but deposits may come from a registered
                # compute stream (the conditioning stream): the end-of-backward
                # join must still make the optimizer's stream wait for it
                self._queue_end_callback()
            yield
            return
        idx = dev.index if dev.index is not None else torch.cuda.current_device()
        side = self._side(idx)
        side.wait_stream(torch.cuda.current_stream(idx))
        with torch.cuda.stream(side):
            yield
        for t in keep:
            if t is not None:
                t.record_stream(side)
        self._forked.add(idx)
        if not self._cb_queued:
            try:
                torch.autograd.Variable._execution_engine.queue_callback(self._end_of_backward)
                self._cb_queued = True
            except RuntimeError:        # not inside a backward pass: join now
                self.join()

    def add_compute_stream(self, st) -> None:
        """Register another stream that runs forward / backward work (the
        model's conditioning stream): collectives wait for it as well, and
        the end-of-backward join rejoins it."""
        if all(st is not s for s in self._compute):
            self._compute.append(st)

    def _wait_compute(self, st, idx) -> None:
        for c in self._compute:
            if c.device.index == idx and c != torch.cuda.current_stream(idx):
                st.wait_stream(c)

    def _end_of_backward(self) -> None:
        self._cb_queued = False
        self.flush()
        self.join()

    def _queue_end_callback(self) -> None:
        if not self._cb_queued:
            try:
                torch.autograd.Variable._execution_engine.queue_callback(self._end_of_backward)
                self._cb_queued = True
            except RuntimeError:        # not inside a backward pass
                pass

    # ------------------------------------------------ weight-gradient jobs
    def submit(self, dev: torch.device, fn: Callable[[], None], keep=(), done=(), spec=None,
               work: float = 0.0) -> None:
        """Run one weight-gradient job: ``fn()`` launches kernels that deposit
        into sink targets, then the parameters in ``done`` are reported.
        Eager: now, on the side stream (:meth:`producer`).  Graph capture with
        deferral on: queued and flushed in batches behind one fork each.
        ``spec``: the same job as a grouped-kernel descriptor
        (hip_impl.wgrad_job); a flush runs all queued specs as ONE grouped
        launch (:attr:`group_fn`) instead of their closures.  ``work``: the
        job's FLOPs for work-based flushing (taken from a weight-gradient
        spec when not given)."""
        capturing = dev.type == "cuda" and torch.cuda.is_current_stream_capturing()
        # (queueing does not depend on the side stream: with it off the flush
        # runs on the current stream, so the same jobs group the same way and
        # the gradients are bitwise those of the side-stream step)
        # (eager grouping: a closure job submitted while grouped jobs are
        # queued is queued behind them -- it may read what they produce, e.g.
        # the attention block's C x C split of the queued M = dy^T a job)
        if dev.type == "cuda" and ((self.graph_defer and capturing) or
                                   (self.eager_group and (spec is not None or self._queue) and not capturing)):
            # the submitting stream travels with the job: its inputs were
            # produced there, and it need not be the stream that flushes
            # (conditioning-stream jobs are often flushed from the compute
            # stream -- see flush())
            self._queue.append((fn, tuple(t for t in keep if t is not None), tuple(p for p in done if p is not None),
                                torch.cuda.current_stream(dev.index if dev.index is not None else None), spec))
            self._queue_end_callback()
            if self.defer_work > 0.0:
                if not work and spec is not None and hasattr(spec, "taps"):
                    work = 2.0 * spec.N * spec.H * spec.W * spec.OC * spec.IC * spec.taps
                self._qwork += work
            if len(self._queue) >= self.defer_batch or self._completes_bucket(done) or \
                    (self.defer_work > 0.0 and self._qwork >= self.defer_work):
                self.flush()
            return
        with self.producer(dev, *keep):
            if self.eager_single and spec is not None and self.group_fn is not None:
                self.group_fn([spec])
            else:
                fn()
        for p in done:
            if p is not None:
                self.done(p)

    def _completes_bucket(self, done) -> bool:
        """Bucket-aware flushing: would reporting the queued jobs' parameters
        complete an all-reduce bucket?  (A parameter completes when the queue
        holds all of its remaining uses.)"""
        if self.bucket_flush is None:
            return False
        for p in done:
            if p is not None and self.managed(p):
                self._qcount[id(p)] = self._qcount.get(id(p), 0) + 1
        full = [self.index[k] for k, c in self._qcount.items() if self.uses.get(k, 0) == c]
        return bool(full) and self.bucket_flush(full)

    def flush(self) -> None:
        """Issue the queued weight-gradient jobs on the side stream behind ONE
        wait on the compute stream, then report their parameters."""
        self._qcount = {}
        self._qwork = 0.0
        if not self._queue:
            return
        q, self._queue = self._queue, []
        grouped = self.group_fn is not None
        if not self.stream_enabled:
            # no side stream: issue in place (the queue was filled from this
            # stream, or from a registered compute stream that the
            # end-of-backward join covers)
            idx = torch.cuda.current_device()
            cur = torch.cuda.current_stream(idx)
            for st in {j[3].cuda_stream: j[3] for j in q}.values():
                if st.cuda_stream != cur.cuda_stream:
                    cur.wait_stream(st)
            if grouped:
                specs = [j[4] for j in q if j[4] is not None]
                if specs:
                    self.group_fn(specs)
            for fn, _, _, _, spec in q:
                if spec is None or not grouped:
                    fn()
            for _, keep, _, st, _ in q:
                if st.cuda_stream != cur.cuda_stream:       # read here, produced on another stream
                    for t in keep:
                        t.record_stream(cur)
            for _, _, done, _, _ in q:
                for p in done:
                    self.done(p)
            return
        idx = torch.cuda.current_device()
        side = self._side(idx)
        # wait for every stream a queued job was submitted from, not only the
        # flushing one: a job queued from the conditioning stream's backward
        # (logSNR MLP, conditioning convs, level-batched FiLM) reads inputs
        # that stream produced, and the batch is usually flushed from the
        # compute stream.  Waiting on the flushing stream alone let those
        # jobs read their inputs before they were written (run-to-run
        # differences of the conditioning gradients in the replayed step,
        # tests/test_ops_gpu.py::test_graph_step_bitwise_deterministic).
        waited = []
        for st in [torch.cuda.current_stream(idx)] + [j[3] for j in q]:
            if all(st.cuda_stream != w.cuda_stream for w in waited):
                side.wait_stream(st)
                waited.append(st)
        with torch.cuda.stream(side):
            if grouped:
                specs = [j[4] for j in q if j[4] is not None]
                if specs:
                    self.group_fn(specs)
            for fn, _, _, _, spec in q:
                if spec is None or not grouped:
                    fn()
        for _, keep, _, _, _ in q:
            for t in keep:
                t.record_stream(side)
        self._forked.add(idx)
        for _, _, done, _, _ in q:
            for p in done:
                self.done(p)

    def join(self) -> None:
        """Make the current stream wait for every deposited gradient (and for
        the registered compute streams)."""
        for idx in list(self._forked):
            torch.cuda.current_stream(idx).wait_stream(self._streams[idx])
        self._forked.clear()
        if self._compute and torch.cuda.is_available() and torch.cuda.is_initialized():
            idx = torch.cuda.current_device()
            self._wait_compute(torch.cuda.current_stream(idx), idx)

    def refork(self, st) -> None:
        """Make the registered compute streams wait on ``st``: after a
        segmented capture was cut (engine/graphs.py comm_mode "seg", the
        capture stream joined every stream, ended its graph and began the
        next one), a compute stream that still has backward work to issue
        must be part of the NEW capture before it launches anything --
        autograd issues same-stream successors without a cross-stream wait.
        (The weight-gradient stream needs none: every flush forks it anew.)"""
        idx = torch.cuda.current_device()
        for c in self._compute:
            if c.device.index == idx and c.cuda_stream != st.cuda_stream:
                c.wait_stream(st)

    @contextlib.contextmanager
    def collective(self, main=None):
        """Issue a collective over deposited gradients: from behind the side
        stream (which first catches up with the compute stream), so it reads
        both streams' gradients without stalling the compute stream.
        ``main``: the stream the backward started on (GradReducer.reset):
        waited for too when the collective is issued from another stream's
        context (a flush from the conditioning stream's backward), so a bucket
        never narrows a gradient that the trunk stream still writes."""
        if not (torch.cuda.is_available() and torch.cuda.is_initialized()):
            yield
            return
        idx = torch.cuda.current_device()
        cur = torch.cuda.current_stream(idx)
        others = [s for s in ([main] if main is not None else []) + [c for c in self._compute if c.device.index == idx]
                  if s.cuda_stream != cur.cuda_stream]
        if _DIAG_NO_STREAM_WAITS:
            others = []                     # diagnostic only: the round-5 ordering (tools/diag_bucket_flush_race.py)
        if not self._forked and not others:
            # every deposit so far was made on this stream: RCCL's stream waits for it
            yield
            return
        # Behind the side stream, which waits for this stream, the backward's
        # main stream and the registered compute streams -- also when nothing
        # has forked yet (deposits on the conditioning stream, or the side
        # stream off): a collective must never read a bucket that another
        # stream still writes.
        side = self._side(idx)
        side.wait_stream(cur)
        for s in others:
            if s.cuda_stream != side.cuda_stream:
                side.wait_stream(s)
        self._forked.add(idx)               # the next join() rejoins it
        with torch.cuda.stream(side):
            yield

    def reset(self) -> None:
        """Start of a step (before its backward).  Also clears the queued
        end-of-backward flag: a backward that raised (e.g. a failed graph
        capture) drops autograd's final callbacks, and a stale flag would stop
        the next backward from queueing its flush + join."""
        self._qcount = {}
        self._qwork = 0.0
        self.uses = {}
        self.seen = set()
        self._queue = []
        self._cb_queued = False


SINK = GradSink()
