"""HIP-graph training step: the whole per-step launch stream replayed from
two captured graphs instead of ~2,000 Python-issued launches.

Why: at the scaling config (global batch 128 over 8 GPUs = 16 examples per
GPU) the eager step is launch-bound -- the host needs about as long to issue
the forward/backward kernels (autograd + ctypes per op) as the GPU needs to run
them.  A replayed graph issues the same kernels with no host work in between.

Layout of one step (MI355X, one process per GPU):

  graph A (per micro-batch): q_sample randoms (registered generator) ->
      X-UNet forward -> backward; HIP weight-gradient kernels deposit into the
      flat fp32 gradient buffer (GradSink), the micro-batch loss is added to a
      device accumulator.  Inputs are copied into static buffers first.
  [world > 1, comm_mode "graph"] the bucketed RCCL all-reduces are captured
      INTO graph A: the same gradient hooks / sink notifications that drive
      the eager reducer (parallel/ddp.py) fire during capture, so each bucket's
      collective is recorded on RCCL's stream as soon as its last gradient is
      deposited, with event edges from the compute stream; on replay the
      reduction of bucket k runs concurrently with the backward kernels of
      the layers below it, exactly like the eager overlapped step, and only
      the last (small, first-layer) buckets are exposed.  Graph A ends by
      joining RCCL's stream (work.wait() captured as an edge).  A bf16
      payload (dist.grad_dtype) narrows each bucket into a persistent bf16
      mirror on the collective's stream and widens it back inside the graph.
      ``dist.force_comm`` runs this topology on a 1-rank RCCL group (tests).
  [world > 1, comm_mode "seg"] fallback when a probe capture of an RCCL
      collective fails (or D3D_GRAPH_COMM=0): graph A is captured as a CHAIN
      of segment graphs cut at bucket boundaries.  The same gradient hooks /
      sink notifications that issue the collectives in the eager step mark
      the cut points: once >= D3D_GRAPH_SEG MiB of buckets are complete the
      capture stream joins every stream (the weight-gradient stream, the
      conditioning stream), ends its graph and begins the next one in the
      same memory pool, re-forking the conditioning stream into it.  A step
      replays segment k, then issues the eager all-reduces of the buckets
      completed in it on RCCL's stream, then replays segment k + 1: bucket k's
      reduction overlaps the backward of the layers below it, as in the
      captured mode, without any collective inside a graph; only the buckets
      of the last segment are exposed.  The deferred update is kept.
  [world > 1, comm_mode "post"] last resort (the segmented capture failed, or
      D3D_GRAPH_SEG=0, or gloo): eager all-reduce of the flat gradient after
      graph A in 4 async chunks, each chunk's Adam launched as soon as its
      collective lands; bf16 payload by default (dist.post_grad_dtype: the
      reduction is exposed here, so half the bytes is half the exposed time).
      (Overlap by a signal out of ONE running graph was tried: external
      event-record nodes are refused by this stack -- torch's
      Event(external=True) on ROCm and hipEventRecordWithFlags(
      hipEventRecordExternal) inside a capture, hipErrorInvalidValue on the
      box, which also invalidates the capture.)
  graph B: fused Adam reading its per-step hyper-parameters from a device
      block (lr warmup / bias correction change every step; the 1/world
      gradient average is folded in) -> batched weight repack -> gradient /
      loss-accumulator zeroing.

Per-step values that a replay cannot see from Python travel through device
words refreshed before the replays: the dropout seed (``hip_impl._SEED_DEV``,
added to every mask kernel's baked seed) and the Adam block ``hp``.
"""
from __future__ import annotations

import contextlib
import gc
import os
from typing import Optional

import torch
import torch.distributed as dist


@contextlib.contextmanager
def _gc_paused():
    """No Python garbage collection while a stream is being captured: a dead
    reference cycle (e.g. a previous Trainer and its CUDAGraphs) finalised by
    a collection that happens to run mid-capture destroys a graph / releases a
    graph memory pool inside the capture -- an illegal call that aborts the
    process (torch >= 2.9 no longer collects before capture by default).  The
    cycles are collected here, before the capture begins."""
    was = gc.isenabled()
    gc.collect()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()


def probe_graph_collective(device: torch.device) -> bool:
    """True when an RCCL all-reduce can be captured in a HIP graph and replayed
    correctly on every rank.  Run once, eagerly, before the step capture; the
    verdict is agreed over the group (MIN), so all ranks take the same path."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_backend() != "nccl":
        return False
    ok = 1.0
    try:
        world = dist.get_world_size()
        x = torch.zeros(4096, device=device)
        s = torch.cuda.Stream(device=device)
        s.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(s):          # warm the collective outside the capture
            dist.all_reduce(x)
        torch.cuda.current_stream(device).wait_stream(s)
        torch.cuda.synchronize(device)      # the warm-up has completed (see _capture on the watchdog)
        g = torch.cuda.CUDAGraph()
        with _gc_paused(), torch.cuda.graph(g, capture_error_mode="thread_local"):
            w = dist.all_reduce(x, async_op=True)
            w.wait()
            x.mul_(2.0)
        for rep in range(2):
            x.fill_(float(dist.get_rank() + 1 + rep))
            g.replay()
        torch.cuda.synchronize(device)
        want = 2.0 * (world * (world + 1) / 2 + world)
        ok = float(bool(torch.all(x == want).item()))
    except Exception as e:                   # noqa: BLE001 -- any failure means "do not capture"
        print(f"[graphs] RCCL graph-capture probe failed ({type(e).__name__}: {e}); "
              "all-reduce runs after the graph", flush=True)
        ok = 0.0
    flag = torch.tensor([ok], device=device)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    return bool(flag.item() > 0.5)


_FUSED_UPDATE = True
# Deferred optimizer step: the Adam update of step t runs inside the replay of
# step t+1's graph A, the bulk of it on a side stream overlapped with the
# forward (bs16: the ~1 ms bandwidth-bound update hides behind the first
# encoder levels' compute-bound convolutions).  Parameters read by the forward
# wait on it exactly where they are first used (models.xunet.PARAM_FENCE);
# flush() applies a pending update (checkpoints, evaluation, the end).
_DEFER_UPDATE = os.environ.get("D3D_DEFER_UPDATE", "1") != "0"
# Adam hyper-parameter block that leaves p, m, v and the EMA bit-identical
# (b1 = b2 = 1, step 0, no weight decay, gradient scale 0, EMA weight 0): the
# "previous update" of the first replay and of the replay after a flush.
_NOOP_HP = [1.0, 1.0, 1.0, 0.0, 0.0, 1.0, 0.0, 0.0]


def _seg_mb() -> float:
    """comm_mode "seg": cut the capture once this many MiB of gradient buckets
    are complete (D3D_GRAPH_SEG; 0: no segmented mode, the post-graph
    reduction is the fallback).  Read per GraphedTrainStep."""
    return float(os.environ.get("D3D_GRAPH_SEG", "64"))


def agree_switches(*flags: bool, device=None) -> tuple:
    """Per-rank boolean switches (environment knobs) agreed over the group:
    True only where every rank says True (MIN).  Used before any choice that
    changes the collective sequence a rank runs."""
    if not (dist.is_available() and dist.is_initialized()):
        return tuple(bool(f) for f in flags)
    dev = device if (device is not None and dist.get_backend() == "nccl") else "cpu"
    t = torch.tensor([float(bool(f)) for f in flags], device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return tuple(bool(v > 0.5) for v in t.tolist())


class GraphCaptureError(RuntimeError):
    """The training step could not be captured (on this rank or any other):
    the trainer falls back to the eager step on every rank."""


class GraphedTrainStep:
    def __init__(self, trainer, micro_batch: int, example):
        from ..ops import hip_impl
        self.tr = trainer
        self.H = hip_impl
        dev = trainer.device
        self.mb = micro_batch
        img, R, T, K = example
        # static inputs (one micro-batch)
        self.img = torch.zeros((micro_batch,) + tuple(img.shape[1:]), dtype=img.dtype, device=dev)
        self.R = torch.zeros((micro_batch,) + tuple(R.shape[1:]), dtype=R.dtype, device=dev)
        self.T = torch.zeros((micro_batch,) + tuple(T.shape[1:]), dtype=T.dtype, device=dev)
        self.K = torch.zeros((micro_batch,) + tuple(K.shape[1:]), dtype=K.dtype, device=dev)
        self.frac = torch.ones((), device=dev)
        self._frac = 1                          # chunk count frac holds (1 / _frac)
        self.loss_acc = torch.zeros((), device=dev)
        self.seed = torch.zeros(3, dtype=torch.int64, device=dev)    # [dropout word, draw word, example offset]
        self.hp = torch.zeros(8, device=dev)
        self.pool = torch.cuda.graph_pool_handle()
        self.gA: Optional[torch.cuda.CUDAGraph] = None      # fwd+bwd (+ captured all-reduce)
        self.gA0: Optional[torch.cuda.CUDAGraph] = None     # fwd+bwd without comm (leading micro-batches)
        self.gB: Optional[torch.cuda.CUDAGraph] = None
        self.comm_mode = None
        red = trainer.reducer
        if red is not None and red.active:
            # fp32 and bf16 payloads alike (the bf16 mirror is persistent, see
            # parallel/ddp.py): the collectives are captured inside graph A.
            # The per-rank switches are agreed over the group first (MIN): a
            # rank that probes or captures segments while another does not
            # would run a different collective sequence and hang the job.
            want, seg_ok = agree_switches(os.environ.get("D3D_GRAPH_COMM", "1") != "0",
                                          _seg_mb() > 0 and dist.get_backend() == "nccl", device=dev)
            if want and probe_graph_collective(dev):
                self.comm_mode = "graph"
            elif seg_ok:
                self.comm_mode = "seg"
            else:
                self.comm_mode = "post"
        self.segs: Optional[list] = None        # comm_mode "seg": segment graphs of the last micro-batch
        self.seg_bk: Optional[list] = None      # ... and the buckets completed in each
        # post mode: a persistent narrow mirror of the flat gradient (bf16 payload)
        self.post_mirror = None
        if self.comm_mode == "post" and trainer.cfg.dist.post_grad_dtype == "bf16":
            self.post_mirror = torch.empty(trainer.flat.grad.numel(), dtype=torch.bfloat16, device=dev)
        # Deferred, overlapped optimizer step (see step()): needs the fused
        # update, the in-graph (or no) reduction and one micro-batch per step.
        split = trainer.model.update_parts() if hasattr(trainer.model, "update_parts") else None
        self.defer = (_DEFER_UPDATE and _FUSED_UPDATE and split is not None and self.comm_mode != "post"
                      and micro_batch >= trainer.local_batch)
        self.pending = False
        if self.defer:
            early_ids = {id(p) for p in split[0]}
            fl = trainer.flat
            self.parts = [{i for i, p in enumerate(fl.params) if id(p) in early_ids},
                          {i for i, p in enumerate(fl.params) if id(p) not in early_ids}]
            self.fence_level = split[1]
            self.upd_stream = torch.cuda.Stream(device=dev)
            self.H.set_words(self.hp, _NOOP_HP)

    # ------------------------------------------------------------------
    def _body(self, comm: bool = False, defer: bool = False) -> None:
        tr = self.tr
        if tr.sink is not None:
            tr.sink.reset()
        red = tr.reducer
        if red is not None:
            red.enabled = comm
            red.reset()
        from ..models import xunet as _xunet
        main = torch.cuda.current_stream()
        if defer:
            # the PREVIOUS step's update, overlapped with this forward: the
            # small early part (parameters read before encoder level
            # fence_level) on the compute stream, the rest -- and the gradient
            # zeroing -- on the update stream behind one event that the
            # forward waits on right before it first reads those parameters
            o = tr.optim
            # (each part clears the gradients it consumes: no separate zeroing pass)
            self.H.adam_update_part(o.flat, o.exp_avg, o.exp_avg_sq, o.ema, self.hp, 0, zero_g=True)
            S = self.upd_stream
            S.wait_stream(main)
            ev = torch.cuda.Event()
            with torch.cuda.stream(S):
                self.H.adam_update_part(o.flat, o.exp_avg, o.exp_avg_sq, o.ema, self.hp, 1, zero_g=True)
                ev.record(S)
            self.loss_acc.zero_()
            _xunet.PARAM_FENCE[0] = (self.fence_level, ev)
        try:
            # step word 0 / offset 0 baked: the per-step words and the micro-batch
            # offset come from the device block self.seed (see step())
            batch, mask, eps = tr.diffusion_inputs(self.img, self.R, self.T, self.K, 0, step_word=0)
            y = tr.model(batch, cond_mask=mask, head_nhwc=True)
        finally:
            _xunet.PARAM_FENCE[0] = None
        if defer:
            main.wait_stream(self.upd_stream)
        from .. import ops
        loss = ops.diff_loss_nhwc(y, eps, tr.cfg.diffusion.loss_type)
        (loss * self.frac).backward()
        self.loss_acc.add_(loss.detach() * self.frac)
        if red is not None and comm:
            red.finish()            # remaining buckets + the join of RCCL's stream (captured edges)
        elif tr.sink is not None:
            # the end-of-backward callback normally did this; explicit, so a
            # weight-gradient job still queued can never be left out of the
            # graph (a no-op when the callback ran)
            tr.sink.flush()
            tr.sink.join()
        if red is not None:
            red.enabled = False

    def _update(self) -> None:
        o = self.tr.optim
        if _FUSED_UPDATE:
            # Adam + operand repack + gradient zeroing fused (ops.hip_impl.adam_update_all)
            self.H.adam_update_all(o.flat, o.exp_avg, o.exp_avg_sq, o.ema, self.hp, zero_g=True)
        else:
            self.H.adam_flat_dev(o.flat.data, o.flat.grad, o.exp_avg, o.exp_avg_sq, o.ema, self.hp)
            o.flat.grad.zero_()
        self.loss_acc.zero_()

    def capture(self, nchunks: int = 1) -> None:
        """Capture the graphs; on failure (here or on any rank) raise
        GraphCaptureError on every rank, so all ranks take the same path.  A
        failed SEGMENTED capture is retried once in comm_mode "post"."""
        err = self._capture_agreed(nchunks)
        if err is not None and self.comm_mode == "seg":
            if self.tr.ctx.is_main:
                print(f"[graphs] segmented capture failed ({type(err).__name__}: {err}); "
                      "all-reduce runs after the graph", flush=True)
            self.comm_mode = "post"
            if self.tr.cfg.dist.post_grad_dtype == "bf16":
                self.post_mirror = torch.empty(self.tr.flat.grad.numel(), dtype=torch.bfloat16,
                                               device=self.tr.device)
            self.defer = False
            self.tr.flat.zero_grad()
            self.loss_acc.zero_()
            err = self._capture_agreed(nchunks)
        if err is not None:
            tr = self.tr
            tr.flat.zero_grad()
            self.loss_acc.zero_()
            raise GraphCaptureError(f"{type(err).__name__}: {err}") from err

    def _capture_agreed(self, nchunks: int):
        err = None
        try:
            self._capture(nchunks)
        except Exception as e:            # noqa: BLE001
            err = e
            self._drop()
            try:
                torch.cuda.synchronize()
            except Exception as e2:       # noqa: BLE001 -- a capture the failure left open
                print(f"[graphs] synchronize after the failed capture: {type(e2).__name__}: {e2}", flush=True)
        tr = self.tr
        # (also on a forced 1-rank group: the tests run this agreement path)
        red = tr.reducer
        if dist.is_initialized() and (tr.ctx.world > 1 or (red is not None and red.active)):
            ok = 0.0 if err is not None else 1.0
            # (comm_mode is agreed over the group: every rank runs this exchange or none does)
            if self.comm_mode == "seg" and not self._segments_agree() and err is None:
                ok = 0.0
                err = RuntimeError("segmented capture: the ranks cut different segment layouts")
                self._drop()
            if self.comm_mode == "graph" and not self._issue_order_agrees() and err is None:
                ok = 0.0
                err = RuntimeError("captured collectives: the ranks recorded different bucket sequences")
                self._drop()
            flag = torch.tensor([ok], device=tr.device)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
            if flag.item() < 0.5 and err is None:
                err = RuntimeError("graph capture failed on another rank")
                self._drop()
        return err

    def _segments_agree(self) -> bool:
        """Every rank must issue the eager bucket all-reduces of the segmented
        step in the same sequence (else RCCL pairs different buckets and
        hangs): compare the [bucket -> (segment, position)] layout over the
        group (MIN == MAX)."""
        nb = len(self.tr.reducer.buckets)
        lay = torch.full((2 * nb + 1,), -1.0, device=self.tr.device)
        lay[-1] = float(len(self.segs)) if self.segs is not None else -1.0
        pos = 0
        for si, bks in enumerate(self.seg_bk or []):
            for b in bks:
                if 0 <= b < nb:
                    lay[2 * b] = float(si)
                    lay[2 * b + 1] = float(pos)
                pos += 1
        hi, lo = lay.clone(), lay.clone()
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        return bool(torch.equal(hi, lo))

    def _issue_order_agrees(self) -> bool:
        """comm_mode "graph": the bucket all-reduces recorded into graph A must
        come in the same sequence on every rank (RCCL pairs collectives by
        issue order: a different sequence reduces mismatched buckets or hangs
        at the first replay).  The capture's [bucket -> position] map is
        compared over the group (MIN == MAX), as _segments_agree does for the
        segmented capture.  An empty log (the capture failed) compares as
        all -1 and the failure is reported through the capture flag."""
        red = self.tr.reducer
        nb = len(red.buckets)
        lay = torch.full((nb + 1,), -1.0, device=self.tr.device)
        log = red.issue_log if self.gA is not None else []
        lay[-1] = float(len(log))
        for pos, b in enumerate(log):
            if 0 <= b < nb:
                lay[b] = float(pos)
        hi, lo = lay.clone(), lay.clone()
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        return bool(torch.equal(hi, lo))

    def _drop(self) -> None:
        self.gA = self.gA0 = self.gB = None
        self.segs = self.seg_bk = None
        self.H.set_device_seed(None)
        red = self.tr.reducer
        if red is not None:
            red.seg_cut = None

    def _capture(self, nchunks: int = 1) -> None:
        tr = self.tr
        tr.model.train()
        tr.model.set_dropout_seed(0)             # baked; the per-step part is self.seed
        self.H.set_device_seed(self.seed)
        comm = self.comm_mode == "graph"
        seg = self.comm_mode == "seg"
        self.img.normal_()
        self.R.copy_(torch.eye(3, device=self.R.device).expand_as(self.R))
        self.K.copy_(torch.eye(3, device=self.K.device).expand_as(self.K))
        # warm-up on a side stream: lazy library init, weight caches, allocator
        # (the generator is rewound afterwards so replays draw the same
        # randoms the eager step would)
        gstate = tr.gen.get_state()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                self._body(comm or seg)
        torch.cuda.current_stream().wait_stream(s)
        self.H.refresh_weights()                 # descriptor table final before capture
        # RCCL's watchdog thread keeps polling the events of the warm-up's eager
        # collectives while the capture runs.  That is safe by construction, no
        # timing involved: (1) every capture below is thread_local when
        # collectives are in play, so the watchdog's event queries from its own
        # thread are legal during it; (2) TORCH_NCCL_CUDA_EVENT_CACHE=0
        # (parallel/dist.py) gives every collective fresh events, so no event
        # the watchdog still tracks is re-recorded inside the capture; (3)
        # collectives issued during capture are not handed to the watchdog.
        # The synchronize below only makes the warm-up complete first.
        if _FUSED_UPDATE:
            self.H.prepare_fused_update(tr.flat)
        if self.defer:
            self.H.prepare_update_parts(tr.flat, self.parts)
        torch.cuda.synchronize()
        # RCCL's watchdog thread keeps querying events: thread_local with
        # collectives in play.  The segmented capture is cut (one capture
        # ended, the next begun) from autograd's worker thread, which a
        # thread_local capture refuses (hipErrorStreamCaptureWrongThread): relaxed.
        mode = "relaxed" if seg else ("thread_local" if comm else "global")
        # graphs sharing a memory pool are captured in their replay order
        # (leading micro-batches first)
        with _gc_paused():
            if (comm or seg) and nchunks > 1:
                self.gA0 = torch.cuda.CUDAGraph()
                self.gA0.register_generator_state(tr.gen)
                with torch.cuda.graph(self.gA0, pool=self.pool, capture_error_mode=mode):
                    self._body(False)
            if seg:
                self._capture_segments(mode)
            else:
                self.gA = torch.cuda.CUDAGraph()
                self.gA.register_generator_state(tr.gen)
                with torch.cuda.graph(self.gA, pool=self.pool, capture_error_mode=mode):
                    self._body(comm, defer=self.defer)
            self.gB = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.gB, pool=self.pool, capture_error_mode=mode):
                self._update()
        torch.cuda.synchronize()
        tr.gen.set_state(gstate)
        # scope the device seed word to the replays (an eager forward after
        # this must not add a stale device seed to its dropout seed)
        self.H.set_device_seed(None)
        # warm-up / capture left partial gradients behind
        tr.flat.zero_grad()
        self.loss_acc.zero_()

    # ------------------------------------------------------------ "seg" mode
    def _capture_segments(self, mode: str) -> None:
        """Graph A of the last micro-batch as a chain of segment graphs, cut
        where the gradient buckets complete (see the module doc)."""
        tr = self.tr
        red = tr.reducer
        cs = torch.cuda.Stream()
        cs.wait_stream(torch.cuda.current_stream())
        self._cs, self._mode = cs, mode
        self._seg_bytes = _seg_mb() * 2 ** 20
        self._seg_acc = 0
        g = torch.cuda.CUDAGraph()
        g.register_generator_state(tr.gen)
        self.segs, self.seg_bk = [g], [[]]
        with torch.cuda.stream(cs):
            g.capture_begin(pool=self.pool, capture_error_mode=mode)
            red.seg_cut = self._cut
            try:
                self._body(True, defer=self.defer)
            except BaseException:
                try:
                    self.segs[-1].capture_end()
                except Exception:        # noqa: BLE001 -- the original error is the one to report
                    pass
                raise
            finally:
                red.seg_cut = None
            self.segs[-1].capture_end()
        torch.cuda.current_stream().wait_stream(cs)
        self.gA = self.segs[-1]

    def _cut(self, b: int, cut: bool) -> None:
        """Bucket b is complete (called from backward, on whichever thread
        runs it): record it in the current segment; cut the capture once the
        segment holds >= D3D_GRAPH_SEG MiB of buckets."""
        self.seg_bk[-1].append(b)
        if not cut:
            return
        bk = self.tr.reducer.buckets[b]
        self._seg_acc += (bk["end"] - bk["start"]) * 4
        if self._seg_acc < self._seg_bytes:
            return
        self._seg_acc = 0
        sink = self.tr.sink
        with torch.cuda.stream(self._cs):
            # every stream of the capture rejoins the capture stream (legal
            # end), the next segment begins in the same pool, and the
            # conditioning stream is forked into it again
            sink.join()
            self.segs[-1].capture_end()
            g = torch.cuda.CUDAGraph()
            g.capture_begin(pool=self.pool, capture_error_mode=self._mode)
            self.segs.append(g)
            self.seg_bk.append([])
            sink.refork(self._cs)

    def _seg_issue(self, b: int, works: list) -> None:
        """Eager all-reduce of bucket b on RCCL's stream (behind everything
        replayed so far on the current stream), the reducer's payload."""
        red = self.tr.reducer
        bk = red.buckets[b]
        view = self.tr.flat.grad[bk["start"]: bk["end"]]
        src = red.probe_src(b, view)                 # (test-only race probe: a snapshot, result discarded)
        back = view if src is view else None
        if red.mirror is None:
            works.append((dist.all_reduce(src, group=red.group, async_op=True), None, None))
        else:
            tmp = red.mirror[bk["start"]: bk["end"]]
            tmp.copy_(src)
            works.append((dist.all_reduce(tmp, group=red.group, async_op=True), tmp, back))

    def _replay_segments(self, comm: bool = True) -> None:
        works: list = []
        for g, bks in zip(self.segs, self.seg_bk):
            g.replay()
            if comm:
                for b in bks:
                    self._seg_issue(b, works)
        for w, tmp, view in works:
            w.wait()                      # the current stream waits on RCCL's
            if tmp is not None and view is not None:
                view.copy_(tmp)
        if comm:
            self.tr.reducer.probe_final()

    # ------------------------------------------------------------------
    def _reduce_update_chunked(self) -> None:
        """All-reduce in chunks (bf16 payload through a persistent mirror by
        default), each chunk's Adam behind its own collective (overlaps the
        optimizer with the remaining reduction)."""
        o = self.tr.optim
        p, g, m, v, ema = o.flat.data, o.flat.grad, o.exp_avg, o.exp_avg_sq, o.ema
        n = g.numel()
        k = 4
        cuts = [0] + [min(n, (n * i // k + 255) // 256 * 256) for i in range(1, k)] + [n]
        spans = [(a, b) for a, b in zip(cuts[:-1], cuts[1:]) if b > a]
        mir = self.post_mirror
        works = []
        for a, b in spans:
            if mir is None:
                works.append(dist.all_reduce(g[a:b], async_op=True))
            else:
                mir[a:b].copy_(g[a:b])
                works.append(dist.all_reduce(mir[a:b], async_op=True))
        for (a, b), w in zip(spans, works):
            w.wait()
            if mir is not None:
                g[a:b].copy_(mir[a:b])
            self.H.adam_flat_dev(p[a:b], g[a:b], m[a:b], v[a:b], ema[a:b] if ema is not None else None, self.hp,
                                 refresh=False)
        self.H.refresh_weights()
        g.zero_()
        self.loss_acc.zero_()

    def step(self, img, R, T, K, want_norm: bool = False) -> torch.Tensor:
        tr = self.tr
        B = img.shape[0]
        mb = self.mb
        assert B % mb == 0, (B, mb)
        nchunks = B // mb
        if self.gA is None:
            self.capture(nchunks)
        # same seeds as the eager step (Trainer.train_step): the captured
        # kernels carry the base seeds and add these device words
        word = tr.step * tr.ctx.world + tr.ctx.rank
        if self._frac != nchunks:
            self.frac.fill_(1.0 / nchunks)
            self._frac = nchunks
        from .trainer import dropout_word
        for ci, s in enumerate(range(0, B, mb)):
            # one kernel-argument write (no H2D copy, no host wait): fewer host launches at the step boundary
            self.H.set_words64(self.seed, (dropout_word(word, ci), word, s))
            self.img.copy_(img[s:s + mb])
            self.R.copy_(R[s:s + mb])
            self.T.copy_(T[s:s + mb])
            self.K.copy_(K[s:s + mb])
            last = ci == nchunks - 1
            if last and self.segs is not None:
                self._replay_segments()
            else:
                (self.gA if (last or self.gA0 is None) else self.gA0).replay()
        loss = self.loss_acc.clone()
        world = tr.ctx.world
        o = tr.optim
        clip = tr.cfg.optim.grad_clip
        o.hparams_to(self.hp, 1.0 / world)        # kernel-argument write: no host wait
        post = self.comm_mode == "post"
        if post and (clip > 0 or want_norm):
            # the norm needs the whole reduced gradient first: one reduction, no chunking
            g = tr.flat.grad
            if self.post_mirror is not None:
                self.post_mirror.copy_(g)
                dist.all_reduce(self.post_mirror)
                g.copy_(self.post_mirror)
            else:
                dist.all_reduce(g)
            post = False
        if want_norm or clip > 0:
            norm = o.grad_norm(1.0 / world)
            tr.last_grad_norm = norm
            if clip > 0:
                self.hp[6:7].mul_(o.clip_coef(norm, clip))
        if post:
            self._reduce_update_chunked()
        elif self.defer:
            # the update runs at the start of the next replay of graph A,
            # overlapped with its forward (or at flush())
            self.pending = True
        else:
            self.gB.replay()
        for cb in o.on_step:
            cb()
        return loss

    def measure_comm(self, reps: int = 3) -> Optional[float]:
        """Exposed gradient-communication time per step of the captured step
        (diagnostics after a benchmark; changes the training state): graph A
        is captured once more WITHOUT its collectives (own pool) and the two
        are replayed alternately; the difference of their device times is the
        part of the bucketed all-reduce that the backward did not hide.
        ``post`` mode: the device time of the chunked all-reduce + Adam after
        the graph minus the fused update alone.  None when there is no comm."""
        if self.comm_mode is None or self.gA is None:
            return None
        tr = self.tr
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

        def dev_ms(fn):
            torch.cuda.synchronize()
            ev[0].record()
            for _ in range(reps):
                fn()
            ev[1].record()
            ev[1].synchronize()
            return ev[0].elapsed_time(ev[1]) / reps

        if self.comm_mode == "post":
            with_comm = dev_ms(lambda: (self.gA.replay(), self._reduce_update_chunked()))
            without = dev_ms(lambda: (self.gA.replay(), self._update()))
            return max(0.0, with_comm - without)
        if self.comm_mode == "seg":
            # the segment chain with its eager bucket all-reduces against the
            # same chain replayed without them
            with_comm = dev_ms(self._replay_segments)
            without = dev_ms(lambda: self._replay_segments(comm=False))
            with_comm = min(with_comm, dev_ms(self._replay_segments))
            tr.flat.zero_grad()
            return max(0.0, with_comm - without)
        g0 = torch.cuda.CUDAGraph()
        g0.register_generator_state(tr.gen)
        self.H.set_device_seed(self.seed)
        try:
            torch.cuda.synchronize()
            # (GC paused like every other capture: a collection finalising an
            # old graph mid-capture aborts the process, uncatchably)
            with _gc_paused(), torch.cuda.graph(g0, pool=torch.cuda.graph_pool_handle(),
                                                capture_error_mode="thread_local"):
                self._body(False, defer=self.defer)
        finally:
            self.H.set_device_seed(None)
        t_comm = dev_ms(self.gA.replay)
        t_none = dev_ms(g0.replay)
        t_comm = min(t_comm, dev_ms(self.gA.replay))
        del g0
        tr.flat.zero_grad()
        return max(0.0, t_comm - t_none)

    def flush(self) -> None:
        """Apply a deferred update now (checkpoint, evaluation, end of
        training, switching step paths): afterwards the parameters are those
        of the eager step."""
        if self.defer and self.pending:
            self.gB.replay()
            self.pending = False
            self.H.set_words(self.hp, _NOOP_HP)
