"""Training engine (reference: DDP loop `train.py:200-303`, Lightning module
`lightning/diff3d.py:52-127`).

One process per GPU.  Per step (no host synchronisation in the steady state):
  1. diffusion forward on device: t~U[0,1), lambda(t), eps, z_t, CFG drop
     (10 % of examples get noise instead of the conditioning view and zeroed
     rays; `train.py:80-100`);
  2. X-UNet forward/backward (HIP kernels on MI355X);
  3. bucketed RCCL all-reduce launched from gradient hooks during backward,
     drained before the optimizer;
  4. one fused Adam launch (averaging folded in) + LR schedule.
Rank 0 writes reference-named checkpoints atomically; losses are read back
only every ``log_every`` steps.  Defects D1-D8 of the reference are fixed
(see SURVEY 2.9).
"""
from __future__ import annotations

import copy
import math
import os
import time
from typing import Dict, Iterator, Optional, Tuple

import torch

from .. import ops
from ..config import TrainConfig, dumps, to_dict
from ..models import XUNet
from ..parallel import (DistContext, FlatParams, GradReducer, get_context, check_replicas_in_sync)
from ..utils import (save_checkpoint, load_checkpoint, load_model_weights, find_resume, MetricsLogger,
                     StepTimer, train_flops_per_example, range_push, check_finite)
from .optim import FusedAdam, ema_decay_for, warmup_lr


def dropout_word(step_word: int, chunk: int) -> int:
    """Dropout seed word of micro-batch ``chunk`` of a step (distinct per
    micro-batch: the masks are element-indexed within each launch)."""
    return step_word + (chunk << 40)


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


class Trainer:
    def __init__(self, cfg: TrainConfig, ctx: Optional[DistContext] = None):
        self.cfg = cfg
        self.ctx = ctx or get_context()
        dev = self.ctx.device
        self.device = dev
        if cfg.backend != "auto":
            ops.set_backend(cfg.backend)
        if dev.type == "cuda":
            from ..utils.gemm_tuning import enable_tuned_gemms
            self.tuned_gemms = enable_tuned_gemms()
        if cfg.deterministic:
            torch.use_deterministic_algorithms(True, warn_only=True)
        torch.manual_seed(cfg.seed)
        self.model = XUNet(copy.deepcopy(cfg.model)).to(dev)
        self.dtype = torch.bfloat16 if (dev.type == "cuda" and cfg.dtype == "bf16") else torch.float32
        self.model.compute_dtype = self.dtype
        self.flat = FlatParams(list(self.model.parameters()), device=dev)
        W = self.ctx.world
        if cfg.global_batch % W != 0:
            raise ValueError(f"global_batch {cfg.global_batch} not divisible by world size {W}")
        self.local_batch = cfg.global_batch // W
        self.reducer = None
        if W > 1 or cfg.dist.force_comm:
            self.reducer = GradReducer(self.flat, cfg.dist.bucket_mb, cfg.dist.first_bucket_mb, cfg.dist.grad_dtype,
                                       force=cfg.dist.force_comm)
        # Direct gradient sink: HIP weight-gradient kernels deposit straight
        # into the flat gradient buffer (no AccumulateGrad adds) and report
        # completion to the bucketed reducer themselves.
        self.sink = None
        if dev.type == "cuda" and self.dtype == torch.bfloat16 and cfg.backend != "torch" and \
                os.environ.get("D3D_GRAD_SINK", "1") == "1":
            from ..ops.gradsink import SINK
            views = [self.flat.view(self.flat.grad, i) for i in range(len(self.flat.params))]
            notify = self.reducer.mark_ready if self.reducer is not None else None
            SINK.attach(self.flat.params, views, notify)
            if self.reducer is not None:
                self.reducer.sink = SINK
            self.sink = SINK
            # weight-gradient jobs per side-stream fork in graph capture: 128
            # when no collective waits on the reports (over 64: bs16 +2.9 %,
            # bs64 +1.3 %, bs32 -0.2 %); 32 when the bucketed all-reduces do
            # (over 16 in the 1-rank rehearsal: bs16 +2.4-2.9 %, bs32 +0.9 %)
            # -- a parameter is reported only when its job's batch is flushed,
            # so big batches would start the buckets' reductions late.  The
            # captured collective step misbehaved with MANY captured
            # collectives (16 MiB buckets or smaller: ~30-170 per step) under
            # extra work on the collective path; with the default 64 MiB
            # buckets (9 per step) it stayed bit-exact even at 64-job flushes
            # (profiles/r6/defer_batch.txt).  Values above 32 are clamped.
            # D3D_WGRAD_DEFER_BATCH overrides.
            comm = self.reducer is not None and self.reducer.active
            SINK.defer_batch = int(os.environ.get("D3D_WGRAD_DEFER_BATCH", "32" if comm else "128"))
            if comm and cfg.graph and len(self.reducer.buckets) > 32:
                print(f"[trainer] warning: {len(self.reducer.buckets)} all-reduce buckets per step; the captured "
                      f"collective step was seen to go wrong with ~90+ collectives under extra collective-path "
                      f"work (profiles/r6/defer_batch.txt) -- prefer dist.bucket_mb >= 32", flush=True)
            if comm and SINK.defer_batch > 32 and os.environ.get("D3D_DIAG_BF16_ANY_BATCH", "0") != "1":
                print(f"[trainer] collective step: weight-gradient flush batch {SINK.defer_batch} -> 32", flush=True)
                SINK.defer_batch = 32
            # bucket-aware flushing (opt-in): a queued job that completes a
            # bucket flushes the queue at once, so batches can be big without
            # delaying any bucket's reduction (profiles/r6/bucket_flush.txt)
            SINK.bucket_flush = self.reducer.completes_bucket if comm and \
                os.environ.get("D3D_WGRAD_BUCKET_FLUSH", "0") == "1" else None
            if SINK.bucket_flush is not None and self.reducer.mirror is not None:
                SINK.bucket_flush = None        # (NaN with the bf16 mirror: profiles/r6/bucket_flush.txt)
        oc = cfg.optim
        self.optim = FusedAdam(self.flat, oc.lr, oc.betas, oc.eps, oc.weight_decay,
                               ema_decay_for(cfg.global_batch, oc.ema_halflife_examples))
        self.optim.zero_in_step = True        # train_step zeroes right after each update
        self.sched = None
        if oc.use_cosine:
            self.sched = torch.optim.lr_scheduler.CosineAnnealingLR(self.optim, T_max=oc.cosine_tmax)
        self.warmup_steps = oc.warmup_examples / cfg.global_batch if oc.warmup_examples > 0 else 0.0
        self.step = 0
        self.epoch = 0
        self.gen = torch.Generator(device=dev)
        self.gen.manual_seed(cfg.seed * 1000003 + self.ctx.rank + 1)
        self.out_dir = cfg.out_dir or cfg.transfer or "runs/default"
        self.logger = MetricsLogger(os.path.join(self.out_dir, "metrics.jsonl") if self.ctx.is_main else None)
        self.fault_step = int(os.environ.get("D3D_FAULT_AT_STEP", "-1"))
        self.fault_rank = int(os.environ.get("D3D_FAULT_RANK", "-1"))
        self.epoch_pos = 0          # batches of self.epoch already consumed (mid-epoch resume)
        if cfg.pretrained and not cfg.transfer:
            ck = load_checkpoint(cfg.pretrained, map_location="cpu")
            load_model_weights(self.model, ck["model"])
            if "optim" in ck:
                self.optim.load_state_dict(ck["optim"])
            self.optim.reset_ema()          # EMA starts from the loaded weights, not random init
        if cfg.transfer:
            self.resume(cfg.transfer)
        if self.reducer is not None:
            self.reducer.broadcast_params(0)

    # ------------------------------------------------------------------
    def resume(self, transfer: str) -> bool:
        path = find_resume(transfer)
        if path is None:
            return False
        ck = load_checkpoint(path, map_location="cpu")
        load_model_weights(self.model, ck["model"])
        if "optim" in ck:
            self.optim.load_state_dict(ck["optim"])
        self.optim.load_ema_state_dict(self.model, ck.get("ema"))
        self.step = int(ck.get("step", 0))
        if "sampler_epoch" in ck:           # mid-epoch checkpoint (after_warmup.pt, or latest.pt of a max_steps stop)
            self.epoch = int(ck["sampler_epoch"])
            # position = examples of the epoch consumed by ALL ranks (the shard
            # sampler deals the epoch's permutation round-robin, so any world size
            # resumes at the same global position); older files: batches
            if "epoch_examples" in ck:
                self.epoch_pos = int(ck["epoch_examples"]) // max(self.cfg.global_batch, 1)
            elif int(ck.get("world_size", 1)) == self.ctx.world:
                self.epoch_pos = int(ck.get("epoch_pos", 0))
            else:
                self.epoch_pos = 0
        else:                               # end-of-epoch checkpoint (latest.pt) or reference file
            self.epoch = int(ck.get("epoch", -1)) + 1 if "epoch" in ck else 0
            self.epoch_pos = 0
        rng = ck.get("rng")
        if rng is not None and self.ctx.world == int(ck.get("world_size", 1)) and self.ctx.rank < len(rng):
            self.gen.set_state(rng[self.ctx.rank].to(torch.uint8).cpu())
        return True

    def _gather_rng(self):
        """Every rank's generator state (collective: all ranks call it)."""
        st = self.gen.get_state()
        if self.ctx.world == 1:
            return [st]
        import torch.distributed as dist
        out = [None] * self.ctx.world
        dist.all_gather_object(out, st)
        return out

    def sync(self) -> None:
        """Apply an optimizer update the graph-replayed step still holds
        (engine/graphs.py deferred update): afterwards the parameters, moments
        and EMA are those of the last completed step.  Called before anything
        reads them (checkpoints, evaluation, the end of training)."""
        if self._graphed is not None:
            self._graphed.flush()

    def save(self, name: str, epoch: Optional[int] = None, epoch_pos: Optional[int] = None) -> Optional[str]:
        """Collective (every rank calls it: the RNG states are gathered);
        rank 0 writes.  ``epoch``: completed epoch (reference ``latest.pt``);
        ``epoch_pos``: mid-epoch position of the current epoch."""
        self.sync()
        rng = self._gather_rng()
        if not self.ctx.is_main:
            return None
        path = os.path.join(self.out_dir, name)
        extra = {"config": to_dict(self.cfg), "world_size": self.ctx.world, "rng": rng}
        if epoch_pos is not None:
            extra["sampler_epoch"] = int(self.epoch)
            extra["epoch_pos"] = int(epoch_pos)
            extra["epoch_examples"] = int(epoch_pos) * int(self.cfg.global_batch)
        ema = self.optim.ema_state_dict(self.model)
        if ema is not None:
            extra["ema"] = {k: v.cpu() for k, v in ema.items()}
        save_checkpoint(path, self.model, self.optim, self.step, epoch, extra)
        return path

    # ------------------------------------------------------------------
    def step_seed(self, step_word: Optional[int] = None) -> int:
        """64-bit RNG seed of the training-input draw of one step on this
        rank: base + (step * world + rank) * golden (the graph step bakes the
        base and supplies the step word on the device; ops.diffusion_inputs)."""
        base = (self.cfg.seed * 0x2545F4914F6CDD1D + 0x1234567) & 0xFFFFFFFFFFFFFFFF
        if step_word is None:
            step_word = self.step * self.ctx.world + self.ctx.rank
        return (base + step_word * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF

    def diffusion_inputs(self, img, R, T, K, e0: int = 0, step_word: Optional[int] = None):
        """q_sample + CFG dropout (`train.py:80-100`) for examples e0.. of this
        rank's batch, on device: one fused launch on the HIP path.  The draw is
        counter-based in (step seed, example index), so micro-batching and
        graph replay see exactly the numbers of the full-batch eager step."""
        dc = self.cfg.diffusion
        xz, eps, logsnr, keep = ops.diffusion_inputs(img, self.step_seed(step_word), e0, dc.cond_prob,
                                                     dc.logsnr_min, dc.logsnr_max, self.dtype)
        batch = {"xz": xz, "logsnr": logsnr, "R": R, "t": T, "K": K}
        return batch, keep, eps

    def loss_fn(self, img, R, T, K, e0: int = 0, chunk: int = 0) -> torch.Tensor:
        batch, mask, eps = self.diffusion_inputs(img, R, T, K, e0)
        self.model.set_dropout_seed(dropout_word(self.step * self.ctx.world + self.ctx.rank, chunk))
        y = self.model(batch, cond_mask=mask, head_nhwc=True)
        return ops.diff_loss_nhwc(y, eps, self.cfg.diffusion.loss_type)

    last_grad_norm: Optional[torch.Tensor] = None    # device scalar, set when measured / clipping
    last_allreduce_ms: float = 0.0

    def train_step(self, img, R, T, K, want_stats: bool = False) -> torch.Tensor:
        """One optimizer step.  ``want_stats``: also measure the gradient norm
        (``last_grad_norm``) and the time the optimizer waited on the gradient
        all-reduce (``last_allreduce_ms``, device events) -- log steps only."""
        if self.step == self.fault_step and self.ctx.rank == self.fault_rank:
            os._exit(13)  # fault-injection hook for the failure-detection tests
        g = self.optim.param_groups[0]
        if self.sched is None:
            g["lr"] = warmup_lr(self.step, self.warmup_steps, self.cfg.optim.lr)
        if self.cfg.graph and self.device.type == "cuda" and self.sink is not None:
            from .graphs import GraphCaptureError
            try:
                return self._graph_train_step(img, R, T, K, want_stats)
            except GraphCaptureError as e:
                # every rank raises together (GraphedTrainStep.capture): all
                # continue with the eager step
                if self.ctx.is_main:
                    print(f"[trainer] HIP-graph capture failed ({e}); continuing with the eager step", flush=True)
                self.sync()
                self.cfg.graph = False
                self._graphed = None
        if not self.model.training:
            self.model.train()
        if self.sink is not None:
            self.sink.reset()
        B = img.shape[0]
        mb = self.cfg.micro_batch if 0 < self.cfg.micro_batch < B else B
        chunks = [(s, min(s + mb, B)) for s in range(0, B, mb)]
        total = None
        with range_push("fwd_bwd"):
            for ci, (s, e) in enumerate(chunks):
                last_chunk = ci == len(chunks) - 1
                ctx = self.reducer.no_sync() if (self.reducer is not None and not last_chunk) else _null()
                with ctx:
                    loss = self.loss_fn(img[s:e], R[s:e], T[s:e], K[s:e], e0=s, chunk=ci)
                    (loss * ((e - s) / B)).backward() if len(chunks) > 1 else loss.backward()
                l = loss.detach() * ((e - s) / B)
                total = l if total is None else total + l
        loss = total
        timing = want_stats and self.device.type == "cuda" and self.reducer is not None
        if timing:
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record()
        t_host = time.perf_counter()
        if self.reducer is not None:
            with range_push("allreduce_wait"):
                self.reducer.finish()
        if want_stats and self.device.type != "cuda":
            self.last_allreduce_ms = 1e3 * (time.perf_counter() - t_host)     # gloo: host-blocking wait
        if timing:
            ev1.record()
        scale = 1.0 / self.ctx.world
        clip = self.cfg.optim.grad_clip
        norm = self.optim.grad_norm(scale) if (want_stats or clip > 0) else None
        if norm is not None:
            self.last_grad_norm = norm
        with range_push("optimizer"):
            self.optim.step(grad_scale=scale, max_norm=clip, norm=norm)
            self.optim.zero_grad()
        if timing:
            ev1.synchronize()
            self.last_allreduce_ms = ev0.elapsed_time(ev1)
        if self.sched is not None:
            self.sched.step()
        self.step += 1
        ce = self.cfg.dist.checksum_every
        if ce and self.step % ce == 0 and not check_replicas_in_sync(self.flat):
            raise RuntimeError(f"data-parallel replicas diverged at step {self.step}")
        return loss

    _graphed = None

    def _graph_train_step(self, img, R, T, K, want_stats: bool = False) -> torch.Tensor:
        """Same step, replayed from captured HIP graphs (engine/graphs.py)."""
        from .graphs import GraphedTrainStep
        B = img.shape[0]
        mb = self.cfg.micro_batch if 0 < self.cfg.micro_batch < B else B
        if self._graphed is None or self._graphed.mb != mb:
            self.sync()
            self._graphed = GraphedTrainStep(self, mb, (img, R, T, K))
        if not self.model.training:       # (a full module walk: ~1-2 ms of host time at the step boundary)
            self.model.train()
        loss = self._graphed.step(img, R, T, K, want_norm=want_stats)
        if self.sched is not None:
            self.sched.step()
        self.step += 1
        ce = self.cfg.dist.checksum_every
        if ce and self.step % ce == 0 and not check_replicas_in_sync(self.flat):
            raise RuntimeError(f"data-parallel replicas diverged at step {self.step}")
        return loss

    # ------------------------------------------------------------------
    def make_data(self) -> Tuple[Iterator, Optional[object], Optional[object]]:
        dc = self.cfg.data
        if dc.synthetic:
            from ..data import SyntheticBatches
            it = SyntheticBatches(self.local_batch, dc.imgsize, self.device,
                                  seed=dc.seed * 7919 + self.ctx.rank)
            return it, None, None
        from ..data import SRNDataset, ShardSampler, MultiEpochsDataLoader, CachedSRNDataset, CachedBatchLoader
        if dc.cache:
            ds = CachedSRNDataset("train", dc.cache, seed=dc.seed)
        else:
            ds = SRNDataset("train", dc.path, dc.index, dc.imgsize, seed=dc.seed)
        sampler = ShardSampler(len(ds), self.ctx.rank, self.ctx.world, shuffle=True, seed=dc.seed,
                               with_epoch=True)
        if dc.cache:
            # batch-level mmap gather + uint8 pinned H2D one step ahead (data/fastloader.py)
            return CachedBatchLoader(ds, self.local_batch, sampler, self.device), ds, sampler
        loader = MultiEpochsDataLoader(ds, batch_size=self.local_batch, sampler=sampler,
                                       num_workers=dc.num_workers, drop_last=True,
                                       pin_memory=self.device.type == "cuda")
        return loader, ds, sampler

    def _to_dev(self, batch):
        return tuple(b.to(self.device, non_blocking=True) for b in batch)

    def fit(self, steps_per_epoch: int = 0) -> Dict[str, float]:
        cfg = self.cfg
        data, ds, sampler = self.make_data()
        if cfg.optim.warmup_examples < 0:
            # one pass over the training set (Lightning: n_samples / batch_size steps)
            n = len(ds) if ds is not None else cfg.global_batch
            self.warmup_steps = n / cfg.global_batch
        timer = StepTimer(cfg.global_batch, train_flops_per_example(cfg.model.H), self.device)
        timer.start()
        last = {}
        done = False
        for epoch in range(self.epoch, cfg.num_epochs):
            self.epoch = epoch
            n = self.epoch_pos                # > 0 only for the epoch a mid-epoch checkpoint resumes
            if sampler is not None:
                sampler.set_epoch(epoch, start=n * self.local_batch)
                ds.set_epoch(epoch)
            self.epoch_pos = 0
            it = iter(data)
            data_wait = 0.0
            while True:
                if steps_per_epoch and n >= steps_per_epoch:
                    break
                t_wait = time.perf_counter()
                try:
                    batch = next(it)
                except StopIteration:
                    break
                data_wait += time.perf_counter() - t_wait
                self._profile_hook(self.step)
                log_now = bool(cfg.log_every) and (self.step + 1) % cfg.log_every == 0
                loss = self.train_step(*self._to_dev(batch), want_stats=log_now)
                timer.tick()
                n += 1
                if log_now:
                    lv = float(loss)
                    check_finite(loss, self.step)
                    rep = timer.report()
                    gn = float(self.last_grad_norm) if self.last_grad_norm is not None else float("nan")
                    last = {"step": self.step, "epoch": epoch, "loss": lv,
                            "lr": self.optim.param_groups[0]["lr"], **rep, "grad_norm": gn,
                            "allreduce_wait_ms": self.last_allreduce_ms,
                            "data_wait_ms": 1e3 * data_wait / max(rep["steps"], 1),
                            "hbm_peak_gib": (torch.cuda.max_memory_allocated(self.device) / 2 ** 30
                                             if self.device.type == "cuda" else 0.0)}
                    data_wait = 0.0
                    if self.ctx.is_main:
                        print(f"[step {self.step}] loss {lv:.5f} {rep['examples_per_s']:.1f} ex/s "
                              f"{rep['tflops']:.1f} TFLOP/s", flush=True)
                        self.logger.log(**last)
                    timer.start()
                if cfg.ckpt_every and self.step % cfg.ckpt_every == 0:
                    self.save("after_warmup.pt", epoch_pos=n)
                if cfg.max_steps and self.step >= cfg.max_steps:
                    done = True
                    break
            if done:
                # stopped inside the epoch: latest.pt records the position, so a
                # resume continues this epoch instead of skipping its remainder
                self.save("latest.pt", epoch=epoch - 1, epoch_pos=n)     # epoch: the last completed one
                break
            self.save("latest.pt", epoch=epoch)
        self.sync()
        self._profile_hook(None)
        self.logger.close()
        return last

    _prof = None

    def _profile_hook(self, step) -> None:
        """``profile_steps="a-b"``: torch.profiler (roctracer) over steps [a, b);
        rank 0 writes <out_dir>/profile_rank0.txt (kernel table)."""
        spec = self.cfg.profile_steps
        if not spec:
            return
        a, b = (int(v) for v in spec.split("-"))
        if step is not None and step == a and self._prof is None:
            acts = [torch.profiler.ProfilerActivity.CPU]
            if self.device.type == "cuda":
                acts.append(torch.profiler.ProfilerActivity.CUDA)
            self._prof = torch.profiler.profile(activities=acts)
            self._prof.__enter__()
        elif self._prof is not None and (step is None or step >= b):
            self._prof.__exit__(None, None, None)
            if self.ctx.is_main:
                os.makedirs(self.out_dir, exist_ok=True)
                with open(os.path.join(self.out_dir, f"profile_rank{self.ctx.rank}.txt"), "w") as f:
                    key = "cuda_time_total" if self.device.type == "cuda" else "cpu_time_total"
                    f.write(self._prof.key_averages().table(sort_by=key, row_limit=80))
            self._prof = None
