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
  [world > 1] eager RCCL all-reduce of the flat gradient in D3D_AR_CHUNKS
      (default 4) async collectives, each chunk's Adam launched as soon as
      its collective lands, so the optimizer pass (~0.7 ms) hides behind the
      remaining chunks' reduction (~3 ms for 547 MB over xGMI against a ~33
      ms step), then the batched weight repack and the zeroing.  (The graph
      cannot hold the hook-driven bucketed launches of the eager step.)
  graph B (world == 1): fused Adam reading its per-step hyper-parameters
      from a device block (lr warmup / bias correction change every step) ->
      batched weight repack -> gradient / loss-accumulator zeroing.

Per-step values that a replay cannot see from Python travel through device
words refreshed before the replays: the dropout seed (``hip_impl._SEED_DEV``,
added to every mask kernel's baked seed) and the Adam block ``hp``.
"""
from __future__ import annotations

import math
import os
from typing import Optional

import torch
import torch.distributed as dist


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
        self.loss_acc = torch.zeros((), device=dev)
        self.seed = torch.zeros(1, dtype=torch.int64, device=dev)
        self.hp = torch.zeros(8, device=dev)
        self.pool = torch.cuda.graph_pool_handle()
        self.gA: Optional[torch.cuda.CUDAGraph] = None
        self.gB: Optional[torch.cuda.CUDAGraph] = None

    # ------------------------------------------------------------------
    def _body(self) -> None:
        tr = self.tr
        if tr.sink is not None:
            tr.sink.reset()
        batch, mask, eps = tr.diffusion_inputs(self.img, self.R, self.T, self.K)
        eps_hat = tr.model(batch, cond_mask=mask)
        from ..diffusion import diffusion_loss
        loss = diffusion_loss(eps, eps_hat, tr.cfg.diffusion.loss_type)
        (loss * self.frac).backward()
        self.loss_acc.add_(loss.detach() * self.frac)

    def _update(self) -> None:
        o = self.tr.optim
        self.H.adam_flat_dev(o.flat.data, o.flat.grad, o.exp_avg, o.exp_avg_sq, o.ema, self.hp)
        o.flat.grad.zero_()
        self.loss_acc.zero_()

    def capture(self) -> None:
        tr = self.tr
        tr.model.train()
        tr.model.set_dropout_seed(0)             # baked; the per-step part is self.seed
        self.H.set_device_seed(self.seed)
        if tr.reducer is not None:
            tr.reducer.enabled = False           # the all-reduce runs between the graphs
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
                self._body()
        torch.cuda.current_stream().wait_stream(s)
        self.H.refresh_weights()                 # descriptor table final before capture
        torch.cuda.synchronize()
        self.gA = torch.cuda.CUDAGraph()
        self.gA.register_generator_state(tr.gen)
        with torch.cuda.graph(self.gA, pool=self.pool):
            self._body()
        self.gB = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.gB, pool=self.pool):
            self._update()
        torch.cuda.synchronize()
        tr.gen.set_state(gstate)
        # warm-up / capture left partial gradients behind
        tr.flat.zero_grad()
        self.loss_acc.zero_()

    # ------------------------------------------------------------------
    def _hparams(self, grad_scale: float) -> torch.Tensor:
        o = self.tr.optim
        g = o.param_groups[0]
        lr, (b1, b2), eps, wd = g["lr"], g["betas"], g["eps"], g["weight_decay"]
        o.step_count += 1
        t = o.step_count
        bc1 = 1.0 - b1 ** t
        bc2_sqrt = math.sqrt(1.0 - b2 ** t)
        return torch.tensor([b1, b2, eps, wd, lr / bc1, bc2_sqrt, grad_scale, 1.0 - o.ema_decay],
                            dtype=torch.float32)

    def _reduce_update_chunked(self) -> None:
        """fp32 all-reduce in chunks, each chunk's Adam behind its own
        collective (overlaps the optimizer with the remaining reduction)."""
        o = self.tr.optim
        p, g, m, v, ema = o.flat.data, o.flat.grad, o.exp_avg, o.exp_avg_sq, o.ema
        n = g.numel()
        k = max(1, int(os.environ.get("D3D_AR_CHUNKS", "4")))
        cuts = [0] + [min(n, (n * i // k + 255) // 256 * 256) for i in range(1, k)] + [n]
        spans = [(a, b) for a, b in zip(cuts[:-1], cuts[1:]) if b > a]
        works = [dist.all_reduce(g[a:b], async_op=True) for a, b in spans]
        for (a, b), w in zip(spans, works):
            w.wait()
            self.H.adam_flat_dev(p[a:b], g[a:b], m[a:b], v[a:b], ema[a:b] if ema is not None else None, self.hp,
                                 refresh=False)
        self.H.refresh_weights()
        g.zero_()
        self.loss_acc.zero_()

    def step(self, img, R, T, K) -> torch.Tensor:
        tr = self.tr
        if self.gA is None:
            self.capture()
        B = img.shape[0]
        mb = self.mb
        assert B % mb == 0, (B, mb)
        self.seed.fill_(tr.step * tr.ctx.world + tr.ctx.rank + 1)
        nchunks = B // mb
        self.frac.fill_(1.0 / nchunks)
        for s in range(0, B, mb):
            self.img.copy_(img[s:s + mb])
            self.R.copy_(R[s:s + mb])
            self.T.copy_(T[s:s + mb])
            self.K.copy_(K[s:s + mb])
            self.gA.replay()
        loss = self.loss_acc.clone()
        if tr.ctx.world > 1:
            g = tr.flat.grad
            if tr.cfg.dist.grad_dtype == "bf16":
                gb = g.to(torch.bfloat16)
                dist.all_reduce(gb)
                g.copy_(gb)
            else:
                self.hp.copy_(self._hparams(1.0 / tr.ctx.world))
                self._reduce_update_chunked()
                for cb in tr.optim.on_step:
                    cb()
                return loss
        self.hp.copy_(self._hparams(1.0 / tr.ctx.world))
        self.gB.replay()
        for cb in tr.optim.on_step:
            cb()
        return loss
