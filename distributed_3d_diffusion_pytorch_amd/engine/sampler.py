"""Stochastic-conditioning CFG ancestral sampler (reference:
`sampling.py:78-184`, `train.py:118-166`).

Differences by design (same math, §2.5 of SURVEY):
* everything stays on the device (the reference moves eps to the CPU and does
  the posterior there, two host syncs per step, D11);
* the conditional and unconditional CFG passes run as ONE 2b-batch forward;
* the b guidance-scale chains are independent given the shared stochastic
  conditioning choice, so multi-GPU sampling shards the chains over ranks
  (one process per GPU) instead of ``nn.DataParallel`` replicating 521 MiB of
  weights on every forward (`sampling.py:52`); the record choice RNG is seeded
  identically on every rank so all shards condition on the same view index;
* D9 (noise skipped at t=0.5 where logsnr_next == 0) is opt-in via
  ``ref_quirk``; default adds noise on every step but the last.
"""
from __future__ import annotations

import random
from typing import List, Optional, Sequence, Tuple

import torch

from ..diffusion import logsnr_schedule_cosine, sampler_logsnrs, cfg_posterior


class RecordEntry:
    """One conditioning candidate: images [b,3,H,W] (per-chain), R [3,3], T [3]."""

    def __init__(self, img: torch.Tensor, R: torch.Tensor, T: torch.Tensor):
        self.img, self.R, self.T = img, R, T


class DiffusionSampler:
    def __init__(self, model: torch.nn.Module, timesteps: int = 256, ref_quirk: bool = False,
                 logsnr_min: float = -20.0, logsnr_max: float = 20.0, seed: int = 0, device=None):
        self.model = model
        self.T = timesteps
        self.ref_quirk = ref_quirk
        self.lmin, self.lmax = logsnr_min, logsnr_max
        self.device = device or next(model.parameters()).device
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed)
        self._cpu_gen = torch.Generator()
        self._cpu_gen.manual_seed(seed + 1)
        self.choice_rng = random.Random(seed)
        lam, lam_next = sampler_logsnrs(timesteps, logsnr_min, logsnr_max)
        self.lam, self.lam_next = lam.tolist(), lam_next.tolist()
        self.lam0 = float(logsnr_schedule_cosine(torch.zeros(()), logsnr_min=logsnr_min, logsnr_max=logsnr_max))

    @torch.no_grad()
    def denoise_eps(self, x_cond, z, R, T, K, logsnr: float):
        """CFG pair in one forward: rows [0,b) conditional, [b,2b) unconditional
        (x replaced by noise, rays zeroed via cond_mask=False)."""
        b = z.shape[0]
        dev = z.device
        x_unc = torch.randn(x_cond.shape, generator=self.gen, device=dev, dtype=x_cond.dtype)
        lam = torch.full((2 * b,), float(logsnr), device=dev)
        batch = {"x": torch.cat([x_cond, x_unc]), "z": torch.cat([z, z]),
                 "logsnr": torch.stack([torch.full_like(lam, self.lam0), lam], 1),
                 "R": torch.cat([R, R]), "t": torch.cat([T, T]), "K": torch.cat([K, K])}
        mask = torch.cat([torch.ones(b, dtype=torch.bool, device=dev), torch.zeros(b, dtype=torch.bool, device=dev)])
        eps = self.model(batch, cond_mask=mask).float()
        return eps[:b], eps[b:]

    @torch.no_grad()
    def step(self, z, x_cond, R, T, K, w, k: int):
        lam, lam_next = self.lam[k], self.lam_next[k]
        eps_c, eps_u = self.denoise_eps(x_cond, z, R, T, K, lam)
        if self.ref_quirk:
            add_noise = lam_next != 0.0
        else:
            add_noise = k < self.T - 1
        from .. import ops
        if z.is_cuda and ops.use_hip(z, any_dtype=True):
            # fused on-device CFG combine + x0 clamp + posterior + noise
            # (the reference does this on the CPU, two host syncs per step)
            import math
            from ..ops import hip_impl
            c = -math.expm1(lam - lam_next)
            sig = lambda x: 1.0 / (1.0 + math.exp(-x))  # noqa: E731
            seed = int(torch.randint(0, 2 ** 62, (1,), generator=self._cpu_gen).item())
            return hip_impl.sampler_step(z.contiguous(), eps_c, eps_u, w, math.sqrt(sig(lam)), math.sqrt(sig(-lam)),
                                         math.sqrt(sig(lam_next)), c, math.sqrt(sig(-lam_next) * c), add_noise, seed)
        mean, var = cfg_posterior(z, eps_c, eps_u, w, torch.tensor(lam), torch.tensor(lam_next))
        if not add_noise:
            return mean
        return mean + var.sqrt() * torch.randn(z.shape, generator=self.gen, device=z.device)

    @torch.no_grad()
    def sample(self, record: List[RecordEntry], target_R: torch.Tensor, target_T: torch.Tensor,
               K: torch.Tensor, w: torch.Tensor, progress: bool = False) -> torch.Tensor:
        """Generate the view at (target_R, target_T) for each of the b chains;
        each step conditions on a random entry of ``record`` (stochastic
        conditioning, `sampling.py:137-145`)."""
        model_was_training = self.model.training
        self.model.eval()
        b = w.shape[0]
        dev = self.device
        H, W = record[0].img.shape[-2:]
        z = torch.randn((b, 3, H, W), generator=self.gen, device=dev)
        Kb = K.to(dev).reshape(1, 3, 3).expand(b, 3, 3).contiguous()
        w = w.to(dev).float()
        it = range(self.T)
        if progress:
            try:
                from tqdm import tqdm
                it = tqdm(it, desc="diffusion", leave=False)
            except Exception:
                pass
        for k in it:
            e = record[self.choice_rng.randrange(len(record))]
            R = torch.stack([e.R.to(dev), target_R.to(dev)], 0)[None].expand(b, 2, 3, 3).contiguous()
            T = torch.stack([e.T.to(dev), target_T.to(dev)], 0)[None].expand(b, 2, 3).contiguous()
            z = self.step(z, e.img.to(dev), R, T, Kb, w, k)
        if model_was_training:
            self.model.train()
        return z


def shard_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous, disjoint, covering split of n chains over ranks."""
    base, rem = divmod(n, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)
