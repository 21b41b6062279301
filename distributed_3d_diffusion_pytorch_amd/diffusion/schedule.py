"""Continuous-time DDPM math (cosine logSNR schedule, forward noising,
ancestral CFG posterior).

Parity targets (all device-agnostic here; the reference runs parts of this on
the CPU, D11):
  * logsnr_schedule_cosine  -> `train.py:30-34` (dupes `sampling.py:59-63`)
  * q_sample                -> `train.py:50-60`
  * cfg posterior           -> `train.py:131-166`, `sampling.py:78-112`
  * ancestral step          -> `train.py:118-128`, `sampling.py:115-127`
The on-device fused forms are ``ops.diffusion_inputs`` (t, lambda, eps, q_sample and CFG drop in
one launch) and the sampler kernels driven by ``engine.sampler`` (CFG combine, x0 clamp,
posterior and noise in one launch per step).
"""
from __future__ import annotations

import math
from typing import Tuple

import torch


def _ab(logsnr_min: float, logsnr_max: float) -> Tuple[float, float]:
    b = math.atan(math.exp(-0.5 * logsnr_max))
    a = math.atan(math.exp(-0.5 * logsnr_min)) - b
    return a, b


def logsnr_schedule_cosine(t: torch.Tensor, *, logsnr_min: float = -20.0,
                           logsnr_max: float = 20.0) -> torch.Tensor:
    """lambda(t) = -2 log tan(a t + b);  lambda(0)=+20, lambda(1)~-20."""
    a, b = _ab(logsnr_min, logsnr_max)
    return -2.0 * torch.log(torch.tan(a * t + b))


def alpha_sigma(logsnr: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """alpha = sqrt(sigmoid(l)), sigma = sqrt(sigmoid(-l))."""
    return torch.sigmoid(logsnr).sqrt(), torch.sigmoid(-logsnr).sqrt()


def q_sample(z: torch.Tensor, logsnr: torch.Tensor, noise: torch.Tensor) -> torch.Tensor:
    """z_t = alpha(l) z + sigma(l) eps with per-example logsnr [B]."""
    alpha, sigma = alpha_sigma(logsnr)
    shape = (-1,) + (1,) * (z.dim() - 1)
    return alpha.view(shape) * z + sigma.view(shape) * noise


def diffusion_loss(eps: torch.Tensor, eps_hat: torch.Tensor, loss_type: str = "l2") -> torch.Tensor:
    eps_hat = eps_hat.float()
    eps = eps.float()
    if loss_type == "l2":
        return torch.mean((eps - eps_hat) ** 2)
    if loss_type == "l1":
        return torch.mean((eps - eps_hat).abs())
    if loss_type == "huber":
        return torch.nn.functional.smooth_l1_loss(eps_hat, eps)
    raise NotImplementedError(loss_type)


def sampler_logsnrs(timesteps: int, logsnr_min: float = -20.0, logsnr_max: float = 20.0,
                    dtype=torch.float32) -> Tuple[torch.Tensor, torch.Tensor]:
    """(lambda_k, lambda_{k+1}) for t_k = 1 - k/T, k=0..T-1 (`sampling.py:134-135`)."""
    ts = torch.linspace(1.0, 0.0, timesteps + 1, dtype=dtype)
    lam = logsnr_schedule_cosine(ts, logsnr_min=logsnr_min, logsnr_max=logsnr_max)
    return lam[:-1], lam[1:]


def cfg_posterior(z: torch.Tensor, eps_cond: torch.Tensor, eps_uncond: torch.Tensor,
                  w: torch.Tensor, logsnr: torch.Tensor, logsnr_next: torch.Tensor
                  ) -> Tuple[torch.Tensor, torch.Tensor]:
    """Classifier-free-guided DDPM posterior mean / variance (reference math,
    `train.py:140-166`).  ``w`` is per-example [b]; logsnr scalars."""
    shape = (-1,) + (1,) * (z.dim() - 1)
    w = w.to(z.dtype).view(shape)
    logsnr = torch.as_tensor(logsnr, dtype=z.dtype, device=z.device)
    logsnr_next = torch.as_tensor(logsnr_next, dtype=z.dtype, device=z.device)
    c = -torch.expm1(logsnr - logsnr_next)
    alpha, sigma = alpha_sigma(logsnr)
    alpha_next = torch.sigmoid(logsnr_next).sqrt()
    eps = (1.0 + w) * eps_cond - w * eps_uncond
    x0 = ((z - sigma * eps) / alpha).clamp(-1.0, 1.0)
    mean = alpha_next * (z * (1.0 - c) / alpha + c * x0)
    var = torch.sigmoid(-logsnr_next) * c
    return mean, var
