"""``Diff3D``: the reference's LightningModule API (`lightning/diff3d.py:9-238`)
on top of this framework's components.

PyTorch Lightning is not part of the stack (and not installed); ``Diff3D`` is a
plain ``nn.Module`` exposing the same methods so code written against the
reference keeps working:

  forward(in_x, noise=None, cond_prob=0.1)   noised target + CFG drop -> eps-hat
  training_step(batch, batch_idx, loss_type) warmup + zero_grad + loss (Lightning
                                             would then backward/step; use
                                             ``fit_step`` to do all of it here)
  configure_optimizers()                     fused Adam (+ CosineAnnealingLR)
  warmup()                                   linear warmup over n_samples/batch_size steps
  sample(...), p_mean_variance(...), p_sample(...)   CFG ancestral sampler
  logsnr_schedule_cosine / xt2batch / q_sample        diffusion helpers

Differences by design: the network runs on this framework's NHWC/HIP path,
the optimizer is the flat-buffer fused Adam, and ``sample`` works (the
reference's version uses un-imported ``tqdm``/``time``, D13).
"""
from __future__ import annotations

import operator

from typing import Optional

import torch
import torch.nn as nn

from ..diffusion import logsnr_schedule_cosine as _sched, q_sample as _q, diffusion_loss, cfg_posterior
from ..engine.optim import FusedAdam, warmup_lr
from ..engine.sampler import DiffusionSampler, RecordEntry
from ..models import XUNet
from ..parallel.flat import FlatParams
from ..utils import load_checkpoint, load_model_weights


class Diff3D(nn.Module):
    def __init__(self, pretrained_model: Optional[str] = None, n_samples: int = 10_000_000, image_size: int = 64,
                 batch_size: int = 128, lr: float = 1e-4, use_scheduler: bool = False):
        super().__init__()
        self.n_samples = n_samples
        self.batch_size = batch_size
        self.image_size = image_size
        self.lr = lr
        self.use_scheduler = use_scheduler
        self.step = 0
        self.xunet_denoiser = XUNet(H=image_size, W=image_size, ch=128)
        self.pretrained_optim = None
        self._opt = None
        self._sched = None
        if pretrained_model is not None:
            ck = load_checkpoint(pretrained_model)
            load_model_weights(self.xunet_denoiser, ck["model"])
            self.pretrained_optim = ck.get("optim")

    @property
    def device(self):
        return next(self.parameters()).device

    # ---------------------------------------------------------- diffusion --
    @staticmethod
    def logsnr_schedule_cosine(t, logsnr_min: float = -20.0, logsnr_max: float = 20.0):
        return _sched(t, logsnr_min=logsnr_min, logsnr_max=logsnr_max)

    @staticmethod
    def q_sample(z, logsnr, noise):
        return _q(z, logsnr, noise)

    def xt2batch(self, x, logsnr, z, R, T, K):
        dev = self.device
        lam0 = self.logsnr_schedule_cosine(torch.zeros_like(logsnr))
        if K.dim() == 2:
            K = K[None].expand(x.shape[0], 3, 3)
        return {"x": x.to(dev), "z": z.to(dev), "logsnr": torch.stack([lam0, logsnr], 1).to(dev),
                "R": R.to(dev), "t": T.to(dev), "K": K.to(dev)}

    # ------------------------------------------------------------ training --
    def forward(self, in_x, noise=None, cond_prob: float = 0.1):
        img, R, T, K = in_x
        dev = self.device
        img = img.to(dev)
        B = img.shape[0]
        x, z = img[:, 0], img[:, 1]
        logsnr = self.logsnr_schedule_cosine(torch.rand(B, device=dev))
        if noise is None:
            noise = torch.randn_like(x)
        z_noisy = self.q_sample(z, logsnr, noise)
        cond_mask = torch.rand(B, device=dev) > cond_prob
        x_cond = torch.where(cond_mask[:, None, None, None], x, torch.randn_like(x))
        batch = self.xt2batch(x_cond, logsnr, z_noisy, R, T, K)
        return self.xunet_denoiser(batch, cond_mask=cond_mask)

    def configure_optimizers(self):
        if self._opt is None:
            self._flat = FlatParams(list(self.xunet_denoiser.parameters()))
            self._opt = FusedAdam(self._flat, lr=self.lr, betas=(0.9, 0.99))
            if self.pretrained_optim is not None:
                self._opt.load_state_dict(self.pretrained_optim)
            if self.use_scheduler:
                self._sched = torch.optim.lr_scheduler.CosineAnnealingLR(self._opt, T_max=300)
        return ([self._opt], [self._sched]) if self._sched is not None else [self._opt]

    def optimizers(self):
        self.configure_optimizers()
        return self._opt

    def warmup(self):
        """lr = step / (n_samples/batch_size) * lr until warm (`lightning/diff3d.py:118-127`)."""
        self.optimizers().param_groups[0]["lr"] = warmup_lr(self.step, self.n_samples / self.batch_size, self.lr)

    def training_step(self, batch, batch_idx: int = 0, loss_type: str = "l2"):
        if not self.use_scheduler:
            self.warmup()
        self.optimizers().zero_grad()
        noise = torch.randn_like(batch[0][:, 0].to(self.device))
        pred = self.forward(batch, noise=noise)
        loss = diffusion_loss(noise, pred, loss_type)
        self.step += 1
        if self.use_scheduler and self._sched is not None:
            self._sched.step()
        return loss

    def fit_step(self, batch, loss_type: str = "l2") -> float:
        """training_step + backward + optimizer step (what Lightning would do)."""
        loss = self.training_step(batch, loss_type=loss_type)
        loss.backward()
        self.optimizers().step()
        return float(loss)

    # ------------------------------------------------------------ sampling --
    @torch.no_grad()
    def p_mean_variance(self, x, z, R, T, K, logsnr, logsnr_next, w):
        b = z.shape[0]
        smp = DiffusionSampler(self.xunet_denoiser, 1, device=self.device)
        Kb = K if K.dim() == 3 else K[None].expand(b, 3, 3)
        ec, eu = smp.denoise_eps(x, z, R, T, Kb, float(logsnr))
        return cfg_posterior(z, ec, eu, w, torch.as_tensor(logsnr), torch.as_tensor(logsnr_next))

    @torch.no_grad()
    def p_sample(self, x, z, R, T, K, logsnr, logsnr_next, w):
        mean, var = self.p_mean_variance(x, z, R, T, K, logsnr, logsnr_next, w)
        if float(logsnr_next) == 0.0:
            return mean
        return mean + var.sqrt() * torch.randn_like(z)

    @torch.no_grad()
    def sample(self, model=None, img=None, R=None, T=None, K=None, w=None, timesteps: int = 256, *,
               return_all: bool = True):
        """Fixed-conditioning CFG sampler with the reference's signature
        (`lightning/diff3d.py:151-166`): ``sample(model, img, R, T, K, w,
        timesteps)``.  ``img`` [b, 2, 3, H, W] (frame 0 is the conditioning
        view, as the reference reads ``img[:, 0]``) or [b, 3, H, W]; ``R`` /
        ``T`` PER EXAMPLE [b, 2, ...] (condition, target) poses; ``K`` [3, 3]
        or [b, 3, 3]; ``w`` a scalar or one guidance weight per example;
        ``model`` None -> this module's denoiser.  Returns the per-step images
        (numpy [b, 3, H, W] each, like the reference) or, with
        ``return_all=False``, the final image tensor.  The call without the
        model argument, ``sample(img, R, T, K, w, timesteps)``, is accepted
        too (every positional argument shifts by one, the step count
        included).  Note the return type: the per-step list by default (as
        the reference), the final tensor only with ``return_all=False``."""
        if isinstance(model, torch.Tensor):
            if K is None:
                # sample(img, R, T, K, w=...): the keyword w lands in the wrong slot of the shifted form
                raise TypeError("sample(img, R, T, K, w, timesteps): in the model-less form pass w (and "
                                "timesteps) positionally, or call sample(None, img, R, T, K, w=..., timesteps=...)")
            if w is not None:
                if isinstance(w, bool):
                    raise TypeError("sample(img, R, T, K, w, timesteps): timesteps must be an integer, got bool")
                try:
                    timesteps = operator.index(w)      # int, numpy integers, 0-d integer tensors
                except TypeError:
                    raise TypeError("sample(img, R, T, K, w, timesteps): timesteps must be an integer, "
                                    f"got {type(w).__name__}") from None
            model, img, R, T, K, w = None, model, img, R, T, K
        net = model if model is not None else self.xunet_denoiser
        dev = next(net.parameters()).device
        x = (img[:, 0] if img.dim() == 5 else img).to(dev).float()
        b = x.shape[0]
        R = R.to(dev).float()
        T = T.to(dev).float()
        K = K.to(dev).float()
        Kb = K if K.dim() == 3 else K[None].expand(b, 3, 3).contiguous()
        wt = torch.as_tensor(w, dtype=torch.float32, device=dev).reshape(-1)
        wt = wt.expand(b).contiguous() if wt.numel() == 1 else wt
        smp = DiffusionSampler(net, timesteps, device=dev)
        z = torch.randn_like(x)
        imgs = []
        for k in range(timesteps):
            z = smp.step(z, x, R, T, Kb, wt, k)
            if return_all:
                imgs.append(z.float().cpu().numpy())
        return imgs if return_all else z.float()
