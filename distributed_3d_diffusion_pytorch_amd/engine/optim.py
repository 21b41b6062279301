"""Fused Adam over the flat parameter buffer (+ EMA, warmup, cosine LR).

Reference: ``Adam(lr=1e-4, betas=(0.9, 0.99))`` (`train.py:235`,
`lightning/diff3d.py:106`) run as torch's multi-tensor Adam over 647 tensors;
linear warmup (`train.py:169-177`, `lightning/diff3d.py:118-127`); optional
``CosineAnnealingLR(T_max=300)`` (`lightning/diff3d.py:111-113`); EMA is
documented but not implemented upstream (D16).

Here the whole update -- gradient averaging (``grad_scale = 1/world``), both
moments, bias correction, parameter write and optional EMA -- is ONE HIP kernel
launch over the contiguous fp32 buffers (``adam_flat`` in the native library).
The arithmetic follows ``torch.optim.Adam`` exactly (same operation order), and
``state_dict()`` / ``load_state_dict()`` speak torch Adam's format with
parameters indexed in ``model.parameters()`` order, so reference optimizer
checkpoints load unchanged.
"""
from __future__ import annotations

import math
import os
from typing import Optional

import torch

from ..parallel.flat import FlatParams

FUSED_UPDATE = True      # Adam + operand repack in one pass (hip_impl.adam_update_all)


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, flat: FlatParams, lr: float = 1e-4, betas=(0.9, 0.99), eps: float = 1e-8,
                 weight_decay: float = 0.0, ema_decay: float = 0.0):
        defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay, amsgrad=False,
                        maximize=False, foreach=None, capturable=False, differentiable=False, fused=None)
        super().__init__(flat.params, defaults)
        self.flat = flat
        self.exp_avg = torch.zeros_like(flat.data)
        self.exp_avg_sq = torch.zeros_like(flat.data)
        self.step_count = 0
        self.ema_decay = float(ema_decay)
        self.ema: Optional[torch.Tensor] = flat.data.clone() if ema_decay > 0 else None
        self.on_step = []          # callbacks run after each update (weight caches)
        # the fused HIP update also zeroes the gradient (callers that always
        # zero_grad() right after step(), e.g. engine.Trainer, turn this on)
        self.zero_in_step = False
        self._grad_zeroed = False

    # ------------------------------------------------------------------
    def zero_grad(self, set_to_none: bool = False) -> None:  # noqa: D401 - torch API
        if self._grad_zeroed:
            # the fused update of step() already left the gradient zeroed (one
            # pass over the flat buffer instead of an extra 521 MiB fill)
            self._grad_zeroed = False
            return
        self.flat.zero_grad()

    def grad_norm(self, grad_scale: float = 1.0) -> torch.Tensor:
        """L2 norm of the (averaged) flat gradient, as a device scalar (no sync)."""
        return torch.linalg.vector_norm(self.flat.grad, dtype=torch.float32) * grad_scale

    def hparams_list(self, grad_scale: float) -> list:
        """Advance the step counter and return the per-step hyper-parameter
        block of the device-side Adam kernel (adam.hip ``d3d_adam_dev``):
        [b1, b2, eps, wd, lr/bc1, sqrt(bc2), grad_scale, 1-ema_decay]."""
        g = self.param_groups[0]
        lr, (b1, b2), eps, wd = g["lr"], g["betas"], g["eps"], g["weight_decay"]
        self.step_count += 1
        t = self.step_count
        return [b1, b2, eps, wd, lr / (1.0 - b1 ** t), math.sqrt(1.0 - b2 ** t), grad_scale, 1.0 - self.ema_decay]

    def hparams(self, grad_scale: float) -> torch.Tensor:
        """:meth:`hparams_list` as a host fp32 tensor."""
        return torch.tensor(self.hparams_list(grad_scale), dtype=torch.float32)

    def hparams_to(self, dst: torch.Tensor, grad_scale: float) -> torch.Tensor:
        """Write the block into the device tensor ``dst`` without a host-to-
        device copy (a kernel carries the values), so the host keeps running
        ahead of the GPU across the optimizer step."""
        from ..ops import hip_impl
        return hip_impl.set_words(dst, self.hparams_list(grad_scale))

    @staticmethod
    def clip_coef(norm: torch.Tensor, max_norm: float) -> torch.Tensor:
        """min(1, max_norm / norm) on the device (torch clip_grad_norm_ rule)."""
        return torch.clamp(max_norm / (norm + 1e-6), max=1.0)

    @torch.no_grad()
    def step(self, closure=None, grad_scale: float = 1.0, max_norm: float = 0.0,
             norm: Optional[torch.Tensor] = None):
        """One update.  ``max_norm > 0`` clips the averaged gradient to that
        global L2 norm (``norm``: its precomputed value, else computed here);
        the clip coefficient stays on the device and scales the gradient
        inside the Adam kernel."""
        loss = closure() if closure is not None else None
        p, gr = self.flat.data, self.flat.grad
        coef = None
        if max_norm > 0:
            if norm is None:
                norm = self.grad_norm(grad_scale)
            coef = self.clip_coef(norm, max_norm)
        from .. import ops
        if p.is_cuda and ops.use_hip(p, any_dtype=True):
            from ..ops import hip_impl
            if coef is not None or FUSED_UPDATE:
                hp = self.hparams_to(torch.empty(8, dtype=torch.float32, device=p.device), grad_scale)
                if coef is not None:
                    hp[6:7].mul_(coef)
                if FUSED_UPDATE:        # Adam + bf16 operand repack (+ gradient zeroing) in one pass over the tiles
                    hip_impl.adam_update_all(self.flat, self.exp_avg, self.exp_avg_sq, self.ema, hp,
                                             zero_g=self.zero_in_step)
                    self._grad_zeroed = self.zero_in_step
                else:
                    hip_impl.adam_flat_dev(p, gr, self.exp_avg, self.exp_avg_sq, self.ema, hp)
            else:
                g = self.param_groups[0]
                lr, (b1, b2), eps, wd = g["lr"], g["betas"], g["eps"], g["weight_decay"]
                self.step_count += 1
                t = self.step_count
                hip_impl.adam_flat(p, gr, self.exp_avg, self.exp_avg_sq, self.ema, lr, b1, b2, eps, wd,
                                   lr / (1.0 - b1 ** t), math.sqrt(1.0 - b2 ** t), grad_scale, self.ema_decay)
        else:
            g = self.param_groups[0]
            lr, (b1, b2), eps, wd = g["lr"], g["betas"], g["eps"], g["weight_decay"]
            self.step_count += 1
            t = self.step_count
            bc2_sqrt = math.sqrt(1.0 - b2 ** t)
            step_size = lr / (1.0 - b1 ** t)
            grad = gr if grad_scale == 1.0 else gr * grad_scale
            if coef is not None:
                grad = grad * coef
            if wd != 0.0:
                grad = grad.add(p, alpha=wd)
            self.exp_avg.lerp_(grad, 1.0 - b1)
            self.exp_avg_sq.mul_(b2).addcmul_(grad, grad, value=1.0 - b2)
            denom = (self.exp_avg_sq.sqrt() / bc2_sqrt).add_(eps)
            p.addcdiv_(self.exp_avg, denom, value=-step_size)
            if self.ema is not None:
                self.ema.lerp_(p, 1.0 - self.ema_decay)
        for cb in self.on_step:
            cb()
        return loss

    # ------------------------------------------------------------------
    def state_dict(self):
        groups = []
        for g in self.param_groups:
            d = {k: v for k, v in g.items() if k != "params"}
            d["params"] = list(range(len(self.flat.params)))
            groups.append(d)
        state = {}
        if self.step_count > 0:
            for i, _p in enumerate(self.flat.params):
                state[i] = {"step": torch.tensor(float(self.step_count)),
                            "exp_avg": self.flat.view(self.exp_avg, i).clone(),
                            "exp_avg_sq": self.flat.view(self.exp_avg_sq, i).clone()}
        return {"state": state, "param_groups": groups}

    def load_state_dict(self, sd):
        for g, sg in zip(self.param_groups, sd["param_groups"]):
            for k, v in sg.items():
                if k != "params":
                    g[k] = tuple(v) if k == "betas" else v
        st = sd.get("state", {})
        steps = set()
        with torch.no_grad():
            for i, _p in enumerate(self.flat.params):
                s = st.get(i, st.get(str(i)))
                if s is None:
                    continue
                self.flat.view(self.exp_avg, i).copy_(s["exp_avg"])
                self.flat.view(self.exp_avg_sq, i).copy_(s["exp_avg_sq"])
                steps.add(int(float(s["step"])))
        self.step_count = max(steps) if steps else 0
        for cb in self.on_step:
            cb()

    def ema_state_dict(self, model: torch.nn.Module):
        if self.ema is None:
            return None
        names = [n for n, _ in model.named_parameters()]
        return {n: self.flat.view(self.ema, i).clone() for i, n in enumerate(names)}

    @torch.no_grad()
    def reset_ema(self) -> None:
        """Restart the EMA from the current weights (after loading pretrained
        / transferred weights, so the average never starts from random init)."""
        if self.ema is not None:
            self.ema.copy_(self.flat.data)

    @torch.no_grad()
    def load_ema_state_dict(self, model: torch.nn.Module, sd) -> bool:
        """Restore a saved EMA (``ema_state_dict`` format, optional ``module.``
        prefix).  Returns False (EMA restarted from the weights) when the
        checkpoint has none or it does not cover every parameter."""
        if self.ema is None:
            return False
        if not sd:
            self.reset_ema()
            return False
        sd = {(k[7:] if k.startswith("module.") else k): v for k, v in sd.items()}
        names = [n for n, _ in model.named_parameters()]
        if any(n not in sd for n in names):
            self.reset_ema()
            return False
        for i, n in enumerate(names):
            self.flat.view(self.ema, i).copy_(sd[n].reshape(self.flat.params[i].shape))
        return True


def ema_decay_for(batch_size: int, halflife_examples: float) -> float:
    """Per-step EMA decay for a half-life measured in examples (paper: 500K)."""
    if halflife_examples <= 0:
        return 0.0
    return 0.5 ** (batch_size / halflife_examples)


def warmup_lr(step: int, warmup_steps: float, peak: float) -> float:
    """Linear warmup (`train.py:169-177`): lr = step/last_step * peak."""
    if warmup_steps > 0 and step < warmup_steps:
        return step / warmup_steps * peak
    return peak
