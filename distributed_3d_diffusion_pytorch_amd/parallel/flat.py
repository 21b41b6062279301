"""Flat parameter / gradient storage.

All 647 parameters live as views of ONE contiguous fp32 buffer and their
gradients as views of ONE contiguous fp32 gradient buffer.  That layout is
what makes the rest of the runtime cheap on MI355X:

* the fused Adam kernel updates every parameter in a single launch;
* data-parallel gradient buckets are contiguous slices, so a bucket is
  all-reduced in place by RCCL with no flatten/unflatten copies;
* checkpoint / broadcast / checksum are single-buffer operations.

Parameters are laid out in *reverse* registration order (≈ the order in
which backward produces their gradients), each padded to a 64-element
(256-byte) boundary so every view is 16-byte aligned for vector loads.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import torch

ALIGN = 64


class FlatParams:
    def __init__(self, params: Sequence[torch.nn.Parameter], device=None, reverse: bool = True):
        self.params: List[torch.nn.Parameter] = list(params)
        if not self.params:
            raise ValueError("no parameters")
        device = device or self.params[0].device
        order = list(range(len(self.params)))
        if reverse:
            order = order[::-1]
        self.offsets = [0] * len(self.params)
        off = 0
        for i in order:
            self.offsets[i] = off
            n = self.params[i].numel()
            off += (n + ALIGN - 1) // ALIGN * ALIGN
        self.numel = off
        self.order = order
        self.data = torch.zeros(self.numel, dtype=torch.float32, device=device)
        self.grad = torch.zeros(self.numel, dtype=torch.float32, device=device)
        with torch.no_grad():
            for i, p in enumerate(self.params):
                v = self.view(self.data, i)
                v.copy_(p.detach().to(torch.float32))
                p.data = v
                p.grad = self.view(self.grad, i)

    def view(self, buf: torch.Tensor, i: int) -> torch.Tensor:
        p = self.params[i]
        o = self.offsets[i]
        return buf[o: o + p.numel()].view(p.shape)

    def span(self, i: int) -> Tuple[int, int]:
        o = self.offsets[i]
        return o, o + (self.params[i].numel() + ALIGN - 1) // ALIGN * ALIGN

    def zero_grad(self) -> None:
        self.grad.zero_()

    def rebind_grads(self) -> None:
        """Re-point ``p.grad`` at the flat buffer (after user code replaced it)."""
        for i, p in enumerate(self.params):
            g = self.view(self.grad, i)
            if p.grad is None or p.grad.data_ptr() != g.data_ptr():
                if p.grad is not None:
                    g.copy_(p.grad)
                p.grad = g
