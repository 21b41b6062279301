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
"""
from __future__ import annotations

from typing import Callable, Dict, Optional

import torch


class GradSink:
    def __init__(self) -> None:
        self.enabled = False
        self.views: Dict[int, torch.Tensor] = {}
        self.index: Dict[int, int] = {}
        self.uses: Dict[int, int] = {}
        self.seen = set()
        self.notify: Optional[Callable[[int], None]] = None

    def attach(self, params, views, notify: Optional[Callable[[int], None]] = None) -> None:
        self.views = {id(p): v for p, v in zip(params, views)}
        self.index = {id(p): i for i, p in enumerate(params)}
        self.uses = {}
        self.notify = notify
        self.enabled = True

    def detach(self) -> None:
        self.enabled = False
        self.views, self.index, self.uses, self.notify = {}, {}, {}, None

    def managed(self, p) -> bool:
        return self.enabled and p is not None and id(p) in self.views

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
        return self.enabled and id(p) in self.seen

    def done(self, p) -> None:
        if not self.managed(p):
            return
        k = id(p)
        n = self.uses.get(k, 1) - 1
        self.uses[k] = n
        if n == 0 and self.notify is not None:
            self.notify(self.index[k])

    def reset(self) -> None:
        self.uses = {}
        self.seen = set()


SINK = GradSink()
