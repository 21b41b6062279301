"""Flat-gradient padding screen: every parameter's gradient view is followed
by up to 63 padding elements in the flat buffer (parallel/flat.py).  They are
filled with a sentinel before the step; a weight-gradient kernel that writes
past its parameter's end shows up as a changed sentinel, attributed to the
parameter in front of it."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    dev = torch.device("cuda", 0)
    from distributed_3d_diffusion_pytorch_amd.config import make_config
    from distributed_3d_diffusion_pytorch_amd.engine import Trainer
    from distributed_3d_diffusion_pytorch_amd.parallel import DistContext
    from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches
    ctx = DistContext(device=dev)
    cfg = make_config(None, {"model.H": 64, "model.W": 64, "data.imgsize": 64, "global_batch": B, "micro_batch": 0,
                             "data.synthetic": True, "log_every": 0, "ckpt_every": 0, "graph": False})
    tr = Trainer(cfg, ctx)
    names = [n for n, _ in tr.model.named_parameters()]
    fl = tr.flat
    pads = []
    for i, p in enumerate(fl.params):
        a = fl.offsets[i] + p.numel()
        b = fl.span(i)[1]
        if b > a:
            pads.append((i, a, b))
    SENT = 7777.0
    ostep = tr.optim.step
    bad = []

    def step(*a, **k):
        torch.cuda.synchronize()
        for i, s, e in pads:
            v = fl.grad[s:e]
            if not torch.all(v == SENT):
                bad.append((names[i], int((v != SENT).sum()), e - s))
        for i, s, e in pads:
            fl.grad[s:e] = 0.0
        return ostep(*a, **k)
    tr.optim.step = step
    b = next(SyntheticBatches(B, 64, "cuda", seed=3))
    for it in range(2):
        for i, s, e in pads:
            fl.grad[s:e] = SENT
        torch.cuda.synchronize()
        tr.train_step(*b)
        torch.cuda.synchronize()
        print(f"step {it}: {len(bad)} padding regions written: {bad[:12]}", flush=True)
        bad.clear()
    print(f"{len(pads)} padded parameters checked")


if __name__ == "__main__":
    main()
