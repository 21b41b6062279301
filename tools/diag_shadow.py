"""Shadow re-execution of the weight-gradient jobs: every conv / linear job
that ran on the side stream during backward is re-run after a full device
sync (same inputs, fresh zero targets) and its result compared bit for bit
with what it deposited.  Names the jobs whose concurrent execution produced
a different result than a quiet re-run."""
import inspect
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    dev = torch.device("cuda", 0)
    from distributed_3d_diffusion_pytorch_amd.config import make_config
    from distributed_3d_diffusion_pytorch_amd.engine import Trainer
    from distributed_3d_diffusion_pytorch_amd.parallel import DistContext
    from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches
    from distributed_3d_diffusion_pytorch_amd.ops.gradsink import SINK
    from distributed_3d_diffusion_pytorch_amd.models import xunet as X
    X._COND_STREAM = False
    ctx = DistContext(device=dev)
    cfg = make_config(None, {"model.H": 64, "model.W": 64, "data.imgsize": 64, "global_batch": B, "micro_batch": 0,
                             "data.synthetic": True, "log_every": 0, "ckpt_every": 0, "graph": False,
                             "optim.warmup_examples": 32})
    tr = Trainer(cfg, ctx)
    pname = {id(p): n for n, p in tr.model.named_parameters()}
    jobs = []
    osub = SINK.submit

    def submit(d, fn, keep=(), done=()):
        sig = inspect.signature(fn).parameters
        if "tw" in sig:
            jobs.append((fn, sig["tw"].default, sig["tb"].default if "tb" in sig else None,
                         [pname.get(id(p), "?") for p in done if p is not None], inspect.getsourcelines(fn)[1]))
        return osub(d, fn, keep, done)
    SINK.submit = submit
    ostep = tr.optim.step
    report = []

    def step(*a, **k):
        torch.cuda.synchronize()
        bad = []
        for fn, tw, tb, names, line in jobs:
            zw = torch.zeros_like(tw)
            zb = torch.zeros_like(tb) if tb is not None else None
            kw = {"tw": zw}
            if "tb" in inspect.signature(fn).parameters:
                kw["tb"] = zb
            fn(**kw)
            torch.cuda.synchronize()
            dw = (zw - tw).abs().max().item()
            db = (zb - tb).abs().max().item() if tb is not None else 0.0
            if dw or db:
                bad.append((names, line, f"{dw:.2e}/{tw.abs().max().item():.2e}", f"{db:.2e}"))
        report.append(bad)
        jobs.clear()
        return ostep(*a, **k)
    tr.optim.step = step
    data = SyntheticBatches(B, 64, "cuda", seed=33)
    for s in range(steps):
        tr.train_step(*next(data))
        torch.cuda.synchronize()
        print(f"step {s}: {len(report[-1])} jobs differ from their quiet re-run: {report[-1][:6]}", flush=True)


if __name__ == "__main__":
    main()
