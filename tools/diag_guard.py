"""Out-of-bounds write screen for the weight-gradient jobs: every tensor a
job allocates (split-K slabs, bias partials) gets a sentinel-filled guard
region behind it; after each step the guards are checked.  The jobs run
serialised (synchronize after each) so a violation is attributed to the job
that wrote it.

usage: python tools/diag_guard.py [global_batch]"""
import contextlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

GUARD = 64 * 1024          # elements behind every job allocation
SENT = 1234.5


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    dev = torch.device("cuda", 0)
    from distributed_3d_diffusion_pytorch_amd.config import make_config
    from distributed_3d_diffusion_pytorch_amd.engine import Trainer
    from distributed_3d_diffusion_pytorch_amd.parallel import DistContext
    from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches
    from distributed_3d_diffusion_pytorch_amd.ops.gradsink import SINK
    ctx = DistContext(device=dev)
    data = SyntheticBatches(B, 64, "cuda", seed=33)
    batches = [next(data) for _ in range(2)]
    cfg = make_config(None, {"model.H": 64, "model.W": 64, "data.imgsize": 64, "global_batch": B,
                             "micro_batch": 0, "data.synthetic": True, "log_every": 0, "ckpt_every": 0,
                             "graph": False, "optim.warmup_examples": 0})
    tr = Trainer(cfg, ctx)
    guards = []
    real_empty = torch.empty
    state = {"on": False, "job": None}

    def guarded_empty(*size, dtype=None, device=None, **kw):
        if not state["on"]:
            return real_empty(*size, dtype=dtype, device=device, **kw)
        shape = tuple(size[0]) if len(size) == 1 and isinstance(size[0], (tuple, list, torch.Size)) else size
        n = 1
        for s in shape:
            n *= int(s)
        full = real_empty(n + GUARD, dtype=dtype or torch.float32, device=device or dev)
        full[n:].fill_(SENT)
        guards.append((full, n, state["job"]))
        return full[:n].view(shape)

    orig_producer = SINK.producer

    @contextlib.contextmanager
    def producer(d, *keep):
        state["on"] = True
        state["job"] = [tuple(t.shape) for t in keep if t is not None]
        torch.empty = guarded_empty
        try:
            with orig_producer(d, *keep):
                yield
        finally:
            torch.empty = real_empty
            state["on"] = False
        torch.cuda.synchronize()
        for full, n, job in guards:
            tail = full[n:]
            bad = (tail != SENT).nonzero()
            if bad.numel():
                first = int(bad[0])
                print(f"GUARD VIOLATION job keep-shapes {job}: {bad.numel()} elements written past the end "
                      f"of a {n}-element {full.dtype} allocation (first at +{first})", flush=True)
        guards.clear()

    SINK.producer = producer
    for s, b in enumerate(batches):
        loss = tr.train_step(*b)
        torch.cuda.synchronize()
        print(f"step {s}: loss {loss.item():.6f}", flush=True)


if __name__ == "__main__":
    main()
