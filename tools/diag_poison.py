"""Uninitialised-read screen for the training step: every block the caching
allocator hands out starts as NaN (the allocator is pre-filled with NaN
tensors that are then freed), so a kernel that reads workspace or output
memory it did not write first turns the loss / gradients non-finite.
Forward hooks name the first module whose output is non-finite; the
gradients are checked per parameter after backward.

usage: python tools/diag_poison.py [global_batch] [micro_batch]   (eager step)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def poison(dev, big_gib: float = 48.0, small_mib: int = 256):
    nan = float("nan")
    # large pool: one big segment later split for every >= 1 MiB allocation
    t = torch.empty(int(big_gib * (1 << 30)) // 4, dtype=torch.float32, device=dev)
    t.fill_(nan)
    del t
    # small pool (< 1 MiB requests come from 2 MiB segments): fill a few
    # hundred segments with NaN blocks of assorted sizes
    keep = []
    for sz in (512 << 10, 256 << 10, 128 << 10, 64 << 10, 16 << 10, 4 << 10, 512):
        n = (small_mib << 20) // len((1, 2, 3, 4, 5, 6, 7)) // sz
        for _ in range(max(1, n)):
            keep.append(torch.full((sz // 4,), nan, device=dev))
    del keep
    torch.cuda.synchronize()


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    mb = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    dev = torch.device("cuda", 0)
    from distributed_3d_diffusion_pytorch_amd.config import make_config
    from distributed_3d_diffusion_pytorch_amd.engine import Trainer
    from distributed_3d_diffusion_pytorch_amd.parallel import DistContext
    from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches
    ctx = DistContext(device=dev)
    data = SyntheticBatches(B, 64, "cuda", seed=33)
    batches = [next(data) for _ in range(2)]
    torch.cuda.synchronize()
    poison(dev)
    torch.manual_seed(0)
    cfg = make_config(None, {"model.H": 64, "model.W": 64, "data.imgsize": 64, "global_batch": B,
                             "micro_batch": mb, "data.synthetic": True, "log_every": 0, "ckpt_every": 0,
                             "graph": False, "optim.warmup_examples": 0})
    tr = Trainer(cfg, ctx)
    bad = []

    def hook(mod, inp, out, name=None):
        outs = out if isinstance(out, (tuple, list)) else (out,)
        for o in outs:
            if torch.is_tensor(o) and o.is_floating_point() and not torch.isfinite(o).all():
                bad.append(name)
                break

    for n, m in tr.model.named_modules():
        m.register_forward_hook(lambda mod, i, o, n=n: hook(mod, i, o, n))
    names = [n for n, _ in tr.model.named_parameters()]
    for s, b in enumerate(batches):
        # keep the gradient of this step: run the pieces of train_step by hand
        loss = tr.train_step(*b)
        torch.cuda.synchronize()
        print(f"step {s}: loss {loss.item()!r}; first non-finite module outputs: {bad[:6]}", flush=True)
        p = tr.flat.data
        nf = [names[i] for i in range(len(names))
              if not torch.isfinite(p[tr.flat.offsets[i]: tr.flat.offsets[i] + tr.flat.params[i].numel()]).all()]
        print(f"   non-finite parameters after the update: {len(nf)} {nf[:12]}", flush=True)
        bad.clear()


if __name__ == "__main__":
    main()
