"""Which PyTorch (aten) ops still run inside a training step, and from where.

The HIP path issues its kernels through ctypes, so every aten op that reaches
the dispatcher during a step is torch "glue" (fills, adds, copies, reductions).
This records them with a TorchDispatchMode -- forward, backward (autograd's
worker threads inherit the mode) and, with --graph 1, the capture of the
replayed step -- and prints each op with the innermost framework source lines
that issued it:

    python tools/glue_ops.py --global_batch 16 --graph 1
"""
import argparse
import collections
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from torch.utils._python_dispatch import TorchDispatchMode

# metadata / view ops that launch no kernel
_FREE = ("aten.empty", "aten.view", "aten._unsafe_view", "aten.detach", "aten.as_strided", "aten.t.",
         "aten.alias", "aten.slice", "aten.select", "aten.expand", "aten.reshape", "aten.permute",
         "aten.unsqueeze", "aten.squeeze", "aten.transpose", "aten.split", "aten.unbind", "aten.set_",
         "aten.lift", "aten._to_copy.default(cpu", "aten.is_", "aten.record_stream", "aten.new_empty",
         "aten.empty_like", "aten.empty_strided", "aten._local_scalar_dense", "aten.item")


class Glue(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.ops = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = str(func)
        if not any(name.startswith(f) for f in _FREE):
            dev = [a.device.type for a in args if isinstance(a, torch.Tensor)]
            if "cuda" in dev or not dev:
                fr = [f for f in traceback.extract_stack()[:-1]
                      if "distributed_3d_diffusion_pytorch_amd" in f.filename or f.filename.endswith("bench.py")]
                where = " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in fr[-3:][::-1])
                self.ops[(name, where)] += 1
        return func(*args, **(kwargs or {}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--global_batch", type=int, default=16)
    ap.add_argument("--graph", type=int, default=0)
    ap.add_argument("--imgsize", type=int, default=64)
    a = ap.parse_args()
    from distributed_3d_diffusion_pytorch_amd.config import make_config
    from distributed_3d_diffusion_pytorch_amd.engine import Trainer
    from distributed_3d_diffusion_pytorch_amd.parallel import DistContext
    from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches
    ctx = DistContext(device=torch.device("cuda", 0))
    cfg = make_config(None, {"model.H": a.imgsize, "model.W": a.imgsize, "data.imgsize": a.imgsize,
                             "global_batch": a.global_batch, "micro_batch": 0, "data.synthetic": True,
                             "log_every": 0, "ckpt_every": 0, "graph": bool(a.graph)})
    tr = Trainer(cfg, ctx)
    data = SyntheticBatches(a.global_batch, a.imgsize, "cuda", seed=3)
    b = next(data)
    if not a.graph:
        for _ in range(2):
            tr.train_step(*b)
    torch.cuda.synchronize()
    g = Glue()
    with g:
        tr.train_step(*b)       # graph: the capture (the ops recorded into the replayed graphs) + 1 replay
        if a.graph:
            tr.train_step(*b)
    torch.cuda.synchronize()
    print(f"aten ops in one {'graph capture + 2 replays' if a.graph else 'eager step'} (bs{a.global_batch}):")
    for (name, where), n in sorted(g.ops.items(), key=lambda kv: -kv[1]):
        print(f"{n:5d}  {name:<45} {where}")


if __name__ == "__main__":
    main()
