"""Which Python lines issue the device copies / small torch ops of one eager
training step (torch.profiler with stacks):  python tools/copy_sources.py [--batch 16]"""
import argparse
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--ops", default="aten::copy_,aten::add_,aten::sum,aten::fill_,aten::zero_,aten::mul")
    a = ap.parse_args()
    from distributed_3d_diffusion_pytorch_amd.config import make_config
    from distributed_3d_diffusion_pytorch_amd.engine import Trainer
    from distributed_3d_diffusion_pytorch_amd.parallel import DistContext
    from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches
    ctx = DistContext(device=torch.device("cuda", 0))
    cfg = make_config(None, {"model.H": 64, "model.W": 64, "data.imgsize": 64, "global_batch": a.batch,
                             "micro_batch": a.batch, "data.synthetic": True, "log_every": 0, "ckpt_every": 0,
                             "graph": False})
    tr = Trainer(cfg, ctx)
    data = SyntheticBatches(a.batch, 64, "cuda", seed=3)
    b = next(data)
    for _ in range(2):
        tr.train_step(*b)
    torch.cuda.synchronize()
    wanted = set(a.ops.replace("+", ",").split(","))      # "+" also separates (tools/gpu.sh kbench args)
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU], with_stack=True) as prof:
        tr.train_step(*b)
        torch.cuda.synchronize()
    cnt = collections.Counter()
    for e in prof.events():
        if e.name in wanted:
            st = [s for s in (e.stack or []) if "distributed_3d_diffusion_pytorch_amd" in s or "bench" in s]
            par, q = [], e.cpu_parent
            while q is not None and len(par) < 3:
                par.append(q.name)
                q = q.cpu_parent
            cnt[(e.name, " <- ".join(st[:3]) if st else " < ".join(par) or "?")] += 1
    for (name, where), n in cnt.most_common(40):
        print(f"{n:5d}  {name:14s} {where}")


if __name__ == "__main__":
    main()
