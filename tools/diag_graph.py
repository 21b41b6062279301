"""Graph-replayed vs eager training step at bench shapes: per-step losses and
parameter drift (python tools/diag_graph.py --batch 128 --mb 64 --steps 6)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--mb", type=int, default=64)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--dropout", type=float, default=0.1)
    ap.add_argument("--img", type=int, default=64)
    a = ap.parse_args()
    from distributed_3d_diffusion_pytorch_amd.config import make_config
    from distributed_3d_diffusion_pytorch_amd.engine import Trainer
    from distributed_3d_diffusion_pytorch_amd.parallel import DistContext
    from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches
    ctx = DistContext(device=torch.device("cuda", 0))

    def make(graph):
        cfg = make_config(None, {"model.H": a.img, "model.W": a.img, "model.dropout": a.dropout,
                                 "data.imgsize": a.img, "global_batch": a.batch, "micro_batch": a.mb,
                                 "data.synthetic": True, "log_every": 0, "ckpt_every": 0, "graph": graph})
        return Trainer(cfg, ctx)

    data = SyntheticBatches(a.batch, a.img, "cuda", seed=5)
    batches = [next(data) for _ in range(a.steps)]
    for graph in (False, True):
        torch.manual_seed(0)
        tr = make(graph)
        ls = []
        for b in batches:
            l = tr.train_step(*b)
            ls.append(float(l))
        torch.cuda.synchronize()
        print(f"graph={graph} losses={['%.5f' % x for x in ls]} "
              f"param_norm={tr.flat.data.norm().item():.6f} finite={bool(torch.isfinite(tr.flat.data).all())}",
              flush=True)
        del tr
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
