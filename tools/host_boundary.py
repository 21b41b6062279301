"""Host time spent between consecutive graph-A replays of the bs16 graph step
(the work the device must cover from its queue at each step boundary), and
the host time inside replay()."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    from distributed_3d_diffusion_pytorch_amd.config import make_config
    from distributed_3d_diffusion_pytorch_amd.engine import Trainer
    from distributed_3d_diffusion_pytorch_amd.parallel import DistContext
    from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches
    ctx = DistContext(device=torch.device("cuda", 0))
    cfg = make_config(None, {"model.H": 64, "model.W": 64, "data.imgsize": 64, "global_batch": B,
                             "micro_batch": 0, "data.synthetic": True, "log_every": 0, "ckpt_every": 0,
                             "graph": True})
    tr = Trainer(cfg, ctx)
    pool = [next(SyntheticBatches(B, 64, "cuda", seed=3 + i)) for i in range(2)]
    for i in range(4):
        tr.train_step(*pool[i % 2])
    torch.cuda.synchronize()
    stamps = []
    orig = torch.cuda.CUDAGraph.replay

    def replay(self):
        a = time.perf_counter()
        orig(self)
        stamps.append((a, time.perf_counter()))

    torch.cuda.CUDAGraph.replay = replay
    n = 12
    t0 = time.perf_counter()
    for i in range(n):
        tr.train_step(*pool[i % 2])
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    torch.cuda.CUDAGraph.replay = orig
    inside = [b - a for a, b in stamps]
    between = [stamps[i + 1][0] - stamps[i][1] for i in range(len(stamps) - 1)]
    print(f"replays {len(stamps)}: inside replay() median {1e3 * sorted(inside)[len(inside) // 2]:.3f} ms; "
          f"host between replays median {1e3 * sorted(between)[len(between) // 2]:.3f} ms; "
          f"host loop {1e3 * (t1 - t0) / n:.3f} ms/step, wall {1e3 * (t2 - t0) / n:.3f} ms/step", flush=True)


if __name__ == "__main__":
    main()
