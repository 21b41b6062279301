#!/usr/bin/env python
"""Tune the library GEMMs of the training step (PyTorch TunableOp, see
utils/gemm_tuning.py) on an MI355X and write tuning/tunableop_mi355x.csv.

    python tools/tune_gemms.py [--batches 128,64,32,16] [--out tuning/tunableop_mi355x.csv]

Runs a few EAGER training steps per per-GPU batch (the shapes of the 1/2/4/8-GPU
shares of global batch 128), with TunableOp tuning every new GEMM shape."""
import argparse
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child(batch: int, out: str) -> None:
    import torch
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_max_tuning_duration(int(os.environ.get("D3D_TUNE_MS", "40")))
    tun.set_filename(out)
    if os.path.exists(out):
        tun.read_file(out)
    from distributed_3d_diffusion_pytorch_amd.config import make_config
    from distributed_3d_diffusion_pytorch_amd.engine import Trainer
    from distributed_3d_diffusion_pytorch_amd.parallel import DistContext
    from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches
    mb = 64 if batch > 128 else 0          # bench.py: one micro-batch up to 128 examples at 64x64
    cfg = make_config(None, {"global_batch": batch, "micro_batch": mb, "data.synthetic": True, "log_every": 0,
                             "ckpt_every": 0, "graph": False})
    tr = Trainer(cfg, DistContext(device=torch.device("cuda", 0)))
    data = SyntheticBatches(batch, 64, "cuda", seed=0)
    for _ in range(2):
        tr.train_step(*next(data))
    torch.cuda.synchronize()
    print(f"[tune] batch {batch}: {len(tun.get_results())} tuned GEMMs", flush=True)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="128,64,32,16")
    ap.add_argument("--out", default=os.path.join(ROOT, "tuning", "tunableop_mi355x.csv"))
    ap.add_argument("--child", type=int, default=0)
    a = ap.parse_args()
    if a.child:
        return child(a.child, a.out)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    env = dict(os.environ, D3D_TUNED_GEMMS="0")
    for b in (int(x) for x in a.batches.split(",")):
        # one process per batch: TunableOp writes its table at process exit
        subprocess.run([sys.executable, __file__, "--child", str(b), "--out", a.out], check=True, env=env)
    print(open(a.out).read()[:2000])


if __name__ == "__main__":
    main()
