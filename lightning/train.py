#!/usr/bin/env python
"""Training CLI of the Lightning variant (reference `lightning/train.py:1-46`, T3).

    python lightning/train.py --train_data data/SRN/cars_train [--transfer CKPT.pt] [key=value ...]

Reference behaviour kept: 64x64 images, batch 4, 4 loader workers, index
``<train_data>/cars.pickle``, 100k max steps on one device, linear warmup over
one pass of the training set (n_samples / batch_size steps), ``--transfer``
initialises model + optimizer state from a checkpoint FILE and training starts
at step 0 (`lightning/diff3d.py:40-45`).  ``precision=16`` (fp16 AMP) maps to
this framework's bf16 compute with fp32 master weights.  ``--val_data`` is
accepted and unused, as upstream.  Extra ``key=value`` pairs override the
typed config (``global_batch=8``, ``optim.use_cosine=true``, ...); ``--gpus N``
runs data-parallel over N ranks instead of Lightning's single device.
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--transfer", default="", help="pretrained checkpoint file {'model','optim'}")
    ap.add_argument("--train_data", default=os.path.join("data", "SRN", "cars_train"))
    ap.add_argument("--val_data", default="")
    ap.add_argument("--gpus", type=int, default=0)
    ap.add_argument("--out_dir", default="lightning_logs")
    ap.add_argument("overrides", nargs="*")
    return ap.parse_args(argv)


def to_root_args(args):
    """The equivalent root ``train.py`` invocation (same Trainer)."""
    import train as root_train
    ov = ["data.imgsize=64", "model.H=64", "model.W=64", "global_batch=4", "data.num_workers=4",
          "max_steps=100000", "optim.warmup_examples=-1", "optim.use_cosine=false"]
    if args.transfer:
        ov.append(f"pretrained={args.transfer}")
    ov += list(args.overrides)
    argv = ["--train_data", args.train_data, "--index", os.path.join(args.train_data, "cars.pickle"),
            "--out_dir", args.out_dir]
    if args.gpus:
        argv += ["--gpus", str(args.gpus)]
    return root_train, root_train.parse(argv + ov)


def main(argv=None) -> None:
    args = parse(argv)
    root_train, rargs = to_root_args(args)
    if rargs.gpus > 1 and "WORLD_SIZE" not in os.environ:
        from distributed_3d_diffusion_pytorch_amd.parallel import spawn
        spawn(root_train._spawn_worker, rargs.gpus, (rargs,))
    else:
        root_train.run(rargs)


if __name__ == "__main__":
    main()
