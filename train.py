#!/usr/bin/env python
"""Training CLI (reference: `train.py:307-319` DDP trainer and
`lightning/train.py:19-46`).

Reference-compatible flags: ``--transfer DIR`` (resume from DIR/latest.pt and
keep writing there), ``--train_data PATH`` / ``--val_data PATH`` (Lightning
CLI).  Launch modes:

  python train.py --train_data data/SRN/cars_train            # 1 process
  python train.py --gpus 8 ...                                 # self-spawn 8 ranks
  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 train.py ...   # torchrun env honoured

Everything else is a typed config override: ``key.sub=value`` (see
``distributed_3d_diffusion_pytorch_amd/config.py``), e.g.
``global_batch=128 optim.warmup_examples=10000000 model.H=128``.
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--transfer", default="", help="resume from <dir>/latest.pt (reference flag)")
    ap.add_argument("--train_data", default="", help="SRN instance root (Lightning-CLI flag)")
    ap.add_argument("--val_data", default="", help="accepted for CLI compatibility (unused, as upstream)")
    ap.add_argument("--index", default="", help="index pickle/json {instance: [views]}; default <data>/cars.pickle")
    ap.add_argument("--preset", default="", help="config preset (chairs32_cpu, cars64_8gpu, ...)")
    ap.add_argument("--synthetic", action="store_true", help="on-device synthetic SRN-shaped data")
    ap.add_argument("--gpus", type=int, default=0, help="self-spawn this many local ranks")
    ap.add_argument("--steps", type=int, default=0, help="stop after this many optimizer steps")
    ap.add_argument("--out_dir", default="")
    ap.add_argument("overrides", nargs="*", help="key=value config overrides")
    return ap.parse_args(argv)


def run(args) -> None:
    import torch
    from distributed_3d_diffusion_pytorch_amd.config import make_config, parse_kv
    from distributed_3d_diffusion_pytorch_amd.parallel import init_distributed, cleanup
    from distributed_3d_diffusion_pytorch_amd.engine import Trainer

    ov = parse_kv(args.overrides)
    cfg = make_config(args.preset or None, ov)
    if args.train_data:
        cfg.data.path = args.train_data
        if not args.index and not cfg.data.index:
            for name in ("cars.pickle", "chairs.pickle", "index.pkl", "index.json"):
                cand = os.path.join(args.train_data, name)
                if os.path.exists(cand):
                    cfg.data.index = cand
                    break
    if args.index:
        cfg.data.index = args.index
    if args.synthetic:
        cfg.data.synthetic = True
    if args.transfer:
        cfg.transfer = args.transfer
    if args.out_dir:
        cfg.out_dir = args.out_dir
    if args.steps:
        cfg.max_steps = args.steps
    ctx = init_distributed(cfg.dist.backend, cfg.dist.timeout_s)
    if ctx.device.type == "cpu" and cfg.dtype == "bf16":
        cfg.dtype = "fp32"
    if ctx.is_main:
        print(f"[train] world={ctx.world} device={ctx.device} global_batch={cfg.global_batch} "
              f"img={cfg.model.H} data={'synthetic' if cfg.data.synthetic else cfg.data.path}", flush=True)
    try:
        trainer = Trainer(cfg, ctx)
        trainer.fit()
    finally:
        cleanup()


def _spawn_worker(args) -> None:
    run(args)


def main(argv=None) -> None:
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        from distributed_3d_diffusion_pytorch_amd.parallel import spawn
        spawn(_spawn_worker, args.gpus, (args,))
    else:
        run(args)


if __name__ == "__main__":
    main()
