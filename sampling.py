#!/usr/bin/env python
"""Stochastic-conditioning novel-view sampling CLI (reference: `sampling.py:19-184`).

    python sampling.py --model trained_model.pt --target data/SRN/cars_train/<instance>

Loads every view of the target SRN instance, conditions on view 0 and
autoregressively generates each remaining view with the 256-step CFG sampler,
one chain per guidance weight (default w = 0..7); each step conditions on a
random already-known view of the chain (stochastic conditioning).  Writes
``<out>/{k}/gt.png`` and ``<out>/{k}/{i}.png`` like the reference.

Multi-GPU: ``--gpus N`` (or torchrun) shards the guidance-weight chains over
ranks, one process per GPU; rank 0 gathers and writes the PNGs.
"""
from __future__ import annotations

import argparse
import glob
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="./trained_model.pt")
    ap.add_argument("--target", default="./data/SRN/cars_train/a4d535e1b1d3c153ff23af07d9064736")
    ap.add_argument("--out", default="sampling")
    ap.add_argument("--imgsize", type=int, default=64)
    ap.add_argument("--timesteps", type=int, default=256)
    ap.add_argument("--w", default="0,1,2,3,4,5,6,7", help="guidance weights, one chain each")
    ap.add_argument("--max_views", type=int, default=0, help="generate at most this many views (0 = all)")
    ap.add_argument("--ema", action="store_true", help="use EMA weights when the checkpoint has them")
    ap.add_argument("--ref_quirk", action="store_true", help="reproduce D9 (no noise at logsnr_next == 0)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--gpus", type=int, default=0)
    ap.add_argument("--backend", default="auto")
    return ap.parse_args(argv)


def load_instance(target: str, imgsize: int):
    from distributed_3d_diffusion_pytorch_amd.data.srn import load_image, read_matrix
    imgs, Rs, Ts = [], [], []
    files = sorted(glob.glob(os.path.join(target, "rgb", "*.png")))
    if not files:
        raise FileNotFoundError(f"no views under {target}/rgb")
    for f in files:
        imgs.append(load_image(f, imgsize))
        pose = read_matrix(os.path.join(target, "pose", os.path.basename(f)[:-4] + ".txt"), (4, 4))
        Rs.append(pose[:3, :3])
        Ts.append(pose[:3, 3])
    # the reference takes K from the LAST view's intrinsics file (sampling.py:47-48)
    K = read_matrix(os.path.join(target, "intrinsics", os.path.basename(files[-1])[:-4] + ".txt"), (3, 3))
    return np.stack(imgs), np.stack(Rs), np.stack(Ts), K


def save_png(arr_chw: np.ndarray, path: str) -> None:
    from PIL import Image
    img = ((np.clip(arr_chw.transpose(1, 2, 0), -1, 1) + 1) * 127.5).astype(np.uint8)
    Image.fromarray(img).save(path)


def run(args) -> None:
    import torch
    import torch.distributed as dist
    from distributed_3d_diffusion_pytorch_amd import ops
    from distributed_3d_diffusion_pytorch_amd.models import XUNet
    from distributed_3d_diffusion_pytorch_amd.engine import DiffusionSampler, RecordEntry, shard_range
    from distributed_3d_diffusion_pytorch_amd.parallel import init_distributed, cleanup
    from distributed_3d_diffusion_pytorch_amd.utils import load_checkpoint, load_model_weights

    ctx = init_distributed("auto")
    dev = ctx.device
    if args.backend != "auto":
        ops.set_backend(args.backend)
    imgs, Rs, Ts, K = load_instance(args.target, args.imgsize)
    ck = load_checkpoint(args.model)
    if isinstance(ck.get("config"), dict):       # our checkpoints carry their model config
        from distributed_3d_diffusion_pytorch_amd.config import from_dict
        mcfg = from_dict(ck["config"]).model
        mcfg.H = mcfg.W = args.imgsize
        model = XUNet(mcfg).to(dev)
    else:                                        # reference checkpoints: XUNet(H, W, ch=128)
        model = XUNet(H=args.imgsize, W=args.imgsize, ch=128).to(dev)
    sd = ck.get("ema") if (args.ema and ck.get("ema")) else ck["model"]
    load_model_weights(model, sd)
    model.compute_dtype = torch.bfloat16 if dev.type == "cuda" else torch.float32
    model.eval()

    w_all = torch.tensor([float(x) for x in args.w.split(",")])
    s, e = shard_range(len(w_all), ctx.rank, ctx.world)
    w = w_all[s:e]
    b = len(w)
    # same seed on every rank: identical record choices, and the counter-based
    # noise is keyed by the GLOBAL chain index (chain_offset), so the gathered
    # result does not depend on the number of ranks
    sampler = DiffusionSampler(model, args.timesteps, args.ref_quirk, seed=args.seed, device=dev, chain_offset=s)
    t = lambda a: torch.tensor(a, dtype=torch.float32, device=dev)  # noqa: E731
    record = [RecordEntry(t(imgs[0])[None].expand(b, -1, -1, -1).contiguous(), t(Rs[0]), t(Ts[0]))]
    if ctx.is_main:
        os.makedirs(os.path.join(args.out, "0"), exist_ok=True)
        save_png(imgs[0], os.path.join(args.out, "0", "gt.png"))
    nviews = len(imgs) if not args.max_views else min(len(imgs), args.max_views + 1)
    Kt = t(K)
    for k in range(1, nviews):
        t0 = time.time()
        out = sampler.sample(record, t(Rs[k]), t(Ts[k]), Kt, w) if b > 0 else \
            torch.zeros(0, 3, args.imgsize, args.imgsize, device=dev)
        record.append(RecordEntry(out, t(Rs[k]), t(Ts[k])))
        full = out
        if ctx.world > 1:
            per = (len(w_all) + ctx.world - 1) // ctx.world
            pad = torch.zeros(per, 3, args.imgsize, args.imgsize, device=dev)
            pad[: out.shape[0]] = out
            gathered = [torch.zeros_like(pad) for _ in range(ctx.world)]
            dist.all_gather(gathered, pad)
            full = torch.cat([gathered[r][: shard_range(len(w_all), r, ctx.world)[1]
                                           - shard_range(len(w_all), r, ctx.world)[0]]
                              for r in range(ctx.world)])
        if ctx.is_main:
            d = os.path.join(args.out, str(k))
            os.makedirs(d, exist_ok=True)
            save_png(imgs[k], os.path.join(d, "gt.png"))
            arr = full.float().cpu().numpy()
            for i in range(arr.shape[0]):
                save_png(arr[i], os.path.join(d, f"{i}.png"))
            print(f"[sampling] view {k}/{nviews - 1}: {time.time() - t0:.2f}s", flush=True)
    cleanup()


def main(argv=None) -> None:
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        from distributed_3d_diffusion_pytorch_amd.parallel import spawn
        spawn(run, args.gpus, (args,))
    else:
        run(args)


if __name__ == "__main__":
    main()
