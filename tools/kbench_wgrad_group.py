"""Grouped weight gradients vs one launch pair per job, on the job batches of
one 16-example (8-GPU share) backward: 8-job flushes per level as the sink
issues them.  Prints per-batch device time of (a) the per-job split-K path
(ops.hip_impl._wgrad: kernel + per-job slab reduce) and (b) the grouped launch
(wgrad_group.hip), with model TF/s.

    python tools/kbench_wgrad_group.py [--examples 16] [--pk 32] [--blocks 512]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_3d_diffusion_pytorch_amd.ops import hip_impl as H  # noqa: E402

BF = torch.bfloat16


def batches(n_img):
    """(name, [(N, H, W, IC, OC, taps)]) -- representative 8-job flushes."""
    N = n_img
    return [
        ("L0 3x3 128", [(N, 64, 64, 128, 128, 9)] * 8),
        ("L0 dec", [(N, 64, 64, 384, 128, 9), (N, 64, 64, 128, 128, 9), (N * 4096, 1, 1, 384, 128, 1),
                    (N, 64, 64, 256, 128, 9), (N, 64, 64, 128, 128, 9), (N * 4096, 1, 1, 256, 128, 1),
                    (N, 64, 64, 256, 128, 9), (N, 64, 64, 128, 128, 9)]),
        ("L1 3x3 256", [(N, 32, 32, 256, 256, 9)] * 8),
        ("L2 attn", [(N, 16, 16, 256, 256, 9), (N * 256, 1, 1, 256, 256, 1), (N * 256, 1, 1, 256, 512, 1),
                     (N * 256, 1, 1, 256, 256, 1), (N * 256, 1, 1, 256, 256, 1), (N, 16, 16, 256, 256, 9),
                     (N * 256, 1, 1, 256, 512, 1), (N * 256, 1, 1, 256, 256, 1)]),
        ("L3 attn", [(N, 8, 8, 512, 512, 9), (N * 64, 1, 1, 512, 512, 1), (N * 64, 1, 1, 512, 1024, 1),
                     (N * 64, 1, 1, 512, 512, 1), (N * 64, 1, 1, 512, 512, 1), (N, 8, 8, 512, 512, 9),
                     (N * 64, 1, 1, 512, 1024, 1), (N * 64, 1, 1, 512, 512, 1)]),
        ("L3 dec", [(N, 8, 8, 1024, 512, 9), (N, 8, 8, 512, 512, 9), (N * 64, 1, 1, 1024, 512, 1),
                    (N, 8, 8, 768, 512, 9), (N, 8, 8, 512, 512, 9), (N * 64, 1, 1, 768, 512, 1),
                    (N * 64, 1, 1, 512, 512, 1), (N * 64, 1, 1, 512, 1024, 1)]),
    ]


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3       # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--examples", type=int, default=16)
    ap.add_argument("--pk", type=int, default=32)
    ap.add_argument("--blocks", type=int, default=512)
    ap.add_argument("--minpix", type=int, default=512)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="", help="comma-separated batch-name prefixes")
    ap.add_argument("--skip_old", action="store_true", help="time the grouped launch only")
    a = ap.parse_args()
    H._ensure_impl()
    H._lib.d3d_wgrad_group_cfg(a.blocks, a.pk, a.minpix)
    dev = torch.device("cuda")
    torch.manual_seed(0)
    for name, spec in batches(2 * a.examples):
        if a.only and not any(name.startswith(o.replace("_", " ")) for o in a.only.split(",")):
            continue
        tens = []
        flops = 0.0
        for (N, Hh, W, IC, OC, taps) in spec:
            g = torch.randn(N, Hh, W, OC, device=dev).to(BF)
            x = torch.randn(N, Hh, W, IC, device=dev).to(BF)
            dw = torch.zeros(OC, IC, taps, device=dev)
            db = torch.zeros(OC, device=dev)
            tens.append((g, x, dw, db, N, Hh, W, IC, OC, taps))
            flops += 2.0 * N * Hh * W * OC * IC * taps

        def old():
            for (g, x, dw, db, N, Hh, W, IC, OC, taps) in tens:
                H._wgrad(g, x, OC, IC, N, Hh, W, Hh, W, 1, taps, dW=dw, db=db, accumulate=True)

        jobs = [H.wgrad_job(g, x, OC, IC, N, Hh, W, taps, dw, db) for (g, x, dw, db, N, Hh, W, IC, OC, taps) in tens]
        assert all(j is not None for j in jobs)

        def new():
            H.wgrad_group_run(jobs)

        t_old = float("nan") if a.skip_old else timeit(old, a.iters)
        t_new = timeit(new, a.iters)
        print(json.dumps({"batch": name, "gflop": round(flops / 1e9, 1), "old_us": round(t_old, 1),
                          "new_us": round(t_new, 1), "old_tfs": round(flops / t_old / 1e6, 1),
                          "new_tfs": round(flops / t_new / 1e6, 1), "pk": a.pk, "blocks": a.blocks}), flush=True)


if __name__ == "__main__":
    main()
