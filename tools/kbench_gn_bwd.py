"""GroupNorm backward (statistics-reduce + apply) at the X-UNet level shapes
for a frame batch N: time per mode (0 GN, 1 GN+SiLU, 2 GN+FiLM)."""
import sys

import torch

from distributed_3d_diffusion_pytorch_amd.ops import hip_impl as H

BF = torch.bfloat16
dev = "cuda"
N = int(sys.argv[1]) if len(sys.argv) > 1 else 32


def timeit(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


torch.manual_seed(0)
for Hh, C in ((64, 128), (32, 256), (16, 256), (8, 512)):
    x = torch.randn(N, Hh, Hh, C, device=dev).to(BF)
    dy = torch.randn_like(x)
    w = torch.rand(C, device=dev) + 0.5
    b = torch.randn(C, device=dev) * 0.1
    ss = (torch.randn(N, Hh, Hh, 2 * C, device=dev) * 0.3).to(BF)
    for mode in (0, 1, 2):
        y, stats = H._gn_fwd(mode, x, w, b, 32, 1e-5, ss if mode == 2 else None, 0, 0.0, 0)
        us = timeit(lambda: H._gn_bwd(mode, x, dy, ss if mode == 2 else None, stats, w, b, 32, 0.0, 0))
        mb = x.numel() * 2 * (3 if mode < 2 else 7) / 1e6
        print(f"N{N} {Hh}x{Hh}x{C} mode {mode}: {us:7.1f} us  ({mb / us:5.2f} TB/s over the 2 passes)", flush=True)
