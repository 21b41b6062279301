"""Small-grid conv (conv_small.hip) wave-group configurations at the batch-16
level shapes: forward and input gradient, time and TF/s per configuration
(1: one 4-wave group, 2 / 4: two / four groups with 2-stage rings, 3: two
groups with 4-stage rings, 0: the automatic choice)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from distributed_3d_diffusion_pytorch_amd.ops import hip_impl as H

BF = torch.bfloat16


def timeit(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    torch.manual_seed(0)
    for N, Hh, C in ((32, 8, 512), (32, 16, 256), (64, 8, 512), (32, 8, 1024)):
        x = torch.randn(N, Hh, Hh, C, device="cuda").to(BF)
        w = torch.randn(C, C, 3, 3, device="cuda") * 0.03
        fl = 2.0 * N * Hh * Hh * C * C * 9
        ref = None
        for cfg in (1, 2, 3, 4, 0):
            H._lib.d3d_conv_s64_cfg(cfg)
            with torch.no_grad():
                y = H.conv3x3(x, w, None)
                if ref is None:
                    ref = y.float()
                err = ((y.float() - ref).norm() / ref.norm()).item()
                us = timeit(lambda: H.conv3x3(x, w, None))
            print(f"{N}x{Hh}x{Hh}x{C} fwd cfg{cfg}: {us:7.1f} us {fl / us / 1e6:6.1f} TF/s  rel-vs-cfg1 {err:.1e}",
                  flush=True)
        H._lib.d3d_conv_s64_cfg(0)


if __name__ == "__main__":
    main()
