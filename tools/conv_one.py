"""Run one conv shape (fwd or dgrad) with a chosen kernel impl, for rocprofv3
counter passes:  python tools/conv_one.py --impl w8 --n 128 --h 64 --ci 128 --co 128 [--dgrad]"""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--impl", default="w8")
    ap.add_argument("--n", type=int, default=128)
    ap.add_argument("--h", type=int, default=64)
    ap.add_argument("--ci", type=int, default=128)
    ap.add_argument("--co", type=int, default=128)
    ap.add_argument("--dgrad", action="store_true")
    ap.add_argument("--wgrad", default="", help="weight-gradient kernel impl (reg|bufl|...) instead of fwd")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from distributed_3d_diffusion_pytorch_amd.ops import hip_impl as H
    BF = torch.bfloat16
    H._ensure_impl()
    H.set_conv_impl(a.impl)
    N, Hh, Ci, Co = a.n, a.h, a.ci, a.co
    x = torch.randn(N, Hh, Hh, Ci, device="cuda").to(BF)
    w = torch.randn(Co, Ci, 3, 3, device="cuda") / math.sqrt(9 * Ci)
    b = torch.randn(Co, device="cuda")
    if a.wgrad:
        H.set_wgrad_impl(a.wgrad)
        g = torch.randn(N, Hh, Hh, Co, device="cuda").to(BF)
        fn = lambda: H._wgrad(g, x, Co, Ci, N, Hh, Hh, Hh, Hh, 1, 9)
    elif a.dgrad:
        g = torch.randn(N, Hh, Hh, Co, device="cuda").to(BF)
        wt = H.packed_weight(w, True, 9)
        dx = torch.empty_like(x)
        fn = lambda: H._conv_fwd(g, wt, None, None, None, dx, N, Hh, Hh, Co, H._up(Co, 64), Hh, Hh, Ci, Ci, 1, True, 1.0)
    else:
        wp = H.packed_weight(w, False, 9)
        y = torch.empty(N, Hh, Hh, Co, dtype=BF, device="cuda")
        fn = lambda: H._conv_fwd(x, wp, b, None, None, y, N, Hh, Hh, Ci, H._up(Ci, 64), Hh, Hh, Co, Co, 1, False, 1.0)
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / a.iters
    fl = 2.0 * N * Hh * Hh * Ci * Co * 9
    kind = 'wgrad-' + a.wgrad if a.wgrad else ('dgrad' if a.dgrad else 'fwd')
    print(f"{a.impl} N{N} H{Hh} {Ci}->{Co} {kind}: {us:.1f} us {fl / us / 1e6:.1f} TF/s")


if __name__ == "__main__":
    main()
