"""3x3 conv kernel family by size rule at the per-GPU share of the 8-GPU job
(bs16 = 32 frames): forward (bias + residual + scale + GroupNorm partials, the
step's epilogue) and input gradient for the 64x64x128 and 32x32x256 levels,
under each conv implementation ceiling (halo > w8n > w8w > w8 > bufl), so the
size rule's choice at small grids can be checked against the alternatives.
usage: python tools/kbench_conv_impl_small.py [N frames ...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from distributed_3d_diffusion_pytorch_amd.ops import hip_impl as H

BF = torch.bfloat16


def timeit(fn, iters=30):
    for _ in range(5):
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
    ns = [int(a) for a in sys.argv[1:]] or [32, 64]
    for N in ns:
        for Hh, C in ((64, 128), (32, 256)):
            x = torch.randn(N, Hh, Hh, C, device="cuda").to(BF)
            w = torch.randn(C, C, 3, 3, device="cuda") * 0.03
            b = torch.randn(C, device="cuda") * 0.1
            r = torch.randn(N, Hh, Hh, C, device="cuda").to(BF)
            fl = 2.0 * N * Hh * Hh * C * C * 9
            for impl in ("halo", "w8n", "w8w", "w8", "bufl"):
                H.set_conv_impl(impl)
                with torch.no_grad():
                    f = timeit(lambda: H.conv3x3(x, w, b, residual=r, out_scale=0.7071, gn_groups=32))
                xr = x.clone().requires_grad_(True)
                y = H.conv3x3(xr, w, None)
                g = torch.randn_like(y)
                d = timeit(lambda: torch.autograd.grad(y, xr, g, retain_graph=True))
                print(f"N{N:<4} {Hh}x{Hh}x{C} {impl:5s} fwd {f:7.1f} us {fl / f / 1e6:6.1f} TF/s   "
                      f"dgrad {d:7.1f} us {fl / d / 1e6:6.1f} TF/s", flush=True)
                del xr, y, g
            H.set_conv_impl("halo")
            del x, r
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
