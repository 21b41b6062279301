"""Level-0 (64x64, 128 -> 128) 3x3 conv at bs128 (256 frames): forward time by
epilogue variant (plain / bias / residual+scale / GroupNorm partials / all) and
the input gradient, in isolation (events, median of 20)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from distributed_3d_diffusion_pytorch_amd.ops import hip_impl as H

BF = torch.bfloat16
dev = "cuda"


def timeit(fn, iters=20):
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
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    for Hh, C in ((64, 128), (32, 256)):
        x = torch.randn(N, Hh, Hh, C, device=dev).to(BF)
        w = torch.randn(C, C, 3, 3, device=dev) * 0.03
        b = torch.randn(C, device=dev) * 0.1
        r = torch.randn(N, Hh, Hh, C, device=dev).to(BF)
        fl = 2.0 * N * Hh * Hh * C * C * 9
        with torch.no_grad():
            for name, kw in (("plain", {}), ("bias", {"b": b}), ("res+scale", {"residual": r, "out_scale": 0.7071}),
                             ("gn", {"gn_groups": 32}), ("bias+gn", {"b": b, "gn_groups": 32}),
                             ("all", {"b": b, "residual": r, "out_scale": 0.7071, "gn_groups": 32})):
                bb = kw.pop("b", None)
                us = timeit(lambda: H.conv3x3(x, w, bb, **kw))
                print(f"{Hh}x{Hh}x{C} N{N} fwd {name:10s} {us:8.1f} us {fl / us / 1e6:7.1f} TF/s", flush=True)
        xr = x.clone().requires_grad_(True)
        y = H.conv3x3(xr, w.requires_grad_(False), None)
        g = torch.randn_like(y)
        us = timeit(lambda: torch.autograd.grad(y, xr, g, retain_graph=True))
        print(f"{Hh}x{Hh}x{C} N{N} dgrad      {us:8.1f} us {fl / us / 1e6:7.1f} TF/s", flush=True)
        us = timeit(lambda: H._wgrad(g, x, C, C, N, Hh, Hh, Hh, Hh, 1, 9, want_bias=True))
        print(f"{Hh}x{Hh}x{C} N{N} wgrad      {us:8.1f} us {fl / us / 1e6:7.1f} TF/s", flush=True)
        del x, r, y, g, xr
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
