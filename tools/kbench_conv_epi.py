"""3x3 conv (N frames x HxH, C -> C; default the level-0 64x64 128 -> 128) forward with the epilogue
options the model uses (bias, residual, fused GroupNorm partials) against the
transposed (dgrad) launch of the same kernel: isolates epilogue cost."""
import math
import sys

import torch

from distributed_3d_diffusion_pytorch_amd.ops import hip_impl as H

BF = torch.bfloat16
dev = "cuda"
N = int(sys.argv[1]) if len(sys.argv) > 1 else 128
Hh = int(sys.argv[2]) if len(sys.argv) > 2 else 64
C = int(sys.argv[3]) if len(sys.argv) > 3 else 128
print(f"N{N} {Hh}x{Hh} {C}->{C}", flush=True)


def timeit(fn, iters=20):
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
x = torch.randn(N, Hh, Hh, C, device=dev).to(BF)
w = torch.randn(C, C, 3, 3, device=dev) / math.sqrt(9 * C)
b = torch.randn(C, device=dev)
r = torch.randn(N, Hh, Hh, C, device=dev).to(BF)
y = torch.empty_like(x)
wp = H.packed_weight(w, False, 9)
wt = H.packed_weight(w, True, 9)
fl = 2.0 * N * Hh * Hh * C * C * 9
for name, kw in [("fwd plain", dict(bias=None, res=None, gn=0)), ("fwd bias", dict(bias=b, res=None, gn=0)),
                 ("fwd bias+gn", dict(bias=b, res=None, gn=32)), ("fwd bias+res", dict(bias=b, res=r, gn=0)),
                 ("fwd bias+res+gn", dict(bias=b, res=r, gn=32))]:
    us = timeit(lambda: H._conv_fwd(x, wp, kw["bias"], None, kw["res"], y, N, Hh, Hh, C, C, Hh, Hh, C, C, 1, False,
                                    0.7, 0, 9, kw["gn"]))
    print(f"{name:18s} {us:8.1f} us  {fl / us / 1e6:7.1f} TF/s", flush=True)
us = timeit(lambda: H._conv_fwd(x, wt, None, None, None, y, N, Hh, Hh, C, C, Hh, Hh, C, C, 1, True, 1.0))
print(f"{'dgrad':18s} {us:8.1f} us  {fl / us / 1e6:7.1f} TF/s", flush=True)
