#!/usr/bin/env python
"""Per-kernel micro-benchmark for the gfx950 HIP ops (TFLOP/s / GB/s on the
X-UNet's real shapes), HIP vs the torch/MIOpen/hipBLASLt composition.

    python tools/kbench.py [--ops conv,wgrad,dgrad,linear,attn,gn] [--batch 128] [--iters 20]

Writes one JSON line per (op, shape, backend).  Interleaves backends in one
process (cdna guide 5.4 rule 24) and uses random data (rule 25).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_3d_diffusion_pytorch_amd.ops import hip_impl as H, torch_impl as T  # noqa: E402

BF = torch.bfloat16


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def conv_shapes(N):
    # (H, Cin, Cout, stride) of the 64x64 X-UNet at frame-batch N (=2B)
    return [(64, 128, 128, 1), (32, 256, 256, 1), (16, 256, 256, 1), (8, 512, 512, 1), (64, 384, 128, 1),
            (32, 512, 256, 1), (8, 1024, 512, 1), (64, 144, 1024, 1), (64, 144, 1024, 2)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ops", default="conv,dgrad,wgrad,linear,attn,gn")
    ap.add_argument("--batch", type=int, default=64, help="examples (frame batch N = 2*batch)")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--torch", action="store_true", help="also time the torch composition")
    ap.add_argument("--only_glds_check", action="store_true")
    a = ap.parse_args()
    dev = "cuda"
    N = 2 * a.batch
    ops = a.ops.split(",")
    torch.manual_seed(0)
    out = []

    def rep(op, shape, backend, sec, flops=None, nbytes=None):
        r = {"op": op, "shape": shape, "backend": backend, "us": round(sec * 1e6, 2)}
        if flops:
            r["tflops"] = round(flops / sec / 1e12, 1)
        if nbytes:
            r["gbps"] = round(nbytes / sec / 1e9, 1)
        print(json.dumps(r), flush=True)
        out.append(r)

    for (Hh, Ci, Co, s) in conv_shapes(N):
        x = torch.randn(N, Hh, Hh, Ci, device=dev).to(BF)
        w = torch.randn(Co, Ci, 3, 3, device=dev) / math.sqrt(9 * Ci)
        b = torch.randn(Co, device=dev)
        OH = (Hh - 1) // s + 1
        fl = 2.0 * N * OH * OH * Co * Ci * 9
        shp = f"N{N} H{Hh} {Ci}->{Co} s{s}"
        wp = H.packed_weight(w, False, 9)
        y = torch.empty(N, OH, OH, Co, dtype=BF, device=dev)
        g = torch.randn(N, OH, OH, Co, device=dev).to(BF)
        if "conv" in ops:
            for impl in ("w8w", "halo"):
                H.set_conv_impl(impl)
                rep("conv_fwd", shp, "hip-" + impl,
                    timeit(lambda: H._conv_fwd(x, wp, b, None, None, y, N, Hh, Hh, Ci, H._up(Ci, 64), OH, OH, Co, Co,
                                               s, False, 1.0), a.iters), fl)
            H.set_conv_impl("bufl")
            if a.torch:
                wb, bb = w.to(BF), b.to(BF)
                xc = x.permute(0, 3, 1, 2)
                rep("conv_fwd", shp, "miopen", timeit(lambda: torch.nn.functional.conv2d(xc, wb, bb, s, 1),
                                                      a.iters), fl)
        if "dgrad" in ops and s == 1:
            wt = H.packed_weight(w, True, 9)
            dx = torch.empty_like(x)
            for impl in ("w8w", "halo"):
                H.set_conv_impl(impl)
                rep("conv_dgrad", shp, "hip-" + impl,
                    timeit(lambda: H._conv_fwd(g, wt, None, None, None, dx, N, OH, OH, Co, H._up(Co, 64), Hh, Hh, Ci,
                                               Ci, s, True, 1.0), a.iters), fl)
            H.set_conv_impl("bufl")
        if "wgrad" in ops:
            for impl in ("bufl", "w8"):
                H.set_wgrad_impl(impl)
                rep("conv_wgrad", shp, "hip-" + impl,
                    timeit(lambda: H._wgrad(g, x, Co, Ci, N, Hh, Hh, OH, OH, s, 9), a.iters), fl)
            H.set_wgrad_impl("bufl")
    if "linear" in ops:
        for (P, Ci, Co) in [(N * 4096, 1024, 2048), (N * 1024, 1024, 4608), (N * 256, 1024, 4608),
                            (N * 64, 1024, 3072), (N * 256, 256, 768), (N * 64, 512, 1536), (N * 4096, 384, 128),
                            (N * 4096, 256, 128), (N * 1024, 512, 256)]:
            x = torch.randn(P, Ci, device=dev).to(BF)
            w = torch.randn(Co, Ci, device=dev) / math.sqrt(Ci)
            b = torch.randn(Co, device=dev)
            fl = 2.0 * P * Ci * Co
            shp = f"P{P} {Ci}->{Co}"
            x4 = x.reshape(P, 1, 1, Ci)
            wp = H.packed_weight(w, False, 1)
            y = torch.empty(P, 1, 1, Co, dtype=BF, device=dev)
            g = torch.randn(P, 1, 1, Co, device=dev).to(BF)
            for impl in ("bufl1", "w8w"):
                H.set_conv_impl(impl)
                rep("lin_fwd", shp, "hip-" + impl,
                    timeit(lambda: H._conv_fwd(x4, wp, b, None, None, y, P, 1, 1, Ci, H._up(Ci, 64), 1, 1, Co, Co, 1,
                                               False, 1.0, 0, 1), a.iters), fl)
            H.set_conv_impl("w8w")
            wt = H.packed_weight(w, True, 1)
            g4 = torch.randn(P, 1, 1, Co, device=dev).to(BF)
            dx = torch.empty(P, 1, 1, Ci, dtype=BF, device=dev)
            if P * Co * 2 < (1 << 31):
                rep("lin_dgrad", shp, "hip-w8w", timeit(lambda: H._conv_fwd(g4, wt, None, None, None, dx, P, 1, 1, Co,
                                                                              H._up(Co, 64), 1, 1, Ci, Ci, 1, False,
                                                                              1.0, 0, 1), a.iters), fl)
            if a.torch:
                wb = w.to(BF)
                g2 = g4.reshape(P, Co)
                rep("lin_dgrad", shp, "hipblaslt", timeit(lambda: torch.mm(g2, wb), a.iters), fl)
            for impl in ("reg", "bufl"):
                H.set_wgrad_impl(impl)
                rep("lin_wgrad", shp, "hip-" + impl, timeit(lambda: H._wgrad(g, x4, Co, Ci, P, 1, 1, 1, 1, 1, 1),
                                                             a.iters), fl)
            H.set_wgrad_impl("bufl")
            if a.torch:
                wb = w.to(BF)
                rep("lin_fwd", shp, "hipblaslt", timeit(lambda: torch.addmm(b.to(BF), x, wb.t()), a.iters), fl)
                g2 = g.reshape(P, Co)
                rep("lin_wgrad", shp, "hipblaslt", timeit(lambda: H._mm_f32(g2.t(), x), a.iters), fl)
    if "attn" in ops:
        for (L, C) in [(256, 256), (64, 512), (1024, 256)]:
            qkv = torch.randn(N, L, 3 * C, device=dev).to(BF)
            fl = 4.0 * N * L * L * C
            shp = f"N{N} L{L} C{C}"
            rep("attn_fwd", shp, "hip", timeit(lambda: H.attention(qkv, 4, True), a.iters), fl)
            q = qkv.clone().requires_grad_(True)
            o = H.attention(q, 4, True)
            go = torch.randn_like(o)
            rep("attn_fwd_bwd", shp, "hip",
                timeit(lambda: torch.autograd.grad(H.attention(q, 4, True), q, go), a.iters), 3.5 * fl)
    if "gn" in ops:
        for (Hh, C) in [(64, 128), (32, 256), (8, 512)]:
            x = torch.randn(N, Hh, Hh, C, device=dev).to(BF)
            w, b = torch.ones(C, device=dev), torch.zeros(C, device=dev)
            ss = torch.randn(N, Hh, Hh, 2 * C, device=dev).to(BF)
            nb = x.numel() * 2
            rep("gn_silu", f"N{N} H{Hh} C{C}", "hip", timeit(lambda: H.group_norm(x, w, b, 32, 1e-5, True), a.iters),
                nbytes=3 * nb)
            rep("gn_film", f"N{N} H{Hh} C{C}", "hip",
                timeit(lambda: H.gn_film(x, w, b, ss, 32, 1e-5, 0.1, True, 1), a.iters), nbytes=5 * nb)


if __name__ == "__main__":
    main()
