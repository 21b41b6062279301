"""Small-problem GEMM A/B: the 4-stage LDS ring (gemm.hip NST = 4) against the
2-stage ring on the bs16 shapes that are latency-bound (one or two 64 / 128
tiles per CU: attention projections and NIN skips at 8x8 .. 32x32 and their
input gradients).  Interleaved rounds in one process, one JSON line per shape.

    python tools/kbench_gemm_small.py [--rounds 3] [--iters 50]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_3d_diffusion_pytorch_amd.ops import hip_impl as H

BF = torch.bfloat16

# (label, M = output channels, N = pixels, K = reduction); bs16: 2B = 32 views
SHAPES = [
    ("8x8 proj 512->512", 512, 2048, 512),
    ("8x8 qkv dgrad 1536->512", 512, 2048, 1536),
    ("8x8 qkv fwd 512->1536", 1536, 2048, 512),
    ("16x16 proj 256->256", 256, 8192, 256),
    ("16x16 qkv dgrad 768->256", 256, 8192, 768),
    ("16x16 qkv fwd 256->768", 768, 8192, 256),
    ("16x16 proj 512->512", 512, 8192, 512),
    ("32x32 nin 512->256", 256, 32768, 512),
    ("32x32 proj 256->256", 256, 32768, 256),
    ("8x8 film 1024->4608", 4608, 2048, 1024),
]


def timeit(fn, iters):
    """GPU time per call: `iters` launches captured in one HIP graph and
    replayed (Python-issued launches of a ~5 us kernel measure the launch
    rate, not the kernel)."""
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    for label, M, N, K in SHAPES:
        a = torch.randn(M, K, device=dev).to(BF)
        b = torch.randn(N, K, device=dev).to(BF)
        out = torch.empty(N, M, device=dev, dtype=BF)
        ref = (b.float() @ a.float().t())
        res = {}
        modes = {"8": (-1, -3), "4": (-1, -4), "2": (-2, -4)}     # LDS stage ring depth
        for m in modes.values():
            for v in m:
                H._lib.d3d_gemm_tune(v, 0, 0)
            H.gemm_nt(a, b, out, M, N, K, K, K, M)
            torch.cuda.synchronize()
            err = ((out.float() - ref).norm() / ref.norm()).item()
            assert err < 1e-2, (label, m, err)
        best = {k: 1e9 for k in modes}
        for _ in range(args.rounds):
            for k, m in modes.items():
                for v in m:
                    H._lib.d3d_gemm_tune(v, 0, 0)
                t = timeit(lambda: H.gemm_nt(a, b, out, M, N, K, K, K, M), args.iters)
                best[k] = min(best[k], t)
        H._lib.d3d_gemm_tune(-1, 0, 0)
        H._lib.d3d_gemm_tune(-4, 0, 0)
        fl = 2.0 * M * N * K
        res = {"shape": label, "M": M, "N": N, "K": K, **{f"nst{k}_us": round(v, 2) for k, v in best.items()},
               "tfs_best": round(fl / min(best.values()) / 1e6, 1)}
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
