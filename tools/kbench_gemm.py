"""Ping-pong MFMA GEMM (ops/csrc/gemm.hip) vs hipBLASLt (torch.mm) on the
X-UNet's dense-layer shapes and a square reference GEMM: correctness against
an fp32 product, then interleaved timing rounds in one process.

    python tools/kbench_gemm.py [--rounds 3] [--iters 20] [--only fwd|dgrad]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from distributed_3d_diffusion_pytorch_amd.ops import hip_impl as H

BF = torch.bfloat16

# (label, M = output channels, N = pixels, K = reduction)
SHAPES = [
    ("sq8192", 8192, 8192, 8192),
    ("film fwd P1048576 1024->2048", 2048, 1048576, 1024),
    ("film fwd P262144 1024->4608", 4608, 262144, 1024),
    ("film fwd P16384 1024->9216", 9216, 16384, 1024),
    ("film fwd P524288 1024->2048", 2048, 524288, 1024),
    ("film fwd P131072 1024->4608", 4608, 131072, 1024),
    ("film fwd P65536 1024->2048", 2048, 65536, 1024),
    ("film fwd P16384 1024->4608", 4608, 16384, 1024),
    ("k1024 M1024 P131072", 1024, 131072, 1024),
    ("film dgrad P1048576 2048->1024", 1024, 1048576, 2048),
    ("film dgrad P262144 4608->1024", 1024, 262144, 4608),
    ("film dgrad P524288 2048->1024", 1024, 524288, 2048),
    ("film dgrad P131072 4608->1024", 1024, 131072, 4608),
    ("film dgrad P16384 4608->1024", 1024, 16384, 4608),
    ("qkv fwd P131072 256->768", 768, 131072, 256),
    ("qkv fwd P32768 512->1536", 1536, 32768, 512),
    ("nin fwd P524288 256->128", 128, 524288, 256),
    ("nin fwd P131072 512->256", 256, 131072, 512),
    ("out fwd P32768 512->512", 512, 32768, 512),
    ("res proj P262144 256->256", 256, 262144, 256),
    ("res proj P65536 256->256", 256, 65536, 256),
    ("res proj P65536 512->512", 512, 65536, 512),
    ("res proj P16384 512->512", 512, 16384, 512),
    ("res nin P1048576 256->128", 128, 1048576, 256),
]


def timeit(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="")
    ap.add_argument("--vers", default="1", help="comma list of tile configs timed interleaved (1 = by size, 8 / 4 / 2 forced)")
    ap.add_argument("--gm", type=int, default=0, help="tile-group width (d3d_gemm_tune gm; 0 = default)")
    ap.add_argument("--nobias", action="store_true")
    ap.add_argument("--res", action="store_true", help="with a residual operand R [N, M] (F_RES epilogue)")
    ap.add_argument("--mf_ab", action="store_true", help="also time the generic epilogue (d3d_gemm_mf(0)) as v0")
    ap.add_argument("--waves_ab", action="store_true", help="also time the 4-wave 256x256 tile (d3d_gemm_w8_waves(4)) as v0")
    args = ap.parse_args()
    H._ensure_impl()
    lib = H._lib
    torch.manual_seed(0)
    for label, M, N, K in SHAPES:
        if args.only and args.only not in label:
            continue
        w = (torch.rand(M, K, device="cuda") * 2 - 1).to(BF)
        x = (torch.rand(N, K, device="cuda") * 2 - 1).to(BF)
        bias = None if args.nobias else torch.randn(M, device="cuda")
        y = torch.empty(N, M, dtype=BF, device="cuda")
        r = (torch.rand(N, M, device="cuda") * 2 - 1).to(BF) if args.res else None
        st = H._st()

        def sel(v):
            # v0: the A/B side (--mf_ab: generic epilogue, --waves_ab: 4-wave 256 tile)
            lib.d3d_gemm_mf(0 if (v == 0 and args.mf_ab) else 1)
            lib.d3d_gemm_w8_waves(4 if (v == 0 and args.waves_ab) else 8)
            lib.d3d_gemm_tune(v if v else 1, args.gm, 0)

        def ours(v=None):
            if v is not None:
                sel(v)
            rc = lib.d3d_gemm_nt(w.data_ptr(), x.data_ptr(), y.data_ptr(), H._ptr(bias), H._ptr(r), M, N, K, K, K,
                                 M, M, 1.0, 1.0, st)
            assert rc == 0, rc

        def blas():
            o = torch.addmm(bias.to(BF), x, w.t()) if bias is not None else torch.mm(x, w.t())
            return o.add_(r) if r is not None else o

        vers = [int(v) for v in args.vers.split(",")] + ([0] if (args.mf_ab or args.waves_ab) else [])
        rows = torch.randint(0, N, (256,), device="cuda")
        ref = x[rows].float() @ w.float().t() + (bias if bias is not None else 0) + (r[rows].float() if r is not None else 0)
        errs = {}
        for v in vers:
            y.zero_()
            ours(v)
            torch.cuda.synchronize()
            errs[v] = ((y[rows].float() - ref).norm() / ref.norm()).item()
        for _ in range(3):
            ours()
            blas()
        torch.cuda.synchronize()
        t_o, t_b = {v: [] for v in vers}, []
        for _ in range(args.rounds):
            for v in vers:
                sel(v)
                t_o[v].append(timeit(ours, args.iters))
            sel(1)
            t_b.append(timeit(blas, args.iters))
        fl = 2.0 * M * N * K
        b = min(t_b)
        rec = {"shape": label, "M": M, "N": N, "K": K, "blas_us": round(b, 1), "blas_tflops": round(fl / b / 1e6, 1)}
        for v in vers:
            o = min(t_o[v])
            rec[f"v{v}_err"] = round(errs[v], 5)
            rec[f"v{v}_us"] = round(o, 1)
            rec[f"v{v}_tflops"] = round(fl / o / 1e6, 1)
        print(json.dumps(rec), flush=True)
        del w, x, y


if __name__ == "__main__":
    main()
