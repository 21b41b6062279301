"""The level-0 conditioning conv (51 ray-direction channels padded to 64 ->
emb_ch 1024 at 64x64, per-image bias, frame-broadcast residual, SiLU
companion output) on each conv kernel family, timed by graph replay.

    python tools/kbench_cond_conv.py [frames]        (default 256 = bs128; 32 = bs16)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from distributed_3d_diffusion_pytorch_amd.ops import hip_impl as H

BF = torch.bfloat16


def timeit(fn, iters=15, reps=5):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        with torch.cuda.graph(g, stream=st):
            for _ in range(reps):
                fn()
    torch.cuda.current_stream().wait_stream(st)
    ts = []
    for _ in range(iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        g.replay()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) * 1e3 / reps)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    Hh, IC, OC = 64, 64, 1024
    torch.manual_seed(0)
    x = torch.randn(N, Hh, Hh, IC, device="cuda").to(BF)
    w = torch.randn(OC, IC, 3, 3, device="cuda") * 0.03
    wp = H.packed_weight(w, False)
    assert wp.numel() == (OC + 127) // 128 * 128 * 9 * IC
    b = torch.randn(OC, device="cuda") * 0.1
    rb = torch.randn(N, OC, device="cuda") * 0.1
    res = torch.randn(2, Hh, Hh, OC, device="cuda").to(BF)
    out = torch.empty(N, Hh, Hh, OC, device="cuda", dtype=BF)
    so = torch.empty_like(out)
    fl = 2.0 * N * Hh * Hh * IC * OC * 9
    ref = None
    for impl in ("halo", "w8", "bufl"):
        H.set_conv_impl(impl)
        for silu in (True, False):
            fn = lambda: H._conv_fwd(x, wp, b, rb, res, out, N, Hh, Hh, IC, IC, Hh, Hh, OC, OC, 1, False, 1.0, 2, 9,
                                     silu_out=so if silu else None)
            fn()
            torch.cuda.synchronize()
            if ref is None:
                ref = out.float().clone()
            err = ((out.float() - ref).norm() / ref.norm()).item()
            us = timeit(fn)
            print(f"N{N} cond conv {IC}->{OC} {impl:8s} silu_out={int(silu)}: {us:8.1f} us {fl / us / 1e6:7.1f} TF/s "
                  f"rel {err:.1e}", flush=True)
    H.set_conv_impl("halo")


if __name__ == "__main__":
    main()
