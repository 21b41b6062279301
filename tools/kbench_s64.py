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


def timeit(fn, iters=30, reps=20):
    """Median device time of one call: ``reps`` calls captured into a HIP graph
    and replayed (host launch overhead out of the measurement -- event pairs
    around a single eager call include ~10 us of host time per call)."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        e.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(e) * 1e3 / reps)
    ts.sort()
    return ts[len(ts) // 2]


SHAPES = ((32, 8, 512, 512), (32, 16, 256, 256), (32, 8, 1024, 512), (32, 16, 512, 256), (64, 8, 512, 512),
          (16, 8, 512, 512), (24, 8, 512, 512), (31, 8, 512, 512), (33, 8, 512, 512), (40, 8, 512, 512))


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="0,1,2,3,4", help="indices into SHAPES (N, H, IC, OC)")
    ap.add_argument("--cfgs", default="1,2,3,4,0")
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--dgrad", action="store_true", help="also time the input gradient (TRANS)")
    ap.add_argument("--hsm", default="0", help="small-image halo conv settings to run (0 off, 1 auto, 2/3/4: 1/2/3-4 wave groups)")
    a = ap.parse_args()
    torch.manual_seed(0)
    for si in [int(v) for v in a.shapes.split(",")]:
        N, Hh, IC, OC = SHAPES[si]
        x = torch.randn(N, Hh, Hh, IC, device="cuda").to(BF)
        w = torch.randn(OC, IC, 3, 3, device="cuda") * 0.03
        g = torch.randn(N, Hh, Hh, OC, device="cuda").to(BF)
        fl = 2.0 * N * Hh * Hh * IC * OC * 9
        wpf, wpt = H.packed_weight(w, False), H.packed_weight(w, True)
        # packed operands are flat: [OCp128][9][ICp64] and (transposed) [ICp128][9][OCp64]
        ICp, OCp = (IC + 63) // 64 * 64, (OC + 63) // 64 * 64
        assert wpf.numel() == (OC + 127) // 128 * 128 * 9 * ICp, wpf.shape
        assert wpt.numel() == (IC + 127) // 128 * 128 * 9 * OCp, wpt.shape
        y = torch.empty(N, Hh, Hh, OC, device="cuda", dtype=BF)
        dx = torch.empty(N, Hh, Hh, IC, device="cuda", dtype=BF)

        def fwd():
            H._conv_fwd(x, wpf, None, None, None, y, N, Hh, Hh, IC, ICp, Hh, Hh, OC, OC, 1, False, 1.0)

        def bwd():
            H._conv_fwd(g, wpt, None, None, None, dx, N, Hh, Hh, OC, OCp, Hh, Hh, IC, IC, 1, True, 1.0)

        ref = None
        for hsm, cfg in [(int(h), int(v)) for h in a.hsm.split(",") for v in a.cfgs.split(",")]:
            H._lib.d3d_conv_hsm_cfg(hsm)
            H._lib.d3d_conv_s64_cfg(cfg)
            for name, fn, out in (("fwd", fwd, y), ("dgrad", bwd, dx))[: 2 if a.dgrad else 1]:
                fn()
                torch.cuda.synchronize()
                if ref is None or name not in ref:
                    ref = dict(ref or {}, **{name: out.float().clone()})
                err = ((out.float() - ref[name]).norm() / ref[name].norm()).item()
                us = timeit(fn, a.iters)
                print(f"{N}x{Hh}x{Hh} {IC}->{OC} {name} hsm{hsm} cfg{cfg}: {us:7.1f} us {fl / us / 1e6:6.1f} TF/s  "
                      f"rel-vs-first {err:.1e}", flush=True)
        H._lib.d3d_conv_s64_cfg(0)
        H._lib.d3d_conv_hsm_cfg(1)


if __name__ == "__main__":
    main()
