"""3x3 convs of the four X-UNet levels in isolation, as the training step
launches them: forward without residual (a ResnetBlock's conv1: bias + GN
partials), forward with residual + 1/sqrt2 (conv2), and the input gradient.
JSON lines with median device time and TF/s.

    python tools/kbench_conv_levels.py [N frames ...]     (default: 32 256 = bs16, bs128)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from distributed_3d_diffusion_pytorch_amd.ops import hip_impl as H

BF = torch.bfloat16


def timeit(fn, iters=25, reps=10):
    """Median device time of one call: ``reps`` calls captured into a HIP graph
    and replayed (an event pair around one eager call also counts ~10 us of
    host launch time -- the round-4 numbers of this tool carried it)."""
    for _ in range(3):
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
    g.replay()
    torch.cuda.synchronize()
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
    ns = [int(a) for a in sys.argv[1:]] or [32, 256]
    H._ensure_impl()
    H._lib.d3d_conv_res_cfg(int(os.environ.get("D3D_CONV_RES_ALWAYS", "0")))
    for N in ns:
        levels = [(64, 128, 128), (32, 256, 256), (16, 256, 256), (8, 512, 512)]
        if os.environ.get("KB_CONV_EXTRA"):             # level-entry convs (channel change) and decoder concat widths
            levels = [(32, 128, 256), (16, 256, 256), (8, 256, 512), (64, 384, 128), (64, 256, 128), (32, 512, 256),
                      (32, 384, 256)]
        if os.environ.get("KB_CONV_128"):               # 128x128 images (BASELINE config 4)
            levels = [(128, 128, 128), (64, 256, 256)]
        for Hh, C, OC in levels:
            x = torch.randn(N, Hh, Hh, C, device="cuda").to(BF)
            w = torch.randn(OC, C, 3, 3, device="cuda") * 0.03
            b = torch.randn(OC, device="cuda") * 0.1
            r = torch.randn(N, Hh, Hh, OC, device="cuda").to(BF)
            fl = 2.0 * N * Hh * Hh * C * OC * 9
            with torch.no_grad():
                f1 = timeit(lambda: H.conv3x3(x, w, b, gn_groups=32))
                f2 = timeit(lambda: H.conv3x3(x, w, b, residual=r, out_scale=0.7071, gn_groups=32))
            # input gradient: the transposed-weight conv the backward launches
            g = torch.randn(N, Hh, Hh, OC, device="cuda").to(BF)
            wpt = H.packed_weight(w, True)
            OCp = (OC + 63) // 64 * 64
            assert wpt.numel() == (C + 127) // 128 * 128 * 9 * OCp
            dx = torch.empty(N, Hh, Hh, C, device="cuda", dtype=BF)
            d = timeit(lambda: H._conv_fwd(g, wpt, None, None, None, dx, N, Hh, Hh, OC, OCp, Hh, Hh, C, C, 1, True,
                                           1.0))
            print(json.dumps({"res_always": os.environ.get("D3D_CONV_RES_ALWAYS", "0"), "N": N, "level": f"{Hh}x{Hh}x{C}->{OC}", "fwd_us": round(f1, 1),
                              "fwd_tfs": round(fl / f1 / 1e6, 1), "fwd_res_us": round(f2, 1),
                              "fwd_res_tfs": round(fl / f2 / 1e6, 1), "dgrad_us": round(d, 1),
                              "dgrad_tfs": round(fl / d / 1e6, 1)}), flush=True)
            del x, r, g, dx
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
