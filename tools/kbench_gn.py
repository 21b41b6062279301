"""GroupNorm backward (reduce + apply) in isolation on the X-UNet level shapes,
as the training step launches it: GN+SiLU with a residual-branch gradient
(dres), GN+FiLM(+dropout) and the decoder's virtual-concat GN+SiLU.  JSON lines
with median device time and achieved HBM bandwidth (bytes the two passes must
move: reduce reads x, dy (, ss); apply reads x, dy (, ss, dres), writes dx).

    python tools/kbench_gn.py [N frames ...]     (default: 32 256 = bs16, bs128)
    D3D_GN_CFG=blocks,red_u,app_u  selects the launch shape (ops/csrc/norm.hip)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from distributed_3d_diffusion_pytorch_amd.ops import hip_impl as H

BF = torch.bfloat16


def timeit(fn, iters=25):
    for _ in range(4):
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
    ns = [int(a) for a in sys.argv[1:]] or [32, 256]
    H._ensure_impl()
    G = 32
    cfg = os.environ.get("D3D_GN_CFG", "default")
    for N in ns:
        for Hh, C, C1 in ((64, 128, 0), (32, 256, 0), (16, 256, 0), (8, 512, 0), (64, 256, 128), (32, 512, 256)):
            P = Hh * Hh
            x = torch.randn(N, Hh, Hh, C if not C1 else C1, device="cuda").to(BF)
            x2 = torch.randn(N, Hh, Hh, C - C1, device="cuda").to(BF) if C1 else None
            w = torch.rand(C, device="cuda") + 0.5
            b = torch.randn(C, device="cuda") * 0.1
            dy = torch.randn(N, Hh, Hh, C, device="cuda").to(BF)
            dres = torch.randn(N, Hh, Hh, C, device="cuda").to(BF) if not C1 else None
            ss = torch.randn(N, Hh, Hh, 2 * C, device="cuda").to(BF) * 0.1
            t = N * P * C * 2
            stats = torch.stack([torch.zeros(N * G), torch.ones(N * G)], 1).reshape(-1).cuda()
            rows = []
            for mode in ((1, 2) if not C1 else (1,)):
                if mode == 1:
                    fn = lambda: H._gn_bwd(1, x, dy, None, stats, w, b, G, 0.0, 0, x2=x2, dres=dres, dres_scale=0.7)
                    nbytes = 2 * t + (4 * t if dres is not None else 3 * t)
                else:
                    fn = lambda: H._gn_bwd(2, x, dy, ss, stats, w, b, G, 0.1, 7, ssld=2 * C)
                    nbytes = 3 * t + 2 * t + 4 * t      # reduce: x, dy, ss + dss (2t); apply: x, dy, ss, dx
                us = timeit(fn)
                rows.append({"cfg": cfg, "N": N, "level": f"{Hh}x{Hh}x{C}" + (f" cat{C1}" if C1 else ""),
                             "mode": mode, "us": round(us, 1), "TBps": round(nbytes / us / 1e6, 2)})
            for r in rows:
                print(json.dumps(r), flush=True)
            del x, x2, dy, dres, ss
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
