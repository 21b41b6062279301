"""GroupNorm roofline: every gn_* launch of the X-UNet step at its real
level shapes, timed in isolation, with the HBM bytes it must move and the
achieved TB/s.  Forward = statistics pass (when not fused into the producer)
+ fused finalize/apply; backward = reduce + apply (d3d_gn_bwd2).

Bytes counted (bf16 = 2 B, C-wide rows, N*P pixels):
  stats      : read x                                   (1 unit)
  apply m0/1 : read x, write y                          (2 units)
  apply m2   : read x, ss scale+shift (2C), write y     (4 units)
  bwd m0/1   : reduce read x, dy; apply read x, dy, write dx         (5 units)
  bwd m2     : reduce read x, dy, ss scale, write dss (2C);
               apply read x, dy, ss scale, write dx                   (9 units)
  (+1 unit when the residual-branch gradient dres is folded into the apply)

usage: python tools/kbench_gn.py [frames ...]   (default 256 = bs128, 32 = bs16)
Prints one JSON line per (frames, level, pass, mode)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

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
    frames = [int(a) for a in sys.argv[1:]] or [256, 32]
    torch.manual_seed(0)
    # (H, C, concat-C2): encoder level shapes and the decoder's widest concat
    levels = ((64, 128, 0), (64, 128, 128), (32, 256, 0), (32, 256, 256), (16, 256, 0), (8, 512, 0))
    for N in frames:
        for Hh, C1, C2 in levels:
            C = C1 + C2
            x = torch.randn(N, Hh, Hh, C1, device=dev).to(BF)
            x2 = torch.randn(N, Hh, Hh, C2, device=dev).to(BF) if C2 else None
            dy = torch.randn(N, Hh, Hh, C, device=dev).to(BF)
            dres = torch.randn(N, Hh, Hh, C, device=dev).to(BF)
            w = torch.rand(C, device=dev) + 0.5
            b = torch.randn(C, device=dev) * 0.1
            ss = (torch.randn(N, Hh, Hh, 2 * C, device=dev) * 0.3).to(BF) if not C2 else None
            unit = N * Hh * Hh * C * 2
            tag = f"{Hh}x{Hh}x{C1}" + (f"+{C2}" if C2 else "")
            modes = (1,) if C2 else (0, 1, 2)
            for mode in modes:
                sarg = ss if mode == 2 else None
                _, stats = H._gn_fwd(mode, x, w, b, 32, 1e-5, sarg, 0, 0.1 if mode == 2 else 0.0, 7, x2=x2)
                us = timeit(lambda: H._gn_fwd(mode, x, w, b, 32, 1e-5, sarg, 0, 0.1 if mode == 2 else 0.0, 7,
                                              x2=x2))
                units = 3 if mode < 2 else 5          # stats read + apply
                print(json.dumps({"frames": N, "level": tag, "pass": "fwd(stats+apply)", "mode": mode,
                                  "us": round(us, 1), "GB": round(units * unit / 1e9, 3),
                                  "TBps": round(units * unit / us / 1e6, 2)}), flush=True)
                if not C2:
                    # apply alone, statistics partials handed over as if from the producer's epilogue
                    P = Hh * Hh
                    nch, _ = H._gn_plan(N, P, C)
                    part = torch.empty(N * nch * 32 * 2, dtype=torch.float32, device=dev)
                    H._chk(H._lib.d3d_gn_stats(x.data_ptr(), N, P, C, 32, 1e-5, part.data_ptr(), None, None, 0,
                                               H._st()), "gn_stats")
                    x._d3d_gnpart = (part, 32, 0)
                    us = timeit(lambda: H._gn_fwd(mode, x, w, b, 32, 1e-5, sarg, 0, 0.1 if mode == 2 else 0.0, 7))
                    del x._d3d_gnpart
                    units = 2 if mode < 2 else 4
                    print(json.dumps({"frames": N, "level": tag, "pass": "fwd(apply)", "mode": mode,
                                      "us": round(us, 1), "GB": round(units * unit / 1e9, 3),
                                      "TBps": round(units * unit / us / 1e6, 2)}), flush=True)
                for use_dres in ((False, True) if mode < 2 and not C2 else (False,)):
                    dr = dres if use_dres else None
                    us = timeit(lambda: H._gn_bwd(mode, x, dy, sarg, stats, w, b, 32, 0.1 if mode == 2 else 0.0, 7,
                                                  x2=x2, dres=dr))
                    units = (5 if mode < 2 else 9) + (1 if use_dres else 0)
                    print(json.dumps({"frames": N, "level": tag, "pass": "bwd(reduce+apply)" + ("+dres" if dr is not None else ""),
                                      "mode": mode, "us": round(us, 1), "GB": round(units * unit / 1e9, 3),
                                      "TBps": round(units * unit / us / 1e6, 2)}), flush=True)
            del x, x2, dy, dres, ss
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
