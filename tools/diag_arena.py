"""Stray-write screen for the 1x1 / 3x3 weight-gradient launches: every
operand, the split-K workspace and the dW / db targets are carved out of ONE
sentinel-filled arena with sentinel gaps between them; after the launch every
element outside the two targets and the workspace must still hold the
sentinel.  Shapes: the X-UNet's per-pixel layers at batch 16 / 128."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from distributed_3d_diffusion_pytorch_amd.ops import hip_impl as H

dev = torch.device("cuda", 0)
SENT = -7777.0
GAP = 1 << 16          # fp32 elements between regions


def run(OC, IC, N, Hh, taps):
    H._ensure_impl()
    s, pps = ctypes.c_int(), ctypes.c_int()
    W = Hh
    H._lib.d3d_conv_wgrad_plan3(N, Hh, W, Hh, W, OC, IC, taps, 1, ctypes.byref(s), ctypes.byref(pps))
    P = N * Hh * W
    sizes = {"g": (P * OC + 1) // 2, "x": (P * IC + 1) // 2, "ws": s.value * OC * taps * IC + 2 * s.value * OC,
             "dW": OC * IC * taps, "db": OC}
    offs, o = {}, GAP
    for k, n in sizes.items():
        offs[k] = o
        o += (n + 63) // 64 * 64 + GAP
    arena = torch.full((o,), SENT, dtype=torch.float32, device=dev)
    g = arena[offs["g"]: offs["g"] + sizes["g"]].view(torch.bfloat16)[: P * OC]
    x = arena[offs["x"]: offs["x"] + sizes["x"]].view(torch.bfloat16)[: P * IC]
    g.copy_(torch.randn(P * OC, device=dev).to(torch.bfloat16))
    x.copy_(torch.randn(P * IC, device=dev).to(torch.bfloat16))
    dW = arena[offs["dW"]: offs["dW"] + sizes["dW"]]
    db = arena[offs["db"]: offs["db"] + sizes["db"]]
    dW.zero_()
    db.zero_()
    ws = arena[offs["ws"]: offs["ws"] + sizes["ws"]]
    torch.cuda.synchronize()
    rc = H._lib.d3d_conv_wgrad3(g.data_ptr(), x.data_ptr(), ws.data_ptr(), dW.data_ptr(), db.data_ptr(), N, Hh, W,
                                IC, Hh, W, OC, 1, s.value, pps.value, 1, taps, ctypes.c_float(1.0), H._st())
    torch.cuda.synchronize()
    mask = torch.ones(o, dtype=torch.bool, device=dev)
    for k in ("g", "x", "ws", "dW", "db"):
        mask[offs[k]: offs[k] + sizes[k]] = False
    stray = (arena[mask] != SENT).sum().item()
    where = []
    if stray:
        idx = (mask & (arena != SENT)).nonzero().flatten()
        for i in idx[:3].tolist():
            reg = min(((i - offs[k], k) for k in offs if i >= offs[k]), default=(i, "start"))
            where.append(f"{reg[1]}+{reg[0]}")
    return rc, s.value, pps.value, stray, where


def main():
    shapes = []
    for N in (32, 256):
        for (Hh, C) in ((64, 128), (32, 256), (16, 256), (8, 512)):
            P = N * Hh * Hh
            for (OC, IC) in ((3 * C, C), (C, C), (C // 2 if C > 128 else C, C)):
                shapes.append((OC, IC, P, 1, 1))      # per-pixel layers as 1x1 "images"
            shapes.append((C, C, N, Hh, 9))
    bad = 0
    for OC, IC, N, Hh, taps in shapes:
        try:
            rc, sp, pps, stray, where = run(OC, IC, N, Hh, taps)
        except torch.cuda.OutOfMemoryError:
            continue
        bad += stray > 0
        print(f"OC{OC} IC{IC} N{N} H{Hh} taps{taps}: rc {rc} splits {sp} pps {pps}: stray writes {stray} {where}",
              flush=True)
    print("RESULT", "FAIL" if bad else "PASS")


if __name__ == "__main__":
    main()
