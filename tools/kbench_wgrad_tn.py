"""Microbenchmark: the transposed-read split-K weight-gradient GEMM
(wgrad_gemm.hip, slabs + bias partials, then the slab reduction) against the
hipBLASLt split product (bmm into fp32 slabs) at the FiLM weight-gradient
shapes of the bs128 / bs16 steps.  One JSON line per shape."""
import argparse
import json
import time

import torch

from distributed_3d_diffusion_pytorch_amd.ops import hip_impl as H

SHAPES = [  # rows (pixels of a level, both views), S (sum of 2C), K (embedding)
    (1048576, 2048, 1024), (262144, 4608, 1024), (65536, 4608, 1024), (16384, 9216, 1024),
    (131072, 2048, 1024), (32768, 4608, 1024), (8192, 4608, 1024),
]


ITERS = [10]


def bench(fn, iters=0):
    iters = iters or ITERS[0]
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", type=int, default=0, help="only the shape with this many rows")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--vars", default="0", help="comma list of d3d_wgrad_tn_tune variants")
    a = ap.parse_args()
    ITERS[0] = a.iters
    for rows, S, K in SHAPES:
        if a.only and rows != a.only:
            continue
        dy = (torch.randn(rows, S, device="cuda") * 0.1).to(torch.bfloat16)
        x = torch.randn(rows, K, device="cuda").to(torch.bfloat16)
        fl = 2.0 * rows * S * K
        ref = dy.float().t() @ x.float()
        ws, bws, used = H.wgrad_tn(dy, x)
        err = ((ws.sum(0) - ref).abs().max() / ref.abs().max()).item()
        rec = {"rows": rows, "S": S, "K": K, "splits": used, "err": round(err, 7)}
        for v in [int(x) for x in a.vars.split(",")]:
            H._lib.d3d_wgrad_tn_tune(v)
            t_tn = bench(lambda: H.wgrad_tn(dy, x))
            rec[f"v{v}_us"] = round(t_tn, 1)
            rec[f"v{v}_tflops"] = round(fl / t_tn / 1e6, 1)
        H._lib.d3d_wgrad_tn_tune(0)
        t_bl = bench(lambda: H._film_wgrad_product(dy, x))
        rec.update({"blas_us": round(t_bl, 1), "blas_tflops": round(fl / t_bl / 1e6, 1)})
        print(json.dumps(rec), flush=True)
        del dy, x, ref, ws, bws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
