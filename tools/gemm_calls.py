"""Dense-GEMM launches of one eager training step, by shape and epilogue:
wraps ``ops.hip_impl.gemm_nt`` and prints (M, N, K, flags) counts with the
innermost framework call sites, so the small latency-bound GEMMs of the
attention levels can be attributed:

    python tools/gemm_calls.py --global_batch 16
"""
import argparse
import collections
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--global_batch", type=int, default=16)
    a = ap.parse_args()
    from distributed_3d_diffusion_pytorch_amd.config import make_config
    from distributed_3d_diffusion_pytorch_amd.engine import Trainer
    from distributed_3d_diffusion_pytorch_amd.parallel import DistContext
    from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches
    from distributed_3d_diffusion_pytorch_amd.ops import hip_impl as H
    ctx = DistContext(device=torch.device("cuda", 0))
    cfg = make_config(None, {"model.H": 64, "model.W": 64, "data.imgsize": 64, "global_batch": a.global_batch,
                             "micro_batch": 0, "data.synthetic": True, "log_every": 0, "ckpt_every": 0,
                             "graph": False})
    tr = Trainer(cfg, ctx)
    data = SyntheticBatches(a.global_batch, 64, "cuda", seed=1)
    tr.train_step(*next(data))
    torch.cuda.synchronize()
    calls = collections.Counter()
    orig = H.gemm_nt

    def wrap(A, B, O, M, N, K, *args, **kw):
        fr = [f for f in traceback.extract_stack()[:-1] if "distributed_3d_diffusion_pytorch_amd" in f.filename]
        where = " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in fr[-2:][::-1])
        flags = ",".join(k for k, v in sorted(kw.items()) if v is not None and k in
                         ("bias", "res", "dsilu_of", "gnp"))
        calls[(M, N, K, flags, where)] += 1
        return orig(A, B, O, M, N, K, *args, **kw)

    H.gemm_nt = wrap
    tr.train_step(*next(data))
    torch.cuda.synchronize()
    H.gemm_nt = orig
    tot = sum(calls.values())
    print(f"gemm_nt calls in one eager step at bs{a.global_batch}: {tot}")
    for (M, N, K, fl, w), c in sorted(calls.items(), key=lambda kv: (-kv[1], kv[0][:3])):
        print(f"{c:5d}  M={M:5d} N={N:7d} K={K:5d}  [{fl}]  {w}")


if __name__ == "__main__":
    main()
