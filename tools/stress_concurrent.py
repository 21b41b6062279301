"""Concurrency race screen for single kernels: each op is run once alone
(reference output), then repeatedly while a second HIP stream keeps other
kernels resident on the CUs; every repetition must match the reference bit
for bit.  A kernel whose result changes under co-residency has a
timing-dependent (usually LDS / barrier) race that the sequential tests
cannot see.

usage: python tools/stress_concurrent.py [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from distributed_3d_diffusion_pytorch_amd.ops import hip_impl as H

BF = torch.bfloat16
dev = torch.device("cuda", 0)


def cases():
    torch.manual_seed(0)
    out = []
    # linear / GEMM (gemm.hip) at the attention / NIN / FiLM shapes of bs16
    for (M, N, K, bias, res) in ((768, 8192, 256, True, False), (256, 8192, 256, True, True),
                                 (256, 8192, 768, False, False), (1536, 2048, 512, True, False),
                                 (512, 2048, 1536, False, False), (128, 131072, 256, True, False),
                                 (2048, 32768, 1024, True, False), (1024, 32768, 2048, False, False)):
        a = (torch.randn(M, K, device=dev) * 0.1).to(BF)
        b = torch.randn(N, K, device=dev).to(BF)
        bb = torch.randn(M, device=dev) if bias else None
        r = torch.randn(N, M, device=dev).to(BF) if res else None

        def f(a=a, b=b, bb=bb, r=r, M=M, N=N, K=K):
            o = torch.empty(N, M, dtype=BF, device=dev)
            H.gemm_nt(a, b, o, M, N, K, K, K, M, bias=bb, res=r)
            return o
        out.append((f"gemm M{M} N{N} K{K} bias{int(bias)} res{int(res)}", f))
    # 3x3 conv forward / input gradient (conv.hip) at the bs16 level shapes
    for (N, Hh, C) in ((32, 64, 128), (32, 32, 256), (32, 16, 256), (32, 8, 512)):
        x = torch.randn(N, Hh, Hh, C, device=dev).to(BF)
        w = torch.randn(C, C, 3, 3, device=dev) * 0.05
        xr = torch.randn(N, Hh, Hh, C, device=dev).to(BF)

        def f(x=x, w=w, xr=xr):
            return H.conv3x3(x, w, None, residual=xr, out_scale=0.7071)
        out.append((f"conv3x3 {N}x{Hh}x{Hh}x{C}", f))
        g = torch.randn(N, Hh, Hh, C, device=dev).to(BF)

        def fw(x=x, g=g, C=C, N=N, Hh=Hh):
            dW, db = H._wgrad(g, x, C, C, N, Hh, Hh, Hh, Hh, 1, 9, want_bias=True)
            return torch.cat([dW.flatten(), db])
        out.append((f"conv wgrad {N}x{Hh}x{Hh}x{C}", fw))

        def fl(x=x, g=g, C=C, N=N, Hh=Hh):
            r = N * Hh * Hh
            dW, db = H._wgrad(g.reshape(r, 1, 1, C), x.reshape(r, 1, 1, C), C, C, r, 1, 1, 1, 1, 1, 1,
                              want_bias=True)
            return torch.cat([dW.flatten(), db])
        out.append((f"1x1 wgrad {N * Hh * Hh}x{C}", fl))
    # attention fwd (attention.hip) at the 16x16 / 8x8 levels
    for (N, L, C) in ((32, 256, 256), (32, 64, 512)):
        qkv = torch.randn(N, L, 3 * C, device=dev).to(BF)

        def fa(qkv=qkv):
            return H.attention(qkv, 4, False)
        out.append((f"attention {N}x{L}x{C}", fa))
        do = torch.randn(N, L, C, device=dev).to(BF)

        def fab(qkv=qkv, do=do):
            q = qkv.clone().requires_grad_(True)
            o = H.attention(q, 4, True)
            (g,) = torch.autograd.grad(o, q, do)
            return g
        out.append((f"attention bwd {N}x{L}x{C}", fab))
    # GroupNorm(+SiLU / +FiLM) backward at the bs16 level shapes
    for (N, Hh, C) in ((32, 64, 128), (32, 16, 256), (32, 8, 512)):
        x = torch.randn(N, Hh, Hh, C, device=dev).to(BF)
        dy = torch.randn(N, Hh, Hh, C, device=dev).to(BF)
        w = torch.rand(C, device=dev) + 0.5
        b = torch.randn(C, device=dev) * 0.1
        ss = (torch.randn(N, Hh, Hh, 2 * C, device=dev) * 0.3).to(BF)
        for mode in (1, 2):
            sarg = ss if mode == 2 else None
            _, st = H._gn_fwd(mode, x, w, b, 32, 1e-5, sarg, 0, 0.1 if mode == 2 else 0.0, 7)

            def fg(x=x, dy=dy, sarg=sarg, st=st, w=w, b=b, mode=mode):
                dx, dss, dg, db = H._gn_bwd(mode, x, dy, sarg, st, w, b, 32, 0.1 if mode == 2 else 0.0, 7)
                parts = [dx.float().flatten(), dg, db] + ([dss.float().flatten()] if dss is not None else [])
                return torch.cat(parts)
            out.append((f"gn bwd m{mode} {N}x{Hh}x{Hh}x{C}", fg))
    return out


def noise_setup(kind):
    """Aggressor kernels kept running on the second stream."""
    if kind == "mm+wgrad3x3":
        big = torch.randn(8192, 8192, device=dev).to(BF)
        x = torch.randn(32, 64, 64, 128, device=dev).to(BF)
        g = torch.randn(32, 64, 64, 128, device=dev).to(BF)

        def noise():
            for _ in range(3):
                torch.mm(big, big)
                H._wgrad(g, x, 128, 128, 32, 64, 64, 64, 64, 1, 9, want_bias=True)
        return noise
    # the per-pixel weight gradients of the attention projections (1x1 split-K
    # kernel + slab reduce), bs16 level shapes, many back to back
    shp = [(768, 256, 8192), (256, 256, 8192), (768, 256, 32768), (1536, 512, 2048), (512, 512, 2048)]
    ops = []
    for OC, IC, P in shp:
        g = torch.randn(P, 1, 1, OC, device=dev).to(BF)
        x = torch.randn(P, 1, 1, IC, device=dev).to(BF)
        ops.append((g, x, OC, IC, P))

    def noise():
        for _ in range(6):
            for g, x, OC, IC, P in ops:
                H._wgrad(g, x, OC, IC, P, 1, 1, 1, 1, 1, 1, want_bias=True)
    return noise


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    side = torch.cuda.Stream(device=dev)
    bad = 0
    for nk in ("wgrad1x1", "mm+wgrad3x3"):
      noise = noise_setup(nk)
      print(f"-- aggressor: {nk}", flush=True)
      for name, f in cases():
          ref = f().clone()
          torch.cuda.synchronize()
          mism = 0
          maxd = 0.0
          for i in range(reps):
              side.wait_stream(torch.cuda.current_stream())
              with torch.cuda.stream(side):
                  noise()
              # the op starts while the noise kernels occupy the CUs; vary the
              # overlap by a few small kernels of delay
              for _ in range(i % 4):
                  torch.empty(1, device=dev).zero_()
              o = f()
              torch.cuda.current_stream().wait_stream(side)
              torch.cuda.synchronize()
              if not torch.equal(o, ref):
                  mism += 1
                  maxd = max(maxd, (o.float() - ref.float()).abs().max().item())
          # and alone again
          o = f()
          torch.cuda.synchronize()
          alone = torch.equal(o, ref)
          bad += mism > 0 or not alone
          print(f"{name:38s} concurrent mismatches {mism}/{reps} (max |d| {maxd:.3e}); alone again equal {alone}",
                flush=True)
    print("RESULT", "FAIL" if bad else "PASS", flush=True)


if __name__ == "__main__":
    main()
