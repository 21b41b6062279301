"""Debug: GN-partials GEMM epilogue vs the plain epilogue, per tile config."""
import math
import torch
from distributed_3d_diffusion_pytorch_amd.ops import hip_impl as H

BF = torch.bfloat16
torch.manual_seed(17)
N, L, C = 4, 256, 256
x = torch.randn(N, L, C, device="cuda").to(BF)
w = torch.randn(C, C, device="cuda") / math.sqrt(C)
b = torch.randn(C, device="cuda") * 0.2
r = torch.randn(N, L, C, device="cuda").to(BF)
ref = ((x.float() @ w.to(BF).float().t() + b) + r.float()) / math.sqrt(2)
outs = {}
for cfg in (1, 2, 4, 8):
    H._lib.d3d_gemm_tune(cfg, 0, 0)
    outs[("gn", cfg)] = H.linear(x, w, b, r, 1 / math.sqrt(2), gn_groups=32)
    outs[("plain", cfg)] = H.linear(x, w, b, r, 1 / math.sqrt(2))
H._lib.d3d_gemm_tune(1, 0, 0)
torch.cuda.synchronize()
for k, v in outs.items():
    d = (v.float() - ref).abs()
    ne = (v != outs[("plain", 1)]).sum().item()
    print(k, "maxdiff_vs_fp32 %.4g" % d.max().item(), "ne_vs_plain1", ne,
          "first_bad", (v != outs[("plain", 1)]).nonzero()[:3].tolist())
