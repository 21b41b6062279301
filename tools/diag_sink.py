"""Diagnose sink-vs-autograd gradient differences per parameter (1 GPU)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from distributed_3d_diffusion_pytorch_amd.parallel import FlatParams
from distributed_3d_diffusion_pytorch_amd.ops.gradsink import SINK
from distributed_3d_diffusion_pytorch_amd.models import XUNet
from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches
torch.manual_seed(0)
m = XUNet(H=32, W=32, ch=128).cuda().eval()
with torch.no_grad():
    for p in m.parameters():
        if p.abs().sum() == 0:
            p.normal_(0, 0.02)
m.compute_dtype = torch.bfloat16
flat = FlatParams(list(m.parameters()))
img, R, t, K = next(SyntheticBatches(2, 32, "cuda", seed=0))
batch = {"x": img[:, 0], "z": img[:, 1], "logsnr": torch.tensor([[20.0, 1.0], [20.0, -2.0]], device="cuda"),
         "R": R, "t": t, "K": K}
mask = torch.tensor([True, False], device="cuda")
m(batch, cond_mask=mask).float().square().mean().backward()
ref = flat.grad.clone()
flat.zero_grad()
views = [flat.view(flat.grad, i) for i in range(len(flat.params))]
SINK.attach(flat.params, views, None)
SINK.reset()
m(batch, cond_mask=mask).float().square().mean().backward()
torch.cuda.synchronize()
names = [n for n, _ in m.named_parameters()]
bad = 0
for i, n in enumerate(names):
    a = flat.view(flat.grad, i).float(); b = flat.view(ref, i).float()
    d = ((a - b).norm() / b.norm().clamp_min(1e-12)).item()
    if d > 2e-2:
        bad += 1
        if bad < 40:
            print(f"{n:70s} rel={d:.3g} |ref|={b.norm().item():.3g} |got|={a.norm().item():.3g} uses_left={SINK.uses.get(id(flat.params[i]))}")
print("bad", bad, "of", len(names))
