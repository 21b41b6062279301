"""Diagnose shared-conditioning vs per-example forward on the HIP path:
compares conditioning embeddings, FiLM modulations and model outputs."""
import torch

from distributed_3d_diffusion_pytorch_amd import ops
from distributed_3d_diffusion_pytorch_amd.models import XUNet
from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches

DEV = "cuda"
BF = torch.bfloat16
torch.manual_seed(14)
m = XUNet(H=32, W=32, ch=128).to(DEV)
with torch.no_grad():
    for p in m.parameters():
        if p.abs().sum() == 0:
            p.normal_(0, 0.02)
m.compute_dtype = BF
m.eval()
img, R, t, K = next(SyntheticBatches(4, 32, DEV, seed=2))
b = 4
R1 = R[0].float()
T1 = t[0].float()
K1 = K[0].float()
Rb = R1[None].expand(2 * b, 2, 3, 3).contiguous()
Tb = T1[None].expand(2 * b, 2, 3).contiguous()
Kb = K1[None].expand(2 * b, 3, 3).contiguous()
lg = torch.tensor([[20.0, -1.0]] * (2 * b), device=DEV)
mask = torch.cat([torch.ones(b, dtype=torch.bool, device=DEV), torch.zeros(b, dtype=torch.bool, device=DEV)])
x = torch.randn(2 * b, 3, 32, 32, device=DEV)
z = torch.randn(2 * b, 3, 32, 32, device=DEV)
sc = {"R": R1[None].expand(2, 2, 3, 3), "t": T1[None].expand(2, 2, 3), "K": K1[None].expand(2, 3, 3),
      "logsnr": lg[:2], "cond_mask": torch.tensor([True, False], device=DEV),
      "example_class": torch.cat([torch.zeros(b, dtype=torch.int32, device=DEV),
                                  torch.ones(b, dtype=torch.int32, device=DEV)])}
cls_rows = torch.tensor([0, 1] * b + [2, 3] * b, device=DEV)
for be in ("hip", "torch"):
    ops.set_backend(be)
    with torch.no_grad():
        full = m.conditioningprocessor({"R": Rb, "t": Tb, "K": Kb, "logsnr": lg}, mask, BF)
        cls = m.conditioningprocessor(sc, sc["cond_mask"], BF)
        for i, (f, c) in enumerate(zip(full, cls)):
            d = (f.float() - c.float()[cls_rows]).abs().max().item()
            print(f"[{be}] semb level {i}: shape {tuple(c.shape)} max|full-class| = {d:.3e}")
        for i, blocks in enumerate(m._film_groups()):
            of = ops.film_batch(full[i], [bb.film.dense.weight for bb in blocks], [bb.film.dense.bias for bb in blocks])
            oc = ops.film_batch(cls[i], [bb.film.dense.weight for bb in blocks], [bb.film.dense.bias for bb in blocks])
            d = max((a.float() - c.float()[cls_rows]).abs().max().item() for a, c in zip(of, oc))
            print(f"[{be}] film level {i}: max|full-class| = {d:.3e}")
        y0 = m({"x": x, "z": z, "logsnr": lg, "R": Rb, "t": Tb, "K": Kb}, cond_mask=mask).float()
        y1 = m({"x": x, "z": z}, shared_cond=sc).float()
        print(f"[{be}] model max|full-shared| = {(y0 - y1).abs().max().item():.3e}  |y| = {y0.abs().max().item():.3e}")
