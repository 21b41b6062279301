"""Reference-compatible import path (``from xunet import XUNet``).

Re-exports the MI355X-native X-UNet and its building blocks from
:mod:`distributed_3d_diffusion_pytorch_amd.models` (reference: `xunet.py`).
"""
from distributed_3d_diffusion_pytorch_amd.models import (XUNet, ResnetBlock, AttnBlock, AttnLayer, XUNetBlock,  # noqa
                                                         ConditioningProcessor, FiLM, GroupNorm)
from distributed_3d_diffusion_pytorch_amd.ops import posenc_ddpm, posenc_nerf  # noqa: F401


if __name__ == "__main__":
    # model smoke test (reference `xunet.py:538-560`): b=8 zero batch at 56x56
    import torch
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    model = XUNet(H=56, W=56, ch=128).to(dev)
    if dev == "cuda":
        model.compute_dtype = torch.bfloat16
    b = 8
    batch = {"x": torch.zeros(b, 3, 56, 56, device=dev), "z": torch.zeros(b, 3, 56, 56, device=dev),
             "logsnr": torch.zeros(b, 2, device=dev), "R": torch.eye(3, device=dev).expand(b, 2, 3, 3),
             "t": torch.zeros(b, 2, 3, device=dev),
             "K": torch.tensor([[70.0, 0, 28], [0, 70.0, 28], [0, 0, 1]], device=dev).expand(b, 3, 3)}
    with torch.no_grad():
        out = model(batch, cond_mask=torch.ones(b, dtype=torch.bool, device=dev))
    print(out.shape)
