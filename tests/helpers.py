"""Shared fixtures/helpers for the CPU test-suite."""
import torch

from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches

TINY = dict(H=16, W=16, ch=32, emb_ch=64)


def tiny_model(seed=0, randomize_zero_init=True, **kw):
    from distributed_3d_diffusion_pytorch_amd.models import XUNet
    torch.manual_seed(seed)
    cfg = dict(TINY)
    cfg.update(kw)
    m = XUNet(**cfg)
    if randomize_zero_init:
        with torch.no_grad():
            for p in m.parameters():
                if p.abs().sum() == 0:
                    p.normal_(0, 0.05)
    return m


def tiny_batch(B=2, size=16, seed=0):
    img, R, t, K = next(SyntheticBatches(B, size, "cpu", seed=seed))
    g = torch.Generator().manual_seed(seed)
    logsnr = torch.randn(B, 2, generator=g) * 5
    return {"x": img[:, 0], "z": img[:, 1], "logsnr": logsnr, "R": R, "t": t, "K": K}
