"""Reference-compatible import path (``from xunet import XUNet``).

Re-exports the MI355X-native X-UNet and its building blocks from
:mod:`distributed_3d_diffusion_pytorch_amd.models` (reference: `xunet.py`).
"""
from distributed_3d_diffusion_pytorch_amd.models import (XUNet, ResnetBlock, AttnBlock, AttnLayer, XUNetBlock,  # noqa
                                                         ConditioningProcessor, FiLM, GroupNorm)
from distributed_3d_diffusion_pytorch_amd.ops import posenc_ddpm, posenc_nerf  # noqa: F401
