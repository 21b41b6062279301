"""MI355X-native pose-conditioned novel-view diffusion (3DiM X-UNet) framework.

Capabilities of `halixness/distributed-3d-diffusion-pytorch`, re-designed for
AMD Instinct MI355X (gfx950): hand-written HIP kernels for the hot ops, RCCL
data parallelism over xGMI, and a native runtime around them.
"""
__version__ = "0.1.0"

from . import config  # noqa: F401
