"""``from lightning.diff3d import Diff3D`` (reference `lightning/diff3d.py:9-238`);
see :mod:`distributed_3d_diffusion_pytorch_amd.compat.diff3d`."""
from . import _ROOT  # noqa: F401
from distributed_3d_diffusion_pytorch_amd.compat import Diff3D  # noqa: F401
