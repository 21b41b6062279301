"""Reference-compatible import path (``from diff3d import Diff3D``); see
:mod:`distributed_3d_diffusion_pytorch_amd.compat.diff3d` (reference:
`lightning/diff3d.py`)."""
from distributed_3d_diffusion_pytorch_amd.compat import Diff3D  # noqa: F401
