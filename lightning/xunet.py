"""``from lightning.xunet import XUNet`` (reference `lightning/xunet.py`, the
LightningModule-submodule copy of the X-UNet; `lightning/sampling.py:1` imports
it).  Same model, same parameter names as the root ``xunet``."""
from . import _ROOT  # noqa: F401  (puts the repo root on sys.path)
from xunet import *  # noqa: F401,F403
from xunet import XUNet  # noqa: F401
