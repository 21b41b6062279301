"""Reference-layout entry points of the Lightning variant (`lightning/` in the
reference): ``lightning/train.py`` (T3), ``lightning/sampling.py``,
``lightning.xunet`` / ``lightning.diff3d`` / ``lightning.SRNdataset`` imports.
PyTorch Lightning itself is not part of this stack: everything here runs on the
framework's own trainer, sampler and model."""
import os as _os
import sys as _sys

_ROOT = _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))
if _ROOT not in _sys.path:
    _sys.path.insert(0, _ROOT)
