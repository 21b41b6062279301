"""``from lightning.SRNdataset import dataset, MultiEpochsDataLoader`` (reference
`lightning/SRNdataset.py`, identical to the root copy)."""
from . import _ROOT  # noqa: F401
from SRNdataset import dataset, MultiEpochsDataLoader  # noqa: F401
