"""Reference-compatible import path (``from SRNdataset import dataset,
MultiEpochsDataLoader``); see :mod:`distributed_3d_diffusion_pytorch_amd.data`
(reference: `SRNdataset.py`)."""
from distributed_3d_diffusion_pytorch_amd.data import dataset, MultiEpochsDataLoader, SRNDataset  # noqa: F401
