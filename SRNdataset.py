"""Reference-compatible import path (``from SRNdataset import dataset,
MultiEpochsDataLoader``); see :mod:`distributed_3d_diffusion_pytorch_amd.data`
(reference: `SRNdataset.py`)."""
from distributed_3d_diffusion_pytorch_amd.data import dataset, MultiEpochsDataLoader, SRNDataset  # noqa: F401


if __name__ == "__main__":
    # dataset smoke test (reference `SRNdataset.py:97-105`); without a data
    # root a small synthetic SRN tree is generated first
    import sys
    import tempfile
    from distributed_3d_diffusion_pytorch_amd.data import write_synthetic_srn
    if len(sys.argv) > 1:
        root = sys.argv[1]
    else:
        root = tempfile.mkdtemp()
        write_synthetic_srn(root, num_instances=4, num_views=3, size=64)
    d = dataset("train", root, "", imgsize=64)
    imgs, R, T, K = d[0]
    print(imgs.shape, R.shape, T.shape, K.shape)
