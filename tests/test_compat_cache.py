import os

import numpy as np
import pytest
import torch

from distributed_3d_diffusion_pytorch_amd.data import (write_synthetic_srn, SRNDataset, CachedSRNDataset,
                                                       build_cache)


@pytest.fixture(scope="module")
def srn(tmp_path_factory):
    root = str(tmp_path_factory.mktemp("srn_c"))
    write_synthetic_srn(root, num_instances=6, num_views=4, size=32, seed=2)
    return root


def test_cache_matches_png_dataset(srn, tmp_path):
    cache = build_cache(srn, str(tmp_path / "cache"), imgsize=16)
    a = SRNDataset("train", srn, "", imgsize=16)
    b = CachedSRNDataset("train", cache)
    assert a.ids == b.ids
    for i in range(len(a)):
        ia, Ra, Ta, Ka = a[i]
        ib, Rb, Tb, Kb = b[i]
        assert np.allclose(Ra, Rb) and np.allclose(Ta, Tb) and np.allclose(Ka, Kb)
        assert np.abs(ia - ib).max() < 1e-6


def test_reference_import_paths():
    import xunet
    import SRNdataset
    import diff3d
    assert xunet.XUNet is not None and SRNdataset.dataset is not None and diff3d.Diff3D is not None


def test_diff3d_api(srn):
    from diff3d import Diff3D
    from distributed_3d_diffusion_pytorch_amd.data import collate
    torch.manual_seed(0)
    m = Diff3D(image_size=16, batch_size=2, n_samples=8)
    m.xunet_denoiser = __import__("helpers").tiny_model()
    ds = SRNDataset("train", srn, "", imgsize=16)
    batch = collate([ds[0], ds[1]])
    assert abs(m.logsnr_schedule_cosine(torch.tensor(0.0)).item() - 20.0) < 1e-3
    l0 = m.fit_step(batch)
    assert np.isfinite(l0) and m.step == 1
    # warmup: lr grows linearly over n_samples / batch_size = 4 steps
    assert abs(m.optimizers().param_groups[0]["lr"] - 0.0) < 1e-12
    m.training_step(batch)
    assert abs(m.optimizers().param_groups[0]["lr"] - 0.25e-4) < 1e-12
    x = batch[0][:, 0]
    out = m.sample(x, batch[1].float(), batch[2].float(), batch[3][0].float(), torch.tensor([0.0, 2.0]),
                   timesteps=2)
    assert out.shape == (2, 3, 16, 16) and torch.isfinite(out).all()
