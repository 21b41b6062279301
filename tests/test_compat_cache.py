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
    # reference signature: sample(model, img, R, T, K, w, timesteps) -> per-step list
    imgs = m.sample(m.xunet_denoiser, batch[0], batch[1].float(), batch[2].float(), batch[3][0].float(),
                    torch.tensor([0.0, 2.0]), timesteps=2)
    assert len(imgs) == 2 and imgs[-1].shape == (2, 3, 16, 16) and np.isfinite(imgs[-1]).all()
    # per-example poses are honoured: swapping example 1's target pose changes only example 1
    R2 = batch[1].float().clone()
    R2[1, 1] = torch.linalg.qr(torch.randn(3, 3))[0]
    torch.manual_seed(1)
    a = m.sample(batch[0][:, 0], batch[1].float(), batch[2].float(), batch[3][0].float(), 2.0, timesteps=2,
                 return_all=False)
    torch.manual_seed(1)
    c = m.sample(None, batch[0], R2, batch[2].float(), batch[3][0].float(), 2.0, timesteps=2, return_all=False)
    assert torch.allclose(a[0], c[0]) and not torch.allclose(a[1], c[1])
    # the legacy call without the model: the positional step count shifts with the rest
    imgs3 = m.sample(batch[0][:, 0], batch[1].float(), batch[2].float(), batch[3][0].float(), 2.0, 3)
    assert len(imgs3) == 3
    with pytest.raises(TypeError):
        m.sample(batch[0][:, 0], batch[1].float(), batch[2].float(), batch[3][0].float(), 2.0, 2.5)
    # integer-like step counts (numpy / 0-d tensors) are accepted
    assert len(m.sample(batch[0][:, 0], batch[1].float(), batch[2].float(), batch[3][0].float(), 2.0,
                        np.int64(2))) == 2
    assert len(m.sample(batch[0][:, 0], batch[1].float(), batch[2].float(), batch[3][0].float(), 2.0,
                        torch.tensor(1))) == 1
    # a keyword w in the model-less form gets its own message (not "timesteps must be ...")
    with pytest.raises(TypeError, match="positionally"):
        m.sample(batch[0][:, 0], batch[1].float(), batch[2].float(), batch[3][0].float(), w=2.0)
