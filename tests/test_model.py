import json
import os

import pytest
import torch

from distributed_3d_diffusion_pytorch_amd.models import XUNet, reference_forward, count_params
from helpers import tiny_model, tiny_batch


def test_param_count_and_schema_64():
    m = XUNet(H=64, W=64, ch=128)
    assert count_params(m) == 136_670_627          # SURVEY 2.3 [measured on the reference]
    sd = m.state_dict()
    assert len(sd) == 647
    # spot-check the reference key schema
    expect = {
        "conditioningprocessor.pos_emb": (144, 64, 64),
        "conditioningprocessor.first_emb": (1, 1, 144, 1, 1),
        "conditioningprocessor.logsnr_emb_emb.2.weight": (1024, 1024),
        "conditioningprocessor.convs.3.weight": (1024, 144, 3, 3),
        "conv.weight": (128, 3, 3, 3),
        "xunetblocks.0.0.resnetblock.groupnorm0.gn.weight": (128,),
        "xunetblocks.1.0.resnetblock.dense.weight": (256, 128, 1, 1),
        "xunetblocks.2.0.attnblock_self.attn_layer.attn.in_proj_weight": (768, 256),
        "xunetblocks.2.0.attnblock_cross.attn_layer.attn.out_proj.weight": (256, 256),
        "xunetblocks.0.3.conv2.weight": (128, 128, 3, 3),
        "middle.attnblock_cross.linear.weight": (512, 512, 1, 1),
        "upsample.3.0.resnetblock.conv1.weight": (512, 1024, 3, 3),
        "upsample.1.4.film.dense.weight": (512, 1024),
        "upsample.0.3.resnetblock.dense.weight": (128, 256, 1, 1),
        "lastgn.gn.weight": (128,),
        "lastconv.weight": (3, 128, 3, 3),
    }
    for k, shp in expect.items():
        assert tuple(sd[k].shape) == shp, k
    assert list(sd)[0] == "conditioningprocessor.pos_emb"
    assert list(sd)[-1] == "lastconv.bias"


def test_param_count_128():
    assert count_params(XUNet(H=128, W=128, ch=128)) == 138_440_099


def test_analytic_flops_match_survey():
    """models/flops.py reproduces SURVEY Appendix C's measured forward FLOPs
    per example (235.9 G at 64x64, 969.3 G at 128x128) and splits off the
    conditioning part the shared-conditioning sampler runs per CFG class."""
    from distributed_3d_diffusion_pytorch_amd.models.flops import (forward_flops, image_flops,
                                                                   reference_example_flops)
    m = XUNet(H=64, W=64, ch=128)
    assert abs(reference_example_flops(m) / 1e9 - 235.9) < 0.05
    assert abs(reference_example_flops(XUNet(H=128, W=128, ch=128)) / 1e9 - 969.3) < 0.05
    f = image_flops(m)
    full, shared = forward_flops(m, 128), forward_flops(m, 128, cond_examples=2)
    assert abs(full - shared - 2 * 126 * f["cond"]) < 1e3 and shared < 0.7 * full


def test_zero_init():
    m = XUNet(H=16, W=16, ch=32, emb_ch=64)
    sd = m.state_dict()
    for k, v in sd.items():
        if k.endswith("conv2.weight") or k.endswith("linear.weight") or k == "lastconv.weight":
            assert v.abs().sum() == 0, k
    assert m(tiny_batch(), cond_mask=torch.tensor([True, True])).abs().max() == sd["lastconv.bias"].abs().max()


@pytest.mark.parametrize("mask", [[True, False], [True, True], [False, False]])
def test_forward_matches_reference_oracle(mask):
    m = tiny_model().eval()
    b = tiny_batch()
    cm = torch.tensor(mask)
    out = m(b, cond_mask=cm)
    ref = reference_forward(m.state_dict(), b, cm, emb_ch=64)
    assert out.shape == (2, 3, 16, 16)
    assert (out - ref).abs().max().item() < 1e-4 * max(1.0, ref.abs().max().item())


def test_gradients_match_reference_oracle():
    m = tiny_model().eval()
    b = tiny_batch()
    cm = torch.tensor([True, False])
    out = m(b, cond_mask=cm)
    out.square().mean().backward()
    grads = {n: p.grad.clone() for n, p in m.named_parameters()}
    sd = {n: p.detach().clone().requires_grad_(True) for n, p in m.named_parameters()}
    from distributed_3d_diffusion_pytorch_amd.models import reference_forward_grad
    ref = reference_forward_grad(sd, b, cm, emb_ch=64)
    ref.square().mean().backward()
    for n in grads:
        assert torch.allclose(grads[n], sd[n].grad, atol=1e-5, rtol=1e-3), n


def test_module_prefix_load_roundtrip(tmp_path):
    from distributed_3d_diffusion_pytorch_amd.utils import load_model_weights, add_prefix
    m1, m2 = tiny_model(seed=1), tiny_model(seed=2)
    load_model_weights(m2, add_prefix(m1.state_dict()))
    for (k, a), (_, b) in zip(m1.state_dict().items(), m2.state_dict().items()):
        assert torch.equal(a, b), k


def test_resolution_assert():
    with pytest.raises(AssertionError):
        XUNet(H=12, W=12, ch=32)


def test_rescale_intrinsics_changes_rays():
    m = tiny_model(rescale_intrinsics=True).eval()
    b = tiny_batch()
    cm = torch.tensor([True, True])
    out = m(b, cond_mask=cm)
    ref = reference_forward(m.state_dict(), b, cm, emb_ch=64, rescale_from=128)
    ref0 = reference_forward(m.state_dict(), b, cm, emb_ch=64, rescale_from=0)
    assert (out - ref).abs().max() < 1e-4 * max(1.0, ref.abs().max().item())
    assert (out - ref0).abs().max() > 1e-4
