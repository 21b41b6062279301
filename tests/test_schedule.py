import math

import torch

from distributed_3d_diffusion_pytorch_amd.diffusion import (logsnr_schedule_cosine, q_sample, cfg_posterior,
                                                            sampler_logsnrs, alpha_sigma, diffusion_loss)


def test_schedule_endpoints():
    t = torch.tensor([0.0, 0.5, 1.0])
    lam = logsnr_schedule_cosine(t)
    assert abs(lam[0].item() - 20.0) < 1e-3
    assert lam[1].item() == 0.0           # exactly 0 in fp32
    assert abs(lam[2].item() + 20.0) < 2e-2


def test_schedule_float64_formula():
    t = torch.rand(100, dtype=torch.float64)
    b = math.atan(math.exp(-10.0))
    a = math.atan(math.exp(10.0)) - b
    ref = -2.0 * torch.log(torch.tan(a * t + b))
    assert torch.allclose(logsnr_schedule_cosine(t), ref)


def test_alpha_sigma_unit_variance():
    lam = torch.linspace(-20, 20, 41)
    a, s = alpha_sigma(lam)
    assert torch.allclose(a * a + s * s, torch.ones_like(a), atol=1e-6)


def test_q_sample():
    z = torch.randn(3, 3, 4, 4)
    eps = torch.randn_like(z)
    lam = torch.tensor([-3.0, 0.0, 5.0])
    out = q_sample(z, lam, eps)
    a = torch.sigmoid(lam).sqrt().view(-1, 1, 1, 1)
    s = torch.sigmoid(-lam).sqrt().view(-1, 1, 1, 1)
    assert torch.allclose(out, a * z + s * eps)


def test_cfg_posterior_matches_reference_formula():
    torch.manual_seed(0)
    z = torch.randn(4, 3, 8, 8, dtype=torch.float64)
    ec, eu = torch.randn_like(z), torch.randn_like(z)
    w = torch.tensor([0.0, 1.0, 2.0, 3.0], dtype=torch.float64)
    lam, lamn = torch.tensor(1.3, dtype=torch.float64), torch.tensor(2.1, dtype=torch.float64)
    mean, var = cfg_posterior(z, ec, eu, w, lam, lamn)
    # train.py:140-166, written out
    c = -torch.expm1(lam - lamn)
    wv = w.view(-1, 1, 1, 1)
    e = (1 + wv) * ec - wv * eu
    x0 = ((z - torch.sigmoid(-lam).sqrt() * e) / torch.sigmoid(lam).sqrt()).clamp(-1, 1)
    m_ref = torch.sigmoid(lamn).sqrt() * (z * (1 - c) / torch.sigmoid(lam).sqrt() + c * x0)
    assert torch.allclose(mean, m_ref)
    assert torch.allclose(var, torch.sigmoid(-lamn) * c)


def test_sampler_logsnrs():
    lam, lamn = sampler_logsnrs(256)
    assert lam.shape == (256,) and lamn.shape == (256,)
    assert torch.allclose(lam[1:], lamn[:-1])
    assert lam[0] < -19.9 and lamn[-1] > 19.9
    # the reference's "logsnr_next == 0" fires at step 127 (D9)
    assert (lamn == 0).nonzero().flatten().tolist() == [127]


def test_losses():
    a, b = torch.randn(10), torch.randn(10)
    assert torch.allclose(diffusion_loss(a, b, "l2"), torch.nn.functional.mse_loss(b, a))
    assert torch.allclose(diffusion_loss(a, b, "l1"), torch.nn.functional.l1_loss(b, a))
    assert torch.allclose(diffusion_loss(a, b, "huber"), torch.nn.functional.smooth_l1_loss(b, a))
