import os

import torch

from distributed_3d_diffusion_pytorch_amd.parallel.flat import FlatParams
from distributed_3d_diffusion_pytorch_amd.engine.optim import FusedAdam, warmup_lr, ema_decay_for
from distributed_3d_diffusion_pytorch_amd.utils import save_checkpoint, load_checkpoint, find_resume
from helpers import tiny_model


def _params(seed):
    torch.manual_seed(seed)
    return [torch.nn.Parameter(torch.randn(s)) for s in [(7, 5), (33,), (2, 3, 3, 3)]]


def test_flat_params_views():
    ps = _params(0)
    vals = [p.detach().clone() for p in ps]
    flat = FlatParams(ps)
    for p, v in zip(ps, vals):
        assert torch.equal(p, v)
        assert p.data.data_ptr() >= flat.data.data_ptr()
        assert p.grad is not None and p.grad.data_ptr() >= flat.grad.data_ptr()
    loss = sum((p * p).sum() for p in ps)
    loss.backward()
    for p in ps:
        assert torch.allclose(p.grad, 2 * p.detach())
    assert flat.grad.abs().sum() > 0


def test_fused_adam_matches_torch_and_state_dict():
    ps, ref = _params(0), _params(0)
    flat = FlatParams(ps)
    opt = FusedAdam(flat, lr=1e-2, betas=(0.9, 0.99))
    topt = torch.optim.Adam(ref, lr=1e-2, betas=(0.9, 0.99))
    for _ in range(4):
        gs = [torch.randn_like(p) for p in ps]
        for p, g in zip(ps, gs):
            p.grad.copy_(g * 2)
        for p, g in zip(ref, gs):
            p.grad = g.clone()
        opt.step(grad_scale=0.5)          # DP averaging folded in
        topt.step()
    for p, r in zip(ps, ref):
        assert torch.allclose(p, r, atol=1e-6)
    # torch Adam state_dict interoperability, both directions
    sd = opt.state_dict()
    tsd = topt.state_dict()
    assert set(sd["state"]) == set(tsd["state"])
    for i in sd["state"]:
        assert torch.allclose(sd["state"][i]["exp_avg"], tsd["state"][i]["exp_avg"], atol=1e-7)
    ps2 = _params(5)
    opt2 = FusedAdam(FlatParams(ps2), lr=1e-2)
    opt2.load_state_dict(tsd)
    assert opt2.step_count == 4
    assert torch.allclose(opt2.exp_avg_sq, opt.exp_avg_sq)
    t3 = torch.optim.Adam(_params(1), lr=1e-2)
    t3.load_state_dict(sd)


def test_warmup_and_ema():
    assert warmup_lr(0, 10, 1e-4) == 0.0
    assert warmup_lr(5, 10, 1e-4) == 0.5e-4
    assert warmup_lr(10, 10, 1e-4) == 1e-4
    assert warmup_lr(3, 0, 1e-4) == 1e-4
    d = ema_decay_for(128, 500_000)
    assert 0.999 < d < 1.0
    assert abs(d ** (500_000 / 128) - 0.5) < 1e-6


def test_checkpoint_roundtrip(tmp_path):
    m = tiny_model()
    flat = FlatParams(list(m.parameters()))
    opt = FusedAdam(flat, lr=1e-3)
    for p in m.parameters():
        p.grad.normal_()
    opt.step()
    path = str(tmp_path / "latest.pt")
    save_checkpoint(path, m, opt, step=7, epoch=1)
    ck = load_checkpoint(path)
    assert set(ck) >= {"model", "optim", "step", "epoch"} and ck["step"] == 7
    assert all(not k.startswith("module.") for k in ck["model"])
    # file size ~ params + 2 moments (views were cloned, not whole storages)
    n = sum(p.numel() for p in m.parameters())
    assert os.path.getsize(path) < 4 * n * 4 * 1.5
    assert find_resume(str(tmp_path)) == path
