"""End-to-end CPU plumbing (BASELINE config 1: chairs 32x32 bs2 fp32, shrunk
to a tiny width so it runs in seconds): train -> checkpoint -> resume ->
sample, through the user-facing CLIs."""
import os

import numpy as np
import pytest
import torch

from distributed_3d_diffusion_pytorch_amd.config import make_config
from distributed_3d_diffusion_pytorch_amd.data import write_synthetic_srn
from distributed_3d_diffusion_pytorch_amd.engine import Trainer, DiffusionSampler, RecordEntry, shard_range
from distributed_3d_diffusion_pytorch_amd.parallel import DistContext
from helpers import tiny_model

TINY_OV = {"model.ch": 32, "model.emb_ch": 64, "model.H": 16, "model.W": 16, "data.imgsize": 16,
           "global_batch": 2, "dtype": "fp32", "backend": "torch", "log_every": 1, "ckpt_every": 2,
           "data.num_workers": 0}


@pytest.fixture(scope="module")
def srn_root(tmp_path_factory):
    root = str(tmp_path_factory.mktemp("srn_train"))
    write_synthetic_srn(root, num_instances=5, num_views=4, size=32, seed=1)
    return root


def test_overfit_loss_decreases():
    cfg = make_config("chairs32_cpu", dict(TINY_OV, **{"data.synthetic": True, "optim.lr": 2e-3}))
    tr = Trainer(cfg, DistContext())
    from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches
    batch = next(SyntheticBatches(2, 16, "cpu", seed=0))
    # fixed diffusion noise so the objective is stationary
    tr.step_seed = lambda step_word=None: 1234
    losses = []
    for _ in range(25):
        losses.append(float(tr.train_step(*batch)))
    assert np.isfinite(losses).all()
    assert np.mean(losses[-5:]) < 0.7 * np.mean(losses[:5]), losses


def test_micro_batching_matches_full_batch():
    """The input draw is counter-based in (step seed, example index), so two
    micro-batches of 2 see exactly the noise of the full batch of 4: the
    accumulated gradient (and the loss) must match the full-batch step."""
    from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches
    batch = next(SyntheticBatches(4, 16, "cpu", seed=0))
    grads, losses, params = [], [], []
    for mb in (0, 2):
        cfg = make_config(None, dict(TINY_OV, **{"global_batch": 4, "micro_batch": mb, "model.dropout": 0.0,
                                                 "optim.lr": 1e-3}))
        tr = Trainer(cfg, DistContext())
        grads_step = {}
        tr.optim.on_step.insert(0, lambda tr=tr, d=grads_step: d.setdefault("g", tr.flat.grad.clone()))
        losses.append(float(tr.train_step(*batch)))
        grads.append(grads_step["g"])
        params.append(tr.flat.data.clone())
    assert abs(losses[0] - losses[1]) < 1e-6 * max(1.0, abs(losses[0])), losses
    assert grads[0].abs().max() > 0
    torch.testing.assert_close(grads[1], grads[0], rtol=1e-4, atol=1e-7)
    torch.testing.assert_close(params[1], params[0], rtol=1e-5, atol=1e-7)


def test_train_cli_checkpoint_resume_and_sampling_cli(srn_root, tmp_path):
    import train as train_cli
    import sampling as sampling_cli
    out = str(tmp_path / "run")
    args = ["--train_data", srn_root, "--out_dir", out, "--steps", "4", "num_epochs=100"] + \
        [f"{k}={v}" for k, v in TINY_OV.items()]
    train_cli.main(args)
    assert os.path.exists(os.path.join(out, "latest.pt"))
    assert os.path.exists(os.path.join(out, "after_warmup.pt"))
    ck = torch.load(os.path.join(out, "latest.pt"), weights_only=True)
    assert ck["step"] == 4 and {"model", "optim", "step", "epoch"} <= set(ck)
    # resume continues at the saved step
    train_cli.main(["--train_data", srn_root, "--transfer", out, "--steps", "6", "num_epochs=100"] +
                   [f"{k}={v}" for k, v in TINY_OV.items()])
    ck2 = torch.load(os.path.join(out, "latest.pt"), weights_only=True)
    assert ck2["step"] == 6
    inst = sorted(d for d in os.listdir(srn_root) if os.path.isdir(os.path.join(srn_root, d)))[0]
    so = str(tmp_path / "samples")
    sampling_cli.main(["--model", os.path.join(out, "latest.pt"), "--target", os.path.join(srn_root, inst),
                       "--out", so, "--imgsize", "16", "--timesteps", "3", "--w", "0,2", "--max_views", "2",
                       "--backend", "torch"])
    for k in (0, 1, 2):
        assert os.path.exists(os.path.join(so, str(k), "gt.png"))
    for k in (1, 2):
        assert os.path.exists(os.path.join(so, str(k), "0.png")) and os.path.exists(os.path.join(so, str(k), "1.png"))


def test_sampler_cfg_batched_equals_separate():
    m = tiny_model().eval()
    smp = DiffusionSampler(m, timesteps=4, seed=0)
    B = 2
    from helpers import tiny_batch
    b = tiny_batch(B)
    R, T, K = b["R"], b["t"], b["K"]
    ec, eu = smp.denoise_eps(b["x"], b["z"], R, T, K, 1.0, k=3)
    from distributed_3d_diffusion_pytorch_amd.ops import torch_impl as TI
    x_unc = smp._noise(TI.K_XU, 3, tuple(b["x"].shape), b["x"].device)
    lam = torch.full((B,), 1.0)
    base = {"z": b["z"], "logsnr": torch.stack([torch.full_like(lam, smp.lam0), lam], 1), "R": R, "t": T, "K": K}
    ec2 = m(dict(base, x=b["x"]), cond_mask=torch.ones(B, dtype=torch.bool))
    eu2 = m(dict(base, x=x_unc), cond_mask=torch.zeros(B, dtype=torch.bool))
    assert torch.allclose(ec, ec2, atol=1e-5) and torch.allclose(eu, eu2, atol=1e-5)


def test_sampler_quirk_and_shards():
    m = tiny_model().eval()
    for quirk in (False, True):
        smp = DiffusionSampler(m, timesteps=4, ref_quirk=quirk, seed=0)
        rec = [RecordEntry(torch.zeros(2, 3, 16, 16), torch.eye(3), torch.tensor([0.0, 0.0, 1.3]))]
        out = smp.sample(rec, torch.eye(3), torch.tensor([0.0, 1.3, 0.0]),
                         torch.tensor([[20.0, 0, 8], [0, 20.0, 8], [0, 0, 1]]), torch.tensor([0.0, 3.0]))
        assert out.shape == (2, 3, 16, 16) and torch.isfinite(out).all()
    spans = [shard_range(8, r, 3) for r in range(3)]
    assert spans == [(0, 3), (3, 6), (6, 8)]


def test_sampler_chains_independent_of_sharding():
    """Counter-based noise keyed by the GLOBAL chain index: chains 2..4 of a
    5-chain run equal a 3-chain run with chain_offset=2 (what rank r of a
    multi-GPU sampling job computes)."""
    m = tiny_model().eval()
    K = torch.tensor([[20.0, 0, 8], [0, 20.0, 8], [0, 0, 1]])
    img = torch.rand(5, 3, 16, 16) * 2 - 1
    w = torch.tensor([0.0, 1.0, 2.0, 3.0, 4.0])
    outs = []
    for lo, hi in ((0, 5), (2, 5)):
        smp = DiffusionSampler(m, timesteps=3, seed=7, chain_offset=lo)
        rec = [RecordEntry(img[lo:hi], torch.eye(3), torch.tensor([0.0, 0.0, 1.3])),
               RecordEntry(img[lo:hi].flip(-1), torch.eye(3), torch.tensor([0.0, 1.3, 0.0]))]
        outs.append(smp.sample(rec, torch.eye(3), torch.tensor([1.3, 0.0, 0.0]), K, w[lo:hi]))
    torch.testing.assert_close(outs[1], outs[0][2:], rtol=1e-4, atol=1e-5)


def _signal_model():
    """tiny_model with its zero-init layers randomised, so the output depends
    on the conditioning through every path."""
    m = tiny_model().eval()
    torch.manual_seed(3)
    with torch.no_grad():
        for p in m.parameters():
            if p.abs().sum() == 0:
                p.normal_(0, 0.05)
    return m


def test_shared_cond_forward_matches_per_example():
    """XUNet.forward(shared_cond=) -- conditioning per class, FiLM read
    through the row -> class map -- equals the per-example forward."""
    from helpers import tiny_batch
    m = _signal_model()
    b = tiny_batch(1)
    B = 5
    R = torch.cat([b["R"]] * B)
    T = torch.cat([b["t"]] * B)
    K = torch.cat([b["K"]] * B)
    x = torch.rand(B, 3, 16, 16) * 2 - 1
    z = torch.randn(B, 3, 16, 16)
    lg = torch.tensor([[20.0, -1.5]] * B)
    cls = torch.tensor([0, 1, 1, 0, 1], dtype=torch.int32)
    mask = cls == 0
    with torch.no_grad():
        ref = m({"x": x, "z": z, "logsnr": lg, "R": R, "t": T, "K": K}, cond_mask=mask)
        sc = {"R": R[:2], "t": T[:2], "K": K[:2], "logsnr": lg[:2], "cond_mask": torch.tensor([True, False]),
              "example_class": cls}
        out = m({"x": x, "z": z}, shared_cond=sc)
    assert ref.abs().max() > 1e-3
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-5)
    with pytest.raises(RuntimeError):
        m({"x": x, "z": z}, shared_cond=sc)      # inference only


def test_sampler_shared_cond_matches_per_chain():
    m = _signal_model()
    K = torch.tensor([[20.0, 0, 8], [0, 20.0, 8], [0, 0, 1]])
    img = torch.rand(3, 3, 16, 16) * 2 - 1
    w = torch.tensor([0.0, 1.0, 3.0])
    outs = []
    for share in (False, True):
        smp = DiffusionSampler(m, timesteps=3, seed=5, share_cond=share)
        rec = [RecordEntry(img, torch.eye(3), torch.tensor([0.0, 0.0, 1.3])),
               RecordEntry(img.flip(-1), torch.eye(3), torch.tensor([0.0, 1.3, 0.0]))]
        outs.append(smp.sample(rec, torch.eye(3), torch.tensor([1.3, 0.0, 0.0]), K, w))
    torch.testing.assert_close(outs[1], outs[0], rtol=1e-4, atol=1e-5)


def test_lightning_cli_layout(srn_root, tmp_path):
    """`lightning/train.py` (reference T3): cars.pickle index inside --train_data,
    --transfer initialises from a checkpoint FILE and restarts at step 0,
    warmup spans one pass over the training set."""
    import shutil
    import lightning.train as ltrain
    from lightning.xunet import XUNet as LX
    from lightning.diff3d import Diff3D  # noqa: F401
    from lightning.SRNdataset import dataset  # noqa: F401
    from distributed_3d_diffusion_pytorch_amd.models import XUNet
    assert LX is XUNet
    shutil.copy(os.path.join(srn_root, "index.pkl"), os.path.join(srn_root, "cars.pickle"))
    tiny = [f"{k}={v}" for k, v in TINY_OV.items() if k not in ("global_batch",)]
    out = str(tmp_path / "lt")
    ltrain.main(["--train_data", srn_root, "--out_dir", out, "max_steps=2", "num_epochs=100"] + tiny)
    ck = torch.load(os.path.join(out, "latest.pt"), weights_only=True)
    assert ck["step"] == 2
    # the Lightning defaults reach the trainer config
    _, rargs = ltrain.to_root_args(ltrain.parse(["--train_data", srn_root, "--transfer", "x.pt"]))
    ov = dict(o.split("=", 1) for o in rargs.overrides)
    assert ov["global_batch"] == "4" and ov["optim.warmup_examples"] == "-1" and ov["pretrained"] == "x.pt"
    assert rargs.index.endswith("cars.pickle")
    # --transfer FILE: weights come from the file, the step counter restarts
    out2 = str(tmp_path / "lt2")
    ltrain.main(["--train_data", srn_root, "--out_dir", out2, "--transfer", os.path.join(out, "latest.pt"),
                 "max_steps=1", "num_epochs=100"] + tiny)
    ck2 = torch.load(os.path.join(out2, "latest.pt"), weights_only=True)
    assert ck2["step"] == 1
