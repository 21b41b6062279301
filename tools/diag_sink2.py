"""2 ranks on one GPU (gloo): reducer with/without sink vs manual allreduce; per-bucket report."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def worker(mode):
    import torch.distributed as dist
    from distributed_3d_diffusion_pytorch_amd.parallel import init_distributed, cleanup, FlatParams, GradReducer
    from distributed_3d_diffusion_pytorch_amd.ops.gradsink import SINK
    from distributed_3d_diffusion_pytorch_amd.models import XUNet
    from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches
    ctx = init_distributed("gloo", 120, use_gpu=True)
    torch.manual_seed(0)
    m = XUNet(H=32, W=32, ch=128).cuda().eval()
    with torch.no_grad():
        for p in m.parameters():
            if p.abs().sum() == 0:
                p.normal_(0, 0.02)
    m.compute_dtype = torch.bfloat16
    flat = FlatParams(list(m.parameters()))
    red = GradReducer(flat, bucket_mb=8.0, first_bucket_mb=1.0)
    img, R, t, K = next(SyntheticBatches(2, 32, "cuda", seed=ctx.rank))
    batch = {"x": img[:, 0], "z": img[:, 1], "logsnr": torch.tensor([[20.0, 1.0], [20.0, -2.0]], device="cuda"),
             "R": R, "t": t, "K": K}
    mask = torch.tensor([True, False], device="cuda")
    with red.no_sync():
        m(batch, cond_mask=mask).float().square().mean().backward()
    torch.cuda.synchronize()
    ref = flat.grad.clone()
    dist.all_reduce(ref)
    torch.cuda.synchronize()
    flat.zero_grad()
    red.reset()
    if mode == "sink":
        views = [flat.view(flat.grad, i) for i in range(len(flat.params))]
        SINK.attach(flat.params, views, red.mark_ready)
        red.sink = SINK
        SINK.reset()
    order = []
    orig = red._launch
    def launch(b):
        order.append(b)
        if os.environ.get("SYNC_BEFORE_LAUNCH") == "1":
            torch.cuda.synchronize()
        orig(b)
    red._launch = launch
    m(batch, cond_mask=mask).float().square().mean().backward()
    red.finish()
    torch.cuda.synchronize()
    got = flat.grad.clone()
    if ctx.rank == 0:
        for b, bk in enumerate(red.buckets):
            a, r = got[bk["start"]:bk["end"]], ref[bk["start"]:bk["end"]]
            d = ((a - r).norm() / r.norm().clamp_min(1e-12)).item()
            if d > 1e-2:
                print(f"[{mode}] bucket {b} params {len(bk['params'])} rel {d:.3g} launched_pos {order.index(b) if b in order else -1}")
        print(f"[{mode}] total rel {((got-ref).norm()/ref.norm()).item():.3g}; launch order {order}", flush=True)
    cleanup()


if __name__ == "__main__":
    from distributed_3d_diffusion_pytorch_amd.parallel import spawn
    for mode in ("hooks", "sink"):
        spawn(worker, 2, (mode,))
