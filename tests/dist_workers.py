"""Multi-process worker bodies for test_distributed.py (spawned ranks read
RANK/WORLD_SIZE from the environment like torchrun workers)."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

# several ranks share this host's CPUs: one intra-op pool per rank of the full
# CPU count oversubscribes it many times over
torch.set_num_threads(max(1, (os.cpu_count() or 8) // 4))

TINY_OV = {"model.ch": 32, "model.emb_ch": 64, "model.H": 16, "model.W": 16, "data.imgsize": 16,
           "dtype": "fp32", "backend": "torch", "log_every": 0, "ckpt_every": 0, "data.synthetic": True,
           "dist.timeout_s": 20.0}


def reducer_matches_manual_average(out_dir, bucket_mb, grad_dtype="fp32"):
    from distributed_3d_diffusion_pytorch_amd.parallel import init_distributed, cleanup, FlatParams, GradReducer
    from helpers import tiny_model, tiny_batch
    ctx = init_distributed("gloo", 60, use_gpu=False)
    m = tiny_model(seed=0).eval()      # no dropout: both passes must be identical
    flat = FlatParams(list(m.parameters()))
    red = GradReducer(flat, bucket_mb=bucket_mb, first_bucket_mb=bucket_mb / 4, grad_dtype=grad_dtype)
    assert (red.mirror is not None) == (grad_dtype == "bf16")
    assert len(red.buckets) >= 1
    b = tiny_batch(2, seed=10 + ctx.rank)       # different data per rank
    cm = torch.tensor([True, ctx.rank == 0])
    # local gradient without communication
    with red.no_sync():
        m(b, cond_mask=cm).square().mean().backward()
    local = flat.grad.clone()
    flat.zero_grad()
    red.reset()
    # reduced gradient through the bucketed hooks
    m(b, cond_mask=cm).square().mean().backward()
    red.finish()
    summed = flat.grad.clone()
    ref = local.clone()
    if grad_dtype == "bf16":            # the payload is rounded to bf16 before the sum
        ref = local.to(torch.bfloat16)
        dist.all_reduce(ref)
        ok = torch.allclose(summed, ref.float(), atol=1e-6, rtol=1e-5)
    else:
        dist.all_reduce(ref)
        ok = torch.allclose(summed, ref, atol=1e-6, rtol=1e-5)
    with open(os.path.join(out_dir, f"r{ctx.rank}.txt"), "w") as f:
        f.write(f"{int(ok)} {len(red.buckets)}")
    cleanup()


def trainer_in_sync(out_dir):
    from distributed_3d_diffusion_pytorch_amd.config import make_config
    from distributed_3d_diffusion_pytorch_amd.parallel import init_distributed, cleanup, check_replicas_in_sync
    from distributed_3d_diffusion_pytorch_amd.engine import Trainer
    from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches
    ctx = init_distributed("gloo", 60, use_gpu=False)
    cfg = make_config(None, dict(TINY_OV, **{"global_batch": 4, "out_dir": out_dir, "dist.checksum_every": 1}))
    tr = Trainer(cfg, ctx)
    data = SyntheticBatches(tr.local_batch, 16, "cpu", seed=ctx.rank)
    for _ in range(3):
        tr.train_step(*next(data))
    ok = check_replicas_in_sync(tr.flat)
    tr.save("latest.pt", epoch=0)
    with open(os.path.join(out_dir, f"sync{ctx.rank}.txt"), "w") as f:
        f.write(str(int(ok)))
    cleanup()


def fault_injection(out_dir):
    os.environ["D3D_FAULT_AT_STEP"] = "1"
    os.environ["D3D_FAULT_RANK"] = "1"
    from distributed_3d_diffusion_pytorch_amd.config import make_config
    from distributed_3d_diffusion_pytorch_amd.parallel import init_distributed
    from distributed_3d_diffusion_pytorch_amd.engine import Trainer
    from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches
    ctx = init_distributed("gloo", 10, use_gpu=False)
    cfg = make_config(None, dict(TINY_OV, **{"global_batch": 4, "out_dir": out_dir, "dist.timeout_s": 10.0}))
    tr = Trainer(cfg, ctx)
    data = SyntheticBatches(tr.local_batch, 16, "cpu", seed=ctx.rank)
    for _ in range(4):
        tr.train_step(*next(data))
    # only reached if the dead peer went unnoticed
    with open(os.path.join(out_dir, f"survived{ctx.rank}.txt"), "w") as f:
        f.write("1")


def gpu_sink_reducer(out_dir):
    """Two ranks sharing one GPU over gloo: HIP kernels + direct gradient sink +
    bucketed reducer must equal the manual all-reduce of plain autograd grads."""
    import torch
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
    # reference: plain autograd grads, manual all-reduce
    with red.no_sync():
        m(batch, cond_mask=mask).float().square().mean().backward()
    ref = flat.grad.clone()
    torch.distributed.all_reduce(ref)
    flat.zero_grad()
    red.reset()
    # sink path
    views = [flat.view(flat.grad, i) for i in range(len(flat.params))]
    SINK.attach(flat.params, views, red.mark_ready)
    red.sink = SINK
    SINK.reset()
    m(batch, cond_mask=mask).float().square().mean().backward()
    red.finish()
    got = flat.grad.clone()
    SINK.detach()
    cos = torch.nn.functional.cosine_similarity(got, ref, dim=0).item()
    rel = ((got - ref).norm() / ref.norm()).item()
    with open(os.path.join(out_dir, f"g{ctx.rank}.txt"), "w") as f:
        f.write(f"{cos} {rel}")
    cleanup()


def gpu_graph_vs_eager(out_dir):
    """Two ranks sharing one GPU over gloo: the HIP-graph step (one flat
    all-reduce between the replayed graphs) must track the eager step
    (bucketed all-reduce from backward hooks) and keep the replicas equal."""
    import torch
    from distributed_3d_diffusion_pytorch_amd.config import make_config
    from distributed_3d_diffusion_pytorch_amd.engine import Trainer
    from distributed_3d_diffusion_pytorch_amd.parallel import init_distributed, cleanup
    from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches
    ctx = init_distributed("gloo", 180, use_gpu=True)

    def make(graph):
        cfg = make_config(None, {"model.H": 32, "model.W": 32, "model.dropout": 0.0, "data.imgsize": 32,
                                 "global_batch": 8, "micro_batch": 2, "data.synthetic": True, "log_every": 0,
                                 "ckpt_every": 0, "graph": graph, "optim.warmup_examples": 16})
        return Trainer(cfg, ctx)

    data = SyntheticBatches(4, 32, "cuda", seed=11 + ctx.rank)
    batches = [next(data) for _ in range(3)]
    out = []
    for graph in (False, True):
        torch.manual_seed(0)
        tr = make(graph)
        losses = [float(tr.train_step(*b)) for b in batches]
        tr.sync()
        p = tr.flat.data.clone()
        other = p.clone()
        torch.distributed.broadcast(other, 0)
        out.append((losses, p, (p - other).abs().max().item()))
        del tr
    (le, pe, de), (lg, pg, dg) = out
    d = (pe - pg).abs().max().item()
    with open(os.path.join(out_dir, f"gr{ctx.rank}.txt"), "w") as f:
        f.write(f"{d} {de} {dg} {max(abs(a - b) for a, b in zip(le, lg))}")
    cleanup()


def two_node_emulation(out_dir):
    """4 ranks laid out as 2 "nodes" x 2 local ranks (LOCAL_RANK != RANK on the
    second node, as torchrun exports it on a multi-node job): 2 steps, rank-0
    checkpoint, then every rank resumes from it into a fresh trainer and steps
    again -- replicas must agree after the resume too (SURVEY §4 distributed tier)."""
    rank = int(os.environ["RANK"])
    os.environ["LOCAL_RANK"] = str(rank % 2)
    os.environ["LOCAL_WORLD_SIZE"] = "2"
    from distributed_3d_diffusion_pytorch_amd.config import make_config
    from distributed_3d_diffusion_pytorch_amd.parallel import init_distributed, cleanup, check_replicas_in_sync
    from distributed_3d_diffusion_pytorch_amd.engine import Trainer
    from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches
    ctx = init_distributed("gloo", 60, use_gpu=False)
    assert ctx.local_rank == rank % 2 and ctx.world == 4
    cfg = make_config(None, dict(TINY_OV, **{"global_batch": 8, "out_dir": out_dir}))
    tr = Trainer(cfg, ctx)
    assert tr.local_batch == 2
    data = SyntheticBatches(tr.local_batch, 16, "cpu", seed=ctx.rank)
    for _ in range(2):
        tr.train_step(*next(data))
    ok = check_replicas_in_sync(tr.flat)
    tr.save("latest.pt", epoch=0)
    dist.barrier()
    cfg2 = make_config(None, dict(TINY_OV, **{"global_batch": 8, "out_dir": out_dir, "transfer": out_dir}))
    tr2 = Trainer(cfg2, ctx)
    same = bool(torch.equal(tr2.flat.data, tr.flat.data)) and tr2.step == tr.step == 2
    tr2.train_step(*next(data))
    ok2 = check_replicas_in_sync(tr2.flat) and tr2.step == 3
    with open(os.path.join(out_dir, f"node{ctx.rank}.txt"), "w") as f:
        f.write(f"{int(ok)} {int(same)} {int(ok2)}")
    cleanup()


def capture_agreement(out_dir):
    """8 gloo ranks: the cross-rank checks that guard the graph step's
    collective sequence (engine/graphs.py) -- the captured bucket order
    (comm_mode "graph"), the segment layout (comm_mode "seg") and the
    agreement of per-rank environment switches -- on real reducer buckets."""
    import types
    from distributed_3d_diffusion_pytorch_amd.parallel import init_distributed, cleanup, FlatParams, GradReducer
    from distributed_3d_diffusion_pytorch_amd.engine.graphs import GraphedTrainStep, agree_switches
    from helpers import tiny_model, tiny_batch
    ctx = init_distributed("gloo", 60, use_gpu=False)
    r = ctx.rank
    m = tiny_model(seed=0).eval()
    flat = FlatParams(list(m.parameters()))
    red = GradReducer(flat, bucket_mb=0.05, first_bucket_mb=0.01)
    nb = len(red.buckets)
    # the real issue order of an eager bucketed backward: the same on every rank
    red.reset()
    m(tiny_batch(2, seed=10 + r), cond_mask=torch.tensor([True, True])).square().mean().backward()
    red.finish()
    real = list(red.issue_log)
    st = types.SimpleNamespace(tr=types.SimpleNamespace(reducer=red, device=torch.device("cpu")), gA=object())
    res = [GraphedTrainStep._issue_order_agrees(st)]
    red.issue_log = real[:2][::-1] + real[2:] if r == 3 else list(real)           # rank 3 swaps two buckets
    res.append(GraphedTrainStep._issue_order_agrees(st))
    red.issue_log = list(real)
    st.gA = None if r == 5 else object()                                           # rank 5's capture failed
    res.append(GraphedTrainStep._issue_order_agrees(st))
    # segment layouts: equal, then rank 2 cuts one bucket later
    half = nb // 2
    st.segs = [None, None]
    st.seg_bk = [real[:half], real[half:]]
    res.append(GraphedTrainStep._segments_agree(st))
    if r == 2:
        st.seg_bk = [real[:half + 1], real[half + 1:]]
    res.append(GraphedTrainStep._segments_agree(st))
    # switches: rank 6 turns the captured collectives off, all keep segments on
    res.append(agree_switches(r != 6, True) == (False, True))
    with open(os.path.join(out_dir, f"agree{r}.txt"), "w") as f:
        f.write(f"{nb} {len(real)} " + " ".join(str(int(x)) for x in res))
    cleanup()
