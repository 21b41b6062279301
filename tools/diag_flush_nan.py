"""Diagnostic: the 1-rank RCCL graph step (32x32, bs4, captured collectives,
deferred update) with a given weight-gradient flush batch, reporting after
every step which parameters' complete gradients (the reducer race probe's
copy at finish()) hold non-finite values -- to locate the NaN that flush
batch 32 produces (profiles/r6/defer_batch.txt).

    D3D_WGRAD_DEFER_BATCH=32 python tools/diag_flush_nan.py [graph 0|1] [payload fp32|bf16] [comm|nocomm]
"""
import datetime
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def worker(graph, gd, comm=True):
    import torch
    import torch.distributed as dist
    from distributed_3d_diffusion_pytorch_amd.config import make_config
    from distributed_3d_diffusion_pytorch_amd.engine import Trainer
    from distributed_3d_diffusion_pytorch_amd.parallel import DistContext, cleanup
    from distributed_3d_diffusion_pytorch_amd.parallel.dist import rccl_env_defaults
    from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches
    rccl_env_defaults()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev, timeout=datetime.timedelta(seconds=120))
    ctx = DistContext(device=dev)
    data = SyntheticBatches(4, 32, "cuda", seed=21)
    cfg = make_config(None, {"model.H": 32, "model.W": 32, "data.imgsize": 32, "global_batch": 4, "micro_batch": 0,
                             "data.synthetic": True, "log_every": 0, "ckpt_every": 0, "graph": bool(graph),
                             "optim.warmup_examples": 8, "dist.bucket_mb": float(os.environ.get("DIAG_BUCKET_MB", "16")), "dist.grad_dtype": gd,
                             "dist.force_comm": bool(comm)})
    tr = Trainer(cfg, ctx)
    if not comm:
        print("defer_batch", tr.sink.defer_batch, "(no collectives)", flush=True)
        for step in range(5):
            loss = float(tr.train_step(*next(data)))
            torch.cuda.synchronize()
            print(f"step {step} loss {loss:.5f} params finite {bool(torch.isfinite(tr.flat.data).all())}", flush=True)
        tr.sync()
        torch.cuda.synchronize()
        print("after sync params finite", bool(torch.isfinite(tr.flat.data).all()), flush=True)
        cleanup()
        return
    if os.environ.get("DIAG_NO_PROBE") != "1":
        tr.reducer.enable_race_probe()
    names = [n for n, _ in tr.model.named_parameters()]
    print("defer_batch", tr.sink.defer_batch, "buckets", len(tr.reducer.buckets), flush=True)
    for step in range(4):
        loss = float(tr.train_step(*next(data)))
        torch.cuda.synchronize()
        if tr.reducer.race_probe is None:
            print(f"step {step} loss {loss:.5f} params finite {bool(torch.isfinite(tr.flat.data).all())}", flush=True)
            continue
        snap, final = tr.reducer.race_probe
        bad = []
        for i in range(len(tr.flat.params)):
            s, e = tr.flat.span(i)
            g = final[s:e]
            if not torch.isfinite(g).all():
                bad.append((i, names[i], int((~torch.isfinite(g)).sum())))
        zero = sum(1 for i in range(len(tr.flat.params))
                   if final[tr.flat.span(i)[0]: tr.flat.span(i)[1]].abs().max().item() == 0)
        print(f"step {step} loss {loss:.5f} nonfinite-grad params {len(bad)} zero-grad params {zero} "
              f"params finite {bool(torch.isfinite(tr.flat.data).all())}", flush=True)
        for b in bad[:12]:
            print("   ", b, "bucket", tr.reducer.param_bucket.get(b[0]), flush=True)
    tr.sync()
    torch.cuda.synchronize()
    print("after sync params finite", bool(torch.isfinite(tr.flat.data).all()), flush=True)
    cleanup()


def main():
    from distributed_3d_diffusion_pytorch_amd.parallel import spawn
    graph = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    gd = os.environ.get("DIAG_PAYLOAD") or (sys.argv[2] if len(sys.argv) > 2 else "fp32")
    comm = (sys.argv[3] if len(sys.argv) > 3 else "comm") != "nocomm"
    spawn(_entry, 1, (graph, gd, comm))


def _entry(graph, gd, comm):
    worker(graph, gd, comm)


if __name__ == "__main__":
    main()
