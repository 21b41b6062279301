#!/usr/bin/env python
"""Headline benchmark: X-UNet training throughput on SRN-cars-shaped data.

Metric (BASELINE.json): train imgs/sec for the whole node, SRN cars 64x64,
global batch 128 (reference: ≈29.9 examples/s on 8x RTX 3090, README.md:39).
One "example" = one 2-view training pair.

    python bench.py --gpus N --steps K --warmup W          (self-spawns N ranks)
    torchrun --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Launch: under torchrun (WORLD_SIZE set) every process is one rank.  Without
it and with ``--gpus N > 1`` this process becomes a launcher: it starts N fresh
child interpreters (one per GPU, RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* on
127.0.0.1), never touches the GPU itself, and exits with the worst child status
(reference launcher: ``mp.spawn`` in `train.py:189-193`).

Scaling is *strong* by default: the global batch stays 128 (the published
config) and each of the N ranks trains on 128/N examples per step, so every
point of the 1/2/4/8-GPU curve is the headline config itself.  Pass
``--per_gpu_batch B`` for weak scaling (global = B*N).  Data are synthetic
SRN-shaped batches generated on the device; weights are random-init at the
full 136.7M-parameter architecture; every timed step is a complete
forward + backward + gradient all-reduce + Adam update.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

BASELINE_EX_PER_S = 29.9  # 101,000 steps x 128 / 432,000 s on 8x RTX 3090


def _launch(nprocs: int) -> int:
    """Start ``nprocs`` ranks of this script as child processes (fresh
    interpreters: the launcher itself never initialises the GPU) and wait.
    A failing rank takes the others down (by their exact PIDs)."""
    import signal
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(nprocs):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nprocs), LOCAL_WORLD_SIZE=str(nprocs),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:              # one rank died: end the job instead of hanging in a collective
                    q.send_signal(signal.SIGTERM)
        time.sleep(0.05)
    return rc


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--global_batch", type=int, default=128)
    ap.add_argument("--per_gpu_batch", type=int, default=0, help="weak scaling: fixed per-GPU batch")
    ap.add_argument("--micro_batch", type=int, default=-1, help="-1 = auto")
    ap.add_argument("--imgsize", type=int, default=64)
    ap.add_argument("--backend", default="auto")
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--bucket_mb", type=float, default=64.0)
    ap.add_argument("--grad_dtype", default="fp32")
    ap.add_argument("--force_comm", action="store_true",
                    help="1-GPU rehearsal of the multi-GPU step: a 1-rank RCCL group with the bucketed reducer and "
                         "its collectives on (D3D_GRAPH_COMM=0 / D3D_GRAPH_SEG=0 select the fallback modes)")
    ap.add_argument("--graph", default="auto",
                    help="1: replay the step from captured HIP graphs; auto: when the per-GPU micro-batch is "
                         "<= 64 (graph +2.2 %% at 64, -2.5 %% at 128: profiles/r5/graph_threshold/; at small "
                         "batches the eager step is host-launch-bound)")
    ap.add_argument("--profile", default="", help="write a torch.profiler kernel table (text) here")
    ap.add_argument("--profile_stack", type=int, default=0, help="with --profile: also group by N stack frames")
    ap.add_argument("--mode", default="train", choices=["train", "sample"],
                    help="sample: 256-step stochastic-conditioning CFG sampling wall-clock (BASELINE config 5)")
    ap.add_argument("--sample_batch", type=int, default=64)
    ap.add_argument("--timesteps", type=int, default=256)
    ap.add_argument("--no_share_cond", action="store_true",
                    help="sample: per-chain conditioning instead of once per CFG class (A/B)")
    ap.add_argument("--device", default="auto", choices=["auto", "cpu"],
                    help="cpu: gloo ranks on the host (launcher / plumbing tests)")
    ap.add_argument("--ch", type=int, default=128, help="model width (128 = the benchmarked architecture)")
    ap.add_argument("--emb_ch", type=int, default=1024)
    args = ap.parse_args()
    if args.mode == "sample":
        return bench_sample(args)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(_launch(args.gpus))

    from distributed_3d_diffusion_pytorch_amd.config import make_config
    from distributed_3d_diffusion_pytorch_amd.parallel import init_distributed, cleanup, barrier
    from distributed_3d_diffusion_pytorch_amd.engine import Trainer
    from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches

    ctx = init_distributed("auto", timeout_s=900, use_gpu=False if args.device == "cpu" else None)
    N = ctx.world
    if args.force_comm and N == 1 and ctx.device.type == "cuda":
        import datetime
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29531")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=ctx.device,
                                timeout=datetime.timedelta(seconds=300))
    if args.gpus and args.gpus != N and ctx.rank == 0:
        print(f"[bench] warning: --gpus {args.gpus} but WORLD_SIZE={N}", file=sys.stderr)
    if args.per_gpu_batch:
        global_batch = args.per_gpu_batch * N
        scaling = "weak"
    else:
        global_batch = args.global_batch
        scaling = "strong"
    local = global_batch // N
    mb = args.micro_batch
    if mb < 0:
        # one micro-batch whenever the rank's batch fits comfortably in HBM: at
        # 64x64 the whole 128-example batch is one pass (~+8 % over two passes
        # of 64, profiles/ab_bs128_modes_r2.txt); larger images split into 64s
        mb = 0 if local * args.imgsize * args.imgsize <= 128 * 64 * 64 else 64
    if args.graph == "auto":
        graph = ctx.device.type == "cuda" and (mb or local) <= 64
    else:
        graph = bool(int(args.graph))
    cfg = make_config(None, {"model.H": args.imgsize, "model.W": args.imgsize, "data.imgsize": args.imgsize,
                             "model.ch": args.ch, "model.emb_ch": args.emb_ch,
                             "global_batch": global_batch, "micro_batch": mb, "data.synthetic": True,
                             "backend": args.backend, "dtype": args.dtype, "log_every": 0, "ckpt_every": 0,
                             "dist.bucket_mb": args.bucket_mb, "dist.grad_dtype": args.grad_dtype,
                             "dist.force_comm": bool(args.force_comm), "graph": graph})
    trainer = Trainer(cfg, ctx)
    data = SyntheticBatches(local, args.imgsize, ctx.device, seed=1234 + ctx.rank)
    pool = [next(data) for _ in range(4)]

    def sync():
        if ctx.device.type == "cuda":
            torch.cuda.synchronize()

    for i in range(args.warmup):
        trainer.train_step(*pool[i % len(pool)])
    sync()
    barrier()
    sync()
    prof = None
    if args.profile:
        prof = torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU,
                                                  torch.profiler.ProfilerActivity.CUDA],
                                      with_stack=bool(args.profile_stack))
        prof.__enter__()
    t0 = time.perf_counter()
    loss = None
    for i in range(args.steps):
        loss = trainer.train_step(*pool[i % len(pool)])
    sync()
    barrier()
    sync()
    dt = time.perf_counter() - t0
    trainer.sync()          # (a deferred update of the last timed step; outside the timed region)
    # memory record of the benchmark itself (the comm diagnostics below capture / run extra steps)
    hbm_peak = round(torch.cuda.max_memory_allocated() / 2 ** 30, 2) if ctx.device.type == "cuda" else None
    retries = torch.cuda.memory_stats().get("num_alloc_retries", 0) if ctx.device.type == "cuda" else None
    comm = comm_diagnostics(trainer, pool, ctx) if (trainer.reducer is not None and trainer.reducer.active) else None
    if prof is not None:
        prof.__exit__(None, None, None)
        if ctx.rank == 0:
            with open(args.profile, "w") as f:
                f.write(prof.key_averages().table(sort_by="cuda_time_total", row_limit=60))
                if args.profile_stack:     # which Python lines issue the glue ops
                    f.write("\n\n" + prof.key_averages(group_by_stack_n=args.profile_stack).table(
                        sort_by="self_cuda_time_total", row_limit=80))
    from distributed_3d_diffusion_pytorch_amd.parallel import all_reduce_max
    dt = all_reduce_max(dt, ctx.device)
    lv = float(loss) if loss is not None else float("nan")
    ms = 1e3 * dt / max(args.steps, 1)
    value = global_batch * args.steps / dt
    if ctx.rank == 0:
        from distributed_3d_diffusion_pytorch_amd.ops import use_hip
        probe = torch.zeros(1, device=ctx.device, dtype=torch.bfloat16)
        out = {
            "metric": f"train imgs/sec (whole node), SRN cars {args.imgsize}x{args.imgsize} bs{global_batch}",
            "value": round(value, 3), "unit": "examples/s", "n_gpus": N, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": round(value / BASELINE_EX_PER_S, 3) if (args.imgsize == 64 and args.ch == 128) else None,
            "dtype": args.dtype, "data": "synthetic (on-device SRN-shaped batches, random-init weights)",
            "config": {"model": (f"XUNet ch{args.ch} ch_mult(1,2,2,4) "
                                 f"{sum(p.numel() for p in trainer.model.parameters()) / 1e6:.1f}M params "
                                 "(3DiM, reference xunet.py)"),
                       "global_batch": global_batch, "seq_len": args.imgsize * args.imgsize,
                       "image_size": args.imgsize, "per_gpu_batch": local, "micro_batch": mb or local,
                       "hip_graph": bool(trainer.cfg.graph),
                       "parallelism": f"dp{N}", "dist_backend": ctx.backend,
                       "graph_comm": getattr(trainer._graphed, "comm_mode", None),
                       "tuned_gemms": bool(getattr(trainer, "tuned_gemms", False)),
                       "backend": "hip" if (ctx.device.type == "cuda" and use_hip(probe)) else "torch"},
            "final_loss": lv,
            # N > 1: what the gradient communication did (measured after the timed steps)
            "comm": comm,
            "hbm_peak_gib": hbm_peak,
            # caching-allocator retries (a full cache flush + device sync each): non-zero means the step
            # ran at the HBM limit and paid for it
            "alloc_retries": retries,
            # (op, shape) pairs that left the HIP kernels for the torch composition (only possible with
            # D3D_ALLOW_TORCH_FALLBACK=1; otherwise such a shape is an error)
            "fallbacks": _fallback_count(),
        }
        print(json.dumps(out), flush=True)
    cleanup()


def _fallback_count() -> int:
    try:
        from distributed_3d_diffusion_pytorch_amd.ops import hip_impl
    except Exception:           # noqa: BLE001 -- no native library (CPU plumbing run)
        return 0
    return len(hip_impl.FALLBACKS)


def comm_diagnostics(trainer, pool, ctx) -> dict:
    """Gradient-communication record of a multi-rank run (untimed, after the
    benchmark): bucket layout and payload, the process group's own world size,
    the step path (eager / graph with the all-reduces captured / post-graph
    chunked) with the capture probe's verdict, and the exposed all-reduce time
    per step (max over ranks):
      * eager step: device events around the reducer's join (host wall-clock
        on gloo);
      * graph step: graph A replayed against a capture of itself without the
        collectives (GraphedTrainStep.measure_comm)."""
    import torch.distributed as dist
    from distributed_3d_diffusion_pytorch_amd.parallel import all_reduce_max
    red = trainer.reducer
    info = red.describe()
    info["world_pg"] = dist.get_world_size() if dist.is_initialized() else 1
    info["backend_pg"] = dist.get_backend() if dist.is_initialized() else None
    g = trainer._graphed
    ms = -1.0
    try:            # (every rank reaches the all_reduce_max below, whatever happens here)
        if trainer.cfg.graph and g is not None:
            info["step"] = "graph"
            info["comm_mode"] = g.comm_mode
            info["probe_ok"] = g.comm_mode == "graph"
            info["segments"] = len(g.segs) if g.segs else None
            ms = g.measure_comm(3)
        else:
            info["step"] = "eager"
            info["comm_mode"] = "eager"
            info["probe_ok"] = None
            vals = []
            for i in range(3):
                trainer.train_step(*pool[i % len(pool)], want_stats=True)
                vals.append(trainer.last_allreduce_ms)
            ms = sum(vals) / len(vals)
    except Exception as e:      # noqa: BLE001 -- a diagnostic must not lose the benchmark line
        info["error"] = f"{type(e).__name__}: {e}"[:200]
    info["exposed_allreduce_ms"] = round(all_reduce_max(float(ms if ms is not None else 0.0), ctx.device), 3)
    return info


def bench_sample(args) -> None:
    """Wall-clock of generating one novel view with the 256-step CFG ancestral
    sampler and stochastic conditioning (sampling.py:129-155) for a batch of
    `sample_batch` chains on one GPU (random-init weights, synthetic poses)."""
    from distributed_3d_diffusion_pytorch_amd.models import XUNet
    from distributed_3d_diffusion_pytorch_amd.models.flops import forward_flops
    from distributed_3d_diffusion_pytorch_amd.engine import DiffusionSampler, RecordEntry
    from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches
    from distributed_3d_diffusion_pytorch_amd import ops
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    if args.backend != "auto":
        ops.set_backend(args.backend)
    torch.manual_seed(0)
    S = args.imgsize
    model = XUNet(H=S, W=S, ch=128).to(dev)
    model.compute_dtype = torch.bfloat16 if dev.type == "cuda" else torch.float32
    model.eval()
    b = args.sample_batch
    img, R, T, K = next(SyntheticBatches(b, S, dev, seed=0))
    record = [RecordEntry(img[:, 0].contiguous(), R[0, 0].float(), T[0, 0].float()),
              RecordEntry(img[:, 1].contiguous(), R[0, 1].float(), T[0, 1].float())]
    w = torch.arange(b, dtype=torch.float32) % 8
    share = not args.no_share_cond
    smp = DiffusionSampler(model, args.timesteps, seed=0, device=dev, share_cond=share)
    # warmup: a few steps through the same code path
    warm = DiffusionSampler(model, max(2, args.warmup), seed=1, device=dev, share_cond=share)
    warm.sample(record, R[1, 0].float(), T[1, 0].float(), K[0].float(), w)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = smp.sample(record, R[1, 0].float(), T[1, 0].float(), K[0].float(), w)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0

    res = {"metric": f"{args.timesteps}-step sample wall-clock, stochastic conditioning, bs{b}, {S}x{S}", "value": round(dt, 3),
           "unit": "s", "n_gpus": 1, "steps": args.timesteps, "warmup": args.warmup,
           "ms_per_step": round(1e3 * dt / args.timesteps, 3), "higher_is_better": False, "scaling": "none",
           "vs_baseline": None, "dtype": "bf16", "data": "synthetic poses/images, random-init weights",
           "config": {"model": "XUNet ch128 136.7M", "global_batch": b, "cfg_batch": 2 * b, "image_size": S,
                      "parallelism": "single", "shared_conditioning": share},
           # FLOPs the step actually executes (models/flops.py: the 2b-example
           # trunk, the conditioning part on the 2 CFG classes when shared)
           "executed_tflops": round(forward_flops(model, 2 * b, 2 if share else None) * args.timesteps / dt / 1e12,
                                    1),
           "finite": bool(torch.isfinite(out).all())}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
