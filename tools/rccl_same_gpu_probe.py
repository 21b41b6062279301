"""Can two RCCL ranks share one GPU on this stack?  (Decides whether the
multi-rank RCCL paths can be exercised on a 1-GPU box.)  Prints one line per
rank; exits non-zero if the collective fails."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def worker():
    import torch
    import torch.distributed as dist
    from distributed_3d_diffusion_pytorch_amd.parallel.dist import rccl_env_defaults
    rccl_env_defaults()
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", timeout=__import__("datetime").timedelta(seconds=60))
    x = torch.full((1024,), float(dist.get_rank() + 1), device="cuda")
    dist.all_reduce(x)
    torch.cuda.synchronize()
    print(f"rank {dist.get_rank()}: all_reduce -> {x[0].item()}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    import torch.multiprocessing as mp
    from distributed_3d_diffusion_pytorch_amd.parallel.dist import _spawn_entry, free_port
    mp.spawn(_spawn_entry, args=(worker, 2, free_port(), ()), nprocs=2, join=True)
