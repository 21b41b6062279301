"""Early FiLM weight gradient vs the bucketed bf16-payload reducer (1-rank
RCCL group, dist.force_comm): per step, NaN / max |grad| of the flat gradient
and parameters, eager and graph, early on and off."""
import datetime
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.distributed as dist


def main():
    from distributed_3d_diffusion_pytorch_amd.config import make_config
    from distributed_3d_diffusion_pytorch_amd.engine import Trainer
    from distributed_3d_diffusion_pytorch_amd.parallel import DistContext
    from distributed_3d_diffusion_pytorch_amd.parallel.dist import rccl_env_defaults
    from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches
    from distributed_3d_diffusion_pytorch_amd.ops import hip_impl as H
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    rccl_env_defaults()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev, timeout=datetime.timedelta(seconds=120))
    ctx = DistContext(device=dev)
    data = SyntheticBatches(4, 32, "cuda", seed=21)
    batches = [next(data) for _ in range(3)]
    gd = sys.argv[1] if len(sys.argv) > 1 else "bf16"
    from distributed_3d_diffusion_pytorch_amd.parallel import ddp as _ddp
    from distributed_3d_diffusion_pytorch_amd.ops.gradsink import SINK
    orig_launch, orig_finish = _ddp.GradReducer._launch, _ddp.GradReducer.finish
    log = []

    def launch(self, b):
        if not self._launched[b]:
            log.append(f"L{b}(q{len(SINK._queue)},f{int(bool(SINK._forked))})@{sid()}")
        return orig_launch(self, b)

    def finish(self):
        log.append(f"F(q{len(SINK._queue)})@{sid()}")
        return orig_finish(self)
    _ddp.GradReducer._launch, _ddp.GradReducer.finish = launch, finish
    orig_flush, orig_join, orig_eob = type(SINK).flush, type(SINK).join, type(SINK)._end_of_backward

    def sid():
        st = torch.cuda.current_stream()
        return f"s{st.cuda_stream % 100000}c{int(torch.cuda.is_current_stream_capturing())}"

    def flush(self):
        if self._queue:
            log.append(f"fl{len(self._queue)}@{sid()}")
        return orig_flush(self)

    def join(self):
        log.append(f"J{len(self._forked)}@{sid()}")
        return orig_join(self)

    def eob(self):
        log.append(f"EOB@{sid()}")
        return orig_eob(self)
    type(SINK).flush, type(SINK).join, type(SINK)._end_of_backward = flush, join, eob
    for early in (False, True):
        H._FILM_EARLY = early
        for graph in (False, True):
            cfg = make_config(None, {"model.H": 32, "model.W": 32, "data.imgsize": 32, "global_batch": 4,
                                     "micro_batch": 0, "data.synthetic": True, "log_every": 0, "ckpt_every": 0,
                                     "graph": graph, "optim.warmup_examples": 8, "dist.bucket_mb": 16.0,
                                     "dist.grad_dtype": gd, "dist.force_comm": True})
            tr = Trainer(cfg, ctx)
            if not early and not graph:
                names = {id(q): n for n, q in tr.model.named_parameters()}
                for bi in (0, 1, len(tr.reducer.buckets) - 1):
                    bk = tr.reducer.buckets[bi]
                    print(f"bucket {bi}: {[names.get(id(tr.flat.params[j]), '?') for j in bk['params']][:40]}",
                          flush=True)
            for i, b in enumerate(batches):
                log.clear()
                loss = float(tr.train_step(*b))
                print("   launches:", " ".join(log), flush=True)
                tr.sync()
                g, p = tr.flat.grad, tr.flat.data
                bad = torch.nonzero(~torch.isfinite(g)).flatten()
                where = ""
                if bad.numel():
                    i0 = int(bad[0])
                    for j, (a, q) in enumerate(zip(tr.flat.offsets, tr.flat.params)):
                        if a <= i0 < a + q.numel():
                            nb = int((~torch.isfinite(g[a:a + q.numel()])).sum())
                            where = f" first bad param #{j} {tuple(q.shape)} ({nb} bad)"
                            break
                names = {id(q): n for n, q in tr.model.named_parameters()}
                badp = [f"{names.get(id(q), '?')}{tuple(q.shape)}:{int((~torch.isfinite(q.data)).sum())}"
                        for q in tr.flat.params if not torch.isfinite(q.data).all()]
                print(f"{gd} early={int(early)} graph={int(graph)} step {i}: loss {loss:.5f} grad nonfinite "
                      f"{bad.numel()} max|g| {g.abs().max().item():.3e} param nonfinite "
                      f"{int((~torch.isfinite(p)).sum())}{where} bad params {badp[:12]} (+{max(0, len(badp) - 12)})",
                      flush=True)
            del tr
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
