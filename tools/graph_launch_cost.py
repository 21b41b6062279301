"""Host-side cost of replaying the captured bs16 training step (HIP graphs):
how long graph.replay() occupies the calling thread vs how long the GPU needs.
If the host time approaches the GPU time, the replayed step is host-bound."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    from distributed_3d_diffusion_pytorch_amd.config import make_config
    from distributed_3d_diffusion_pytorch_amd.engine import Trainer
    from distributed_3d_diffusion_pytorch_amd.parallel import DistContext
    from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches
    ctx = DistContext(device=torch.device("cuda", 0))
    cfg = make_config(None, {"model.H": 64, "model.W": 64, "data.imgsize": 64, "global_batch": B,
                             "micro_batch": 0, "data.synthetic": True, "log_every": 0, "ckpt_every": 0,
                             "graph": True})
    tr = Trainer(cfg, ctx)
    b = next(SyntheticBatches(B, 64, "cuda", seed=3))
    for _ in range(4):
        tr.train_step(*b)
    torch.cuda.synchronize()
    g = tr._graphed
    for name, gr in (("A (fwd+bwd)", g.gA), ("B (update)", g.gB)):
        hs, ts = [], []
        for _ in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            gr.replay()
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            hs.append(t1 - t0)
            ts.append(t2 - t0)
        print(f"graph {name}: host replay() {1e3 * min(hs):.3f} ms, replay+sync {1e3 * min(ts):.3f} ms", flush=True)
    # the full step, back to back: host time per step vs wall per step
    torch.cuda.synchronize()
    n = 10
    t0 = time.perf_counter()
    hs = []
    for _ in range(n):
        a = time.perf_counter()
        tr.train_step(*b)
        hs.append(time.perf_counter() - a)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"train_step host time {1e3 * sum(hs) / n:.3f} ms/step (loop {1e3 * (t1 - t0) / n:.3f}), "
          f"wall {1e3 * (t2 - t0) / n:.3f} ms/step", flush=True)


if __name__ == "__main__":
    main()


def segments(B=16, n=8):
    """Host time of each part of GraphedTrainStep.step over back-to-back steps."""
    from distributed_3d_diffusion_pytorch_amd.config import make_config
    from distributed_3d_diffusion_pytorch_amd.engine import Trainer
    from distributed_3d_diffusion_pytorch_amd.parallel import DistContext
    from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches
    from distributed_3d_diffusion_pytorch_amd.engine.trainer import dropout_word
    ctx = DistContext(device=torch.device("cuda", 0))
    cfg = make_config(None, {"model.H": 64, "model.W": 64, "data.imgsize": 64, "global_batch": B,
                             "micro_batch": 0, "data.synthetic": True, "log_every": 0, "ckpt_every": 0,
                             "graph": True})
    tr = Trainer(cfg, ctx)
    img, R, T, K = next(SyntheticBatches(B, 64, "cuda", seed=3))
    for _ in range(4):
        tr.train_step(img, R, T, K)
    torch.cuda.synchronize()
    g = tr._graphed
    o = tr.optim
    acc = {}

    def tick(k, t):
        now = time.perf_counter()
        acc[k] = acc.get(k, 0.0) + now - t
        return now

    t_all = time.perf_counter()
    for i in range(n):
        t = time.perf_counter()
        word = (tr.step + i) * tr.ctx.world + tr.ctx.rank
        g.frac.fill_(1.0)
        for j, v in enumerate((dropout_word(word, 0), word, 0)):
            g.seed[j].fill_(v)
        t = tick("fills", t)
        g.img.copy_(img)
        g.R.copy_(R)
        g.T.copy_(T)
        g.K.copy_(K)
        t = tick("copies", t)
        g.gA.replay()
        t = tick("gA.replay", t)
        loss = g.loss_acc.clone()
        t = tick("clone", t)
        o.hparams_to(g.hp, 1.0)
        t = tick("set_words", t)
        g.gB.replay()
        t = tick("gB.replay", t)
    t_host = time.perf_counter() - t_all
    torch.cuda.synchronize()
    wall = time.perf_counter() - t_all
    print("host ms/step by segment: " + ", ".join(f"{k} {1e3 * v / n:.3f}" for k, v in acc.items())
          + f" | host total {1e3 * t_host / n:.3f}, wall {1e3 * wall / n:.3f}", flush=True)


if __name__ == "__main__" and os.environ.get("GLC_SEGMENTS"):
    segments()
