"""Localise run-to-run differences of the training step: runs the same
4-step 64x64 batch-16 training several times (graph / eager, weight-gradient
side stream on / off) and reports, per step, which parameters' gradients
(and final Adam moments) differ bitwise from the first run and by how much.

usage: python tools/diag_determinism.py [variants]
  variant = <g|e>:<flags>, flags: s = weight-gradient side stream, c =
  conditioning stream, d = deferred update; runs are compared in pairs
  (1st vs 2nd, 3rd vs 4th, ...), e.g. g:scd,g:scd,g:cd,g:cd,e:sc,e:sc"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

CHECKSUMS = os.environ.get("DIAG_SUMS", "0") == "1"
KINDS = set()
SLOTS = []


def run(graph: bool, side: bool, batches, cond: bool = True, defer: bool = True):
    from distributed_3d_diffusion_pytorch_amd.config import make_config
    from distributed_3d_diffusion_pytorch_amd.engine import Trainer
    from distributed_3d_diffusion_pytorch_amd.parallel import DistContext
    from distributed_3d_diffusion_pytorch_amd.ops.gradsink import SINK
    from distributed_3d_diffusion_pytorch_amd.ops import hip_impl
    from distributed_3d_diffusion_pytorch_amd.models import xunet as X
    from distributed_3d_diffusion_pytorch_amd.engine import graphs as Gm
    SINK.stream_enabled = side
    if os.environ.get("DIAG_SERIAL_SIDE") == "1" and not getattr(SINK, "_diag_patched", False):
        # every side-stream job is joined right away (main waits for it)
        import contextlib
        orig = SINK.producer

        # DIAG_CONCURRENT=<substring>: jobs whose submitting frame matches
        # stay concurrent, every other job is joined right away
        conc = os.environ.get("DIAG_CONCURRENT", "")

        @contextlib.contextmanager
        def producer(dev, *keep):
            import inspect
            # the autograd backward that submitted this job: its first line
            # identifies the op kind (hip_impl _Conv / _Linear / ...)
            f = inspect.currentframe()
            kind = ""
            while f is not None:
                if f.f_code.co_name == "backward":
                    kind = f"{os.path.basename(f.f_code.co_filename)}:{f.f_code.co_firstlineno}"
                    break
                f = f.f_back
            KINDS.add(kind)
            with orig(dev, *keep):
                yield
            if conc and conc == kind:
                return
            if SINK.stream_enabled and dev.type == "cuda" and dev.index in SINK._streams:
                torch.cuda.current_stream().wait_stream(SINK._streams[dev.index])
        SINK.producer = producer
        SINK._diag_patched = True
    X._COND_STREAM = cond
    Gm._DEFER_UPDATE = defer
    torch.manual_seed(0)
    ctx = DistContext(device=torch.device("cuda", 0))
    cfg = make_config(None, {"model.H": 64, "model.W": 64, "data.imgsize": 64, "global_batch": 16,
                             "micro_batch": 0, "data.synthetic": True, "log_every": 0, "ckpt_every": 0,
                             "graph": graph, "optim.warmup_examples": 32})
    tr = Trainer(cfg, ctx)
    names = [n for n, _ in tr.model.named_parameters()]
    sums = []          # (module name, device checksum) of every forward output, in call order
    gsums = []         # (module name, device checksum) of every output GRADIENT, in backward order
    if os.environ.get("DIAG_GSUMS", "0") == "1":
        def fhook(mod, i, o, n=None):
            o = o[0] if isinstance(o, (tuple, list)) else o
            if torch.is_tensor(o) and o.requires_grad:
                o.register_hook(lambda g, n=n: gsums.append((n, g.detach().double().abs().sum())))
        for n, m in tr.model.named_modules():
            if n.count(".") <= 4 and n:
                m.register_forward_hook(lambda mod, i, o, n=n: fhook(mod, i, o, n))
    if CHECKSUMS:
        def hook(mod, i, o, n=None):
            o = o[0] if isinstance(o, (tuple, list)) else o
            if torch.is_tensor(o) and o.is_floating_point():
                sums.append((n, o.detach().double().abs().sum()))
        for n, m in tr.model.named_modules():
            if n.count(".") <= 3 and n:
                m.register_forward_hook(lambda mod, i, o, n=n: hook(mod, i, o, n))
    assert len(names) == len(tr.flat.params)
    grads, losses = [], []
    # how often a residual-gradient hand-off found its GroupNorm already run
    # (ops.hip_impl.ResGradSlot: the two paths round differently)
    from distributed_3d_diffusion_pytorch_amd.ops import hip_impl as Hm
    slot_log = []
    if not hasattr(Hm.ResGradSlot, "_diag_orig"):
        Hm.ResGradSlot._diag_orig = Hm.ResGradSlot.deposit

        def deposit(self, g, scale=1.0):
            ok = Hm.ResGradSlot._diag_orig(self, g, scale)
            SLOTS.append(ok)
            return ok
        Hm.ResGradSlot.deposit = deposit
    SLOTS.clear()
    if not graph:
        # eager: the gradient is consumed by the optimizer inside train_step;
        # snapshot it (after a full device sync) right before the update
        ostep = tr.optim.step

        def step(*a, **k):
            torch.cuda.synchronize()
            grads.append(tr.flat.grad.clone())
            return ostep(*a, **k)
        tr.optim.step = step
    for b in batches:
        losses.append(tr.train_step(*b).item())
        torch.cuda.synchronize()
        if graph:
            grads.append(tr.flat.grad.clone())      # deferred: still live until the next replay
    tr.sync()
    torch.cuda.synchronize()
    out = dict(slots="".join("1" if v else "0" for v in SLOTS), losses=losses, grads=grads, sums=[(n, float(v)) for n, v in sums],
               gsums=[(n, float(v)) for n, v in gsums], p=tr.flat.data.clone(), m=tr.optim.exp_avg.clone(),
               v=tr.optim.exp_avg_sq.clone(), spans=[(tr.flat.offsets[i], tr.flat.params[i].numel())
                                                    for i in range(len(names))] if hasattr(tr.flat, "offsets")
               else None, names=names)
    hip_impl.set_device_seed(None)
    del tr
    torch.cuda.empty_cache()
    return out


def where(flat_diff, tr_spans, names, top=6):
    rows = []
    for (off, n), name in zip(tr_spans, names):
        d = flat_diff[off:off + n]
        mx = d.max().item()
        if mx > 0:
            rows.append((off, mx, int((d > 0).sum().item()), name))
    # flat order is backward (deposit) order: the first differing parameters
    # are the ones closest to where the difference entered the backward
    rows.sort()
    first = [(r[3], r[2], f"{r[1]:.1e}") for r in rows[:top]]
    return first, len(rows)


def main():
    variants = (sys.argv[1] if len(sys.argv) > 1 else "g:scd,g:scd").split(",")
    from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches
    data = SyntheticBatches(16, 64, "cuda", seed=33)
    batches = [next(data) for _ in range(6)]
    for i in range(0, len(variants) - 1, 2):
        va, vb = variants[i], variants[i + 1]
        ra, r = [run(v[0] == "g", "s" in v[2:], batches, "c" in v[2:], "d" in v[2:]) for v in (va, vb)]
        ref = ra
        spans = ref["spans"]
        print(f"== {va} vs {vb}: losses equal {ref['losses'] == r['losses']}", flush=True)
        print(f"   slot hand-offs equal: {ref['slots'] == r['slots']} (refused: {ref['slots'].count('0')} vs "
              f"{r['slots'].count('0')} of {len(ref['slots'])})", flush=True)
        if ref["gsums"]:
            per = len(ref["gsums"]) // len(batches)
            diff = [(k // per, k % per, a[0]) for k, (a, b) in enumerate(zip(ref["gsums"], r["gsums"]))
                    if a[1] != b[1]]
            print(f"   output gradients: {len(ref['gsums'])} recorded ({per}/step), {len(diff)} differ; "
                  f"first (step, index, module) {diff[:8]}", flush=True)
        if ref["sums"]:
            diff = [(k, a[0]) for k, (a, b) in enumerate(zip(ref["sums"], r["sums"])) if a[1] != b[1]]
            print(f"   forward outputs: {len(ref['sums'])} recorded, {len(diff)} differ; first {diff[:5]}",
                  flush=True)
        for k in ("p", "m", "v"):
            d = (ref[k] - r[k]).abs()
            rows, n = where(d, spans, ref["names"])
            print(f"   {k}: {n} params differ; top {rows}", flush=True)
        for s, (ga, gb) in enumerate(zip(ref["grads"], r["grads"])):
            d = (ga - gb).abs()
            rows, n = where(d, spans, ref["names"])
            # relative size: |difference| against the gradient's own magnitude
            rel = []
            for name, cnt, mx in rows[:4]:
                i = ref["names"].index(name)
                off, numel = spans[i]
                rel.append(f"{name}: |g|max {ga[off:off + numel].abs().max().item():.1e}")
            print(f"   step {s} grad: {n} params differ; top {rows}; {rel}", flush=True)


if __name__ == "__main__":
    main()
    print("job kinds:", sorted(KINDS))
