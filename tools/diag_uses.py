import os, sys, collections
sys.path.insert(0, "/root/repo")
import torch
from distributed_3d_diffusion_pytorch_amd.config import make_config
from distributed_3d_diffusion_pytorch_amd.engine import Trainer
from distributed_3d_diffusion_pytorch_amd.parallel import DistContext
from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches
from distributed_3d_diffusion_pytorch_amd.ops.gradsink import SINK
dev = torch.device("cuda", 0)
ctx = DistContext(device=dev)
cfg = make_config(None, {"model.H": 64, "model.W": 64, "data.imgsize": 64, "global_batch": 16, "micro_batch": 0,
                         "data.synthetic": True, "log_every": 0, "ckpt_every": 0, "graph": False})
tr = Trainer(cfg, ctx)
names = {id(p): n for n, p in tr.model.named_parameters()}
auto = collections.Counter()
for n, p in tr.model.named_parameters():
    p.register_hook(lambda g, n=n: auto.update([n]) if g is not None else None)
uses = collections.Counter(); dones = collections.Counter()
ou, od = SINK.use, SINK.done
def use(p, needed=True):
    if needed and SINK.managed(p): uses[names.get(id(p), "?")] += 1
    return ou(p, needed)
def done(p):
    if SINK.managed(p): dones[names.get(id(p), "?")] += 1
    return od(p)
SINK.use, SINK.done = use, done
b = next(SyntheticBatches(16, 64, "cuda", seed=3))
tr.train_step(*b)
torch.cuda.synchronize()
print("params with >1 use:", [(k, v) for k, v in uses.items() if v > 1])
print("n params", len(names), "n autograd-grad params", len(auto))
print("params with autograd grads:", dict(auto))
print("use/done mismatch:", [(k, uses[k], dones[k]) for k in set(uses) | set(dones) if uses[k] != dones[k]])
print("params never deposited:", [n for n in names.values() if n not in dones and n not in auto][:20])
