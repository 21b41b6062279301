"""Stochastic-conditioning CFG ancestral sampler (reference:
`sampling.py:78-184`, `train.py:118-166`).

Differences by design (same math, §2.5 of SURVEY):
* everything stays on the device (the reference moves eps to the CPU and does
  the posterior there, two host syncs per step, D11);
* the conditional and unconditional CFG passes run as ONE 2b-batch forward;
* randomness is counter-based in (seed, step, GLOBAL chain index, element)
  (the hash of ops/csrc/common.h, mirrored bit-for-bit in ops.torch_impl):
  a chain draws the same noise whatever batch or rank it runs in, so
  multi-GPU sampling -- the b guidance-scale chains sharded over ranks, one
  process per GPU, instead of ``nn.DataParallel`` replicating 521 MiB of
  weights on every forward (`sampling.py:52`) -- reproduces the single-GPU
  result; the record-choice RNG is seeded identically on every rank so all
  shards condition on the same view;
* on the HIP path the whole step (CFG input assembly with the unconditional
  noise -> 2b X-UNet forward -> fused CFG combine / x0 clamp / posterior /
  noise, `sampler_step2_k`) is captured ONCE in a HIP graph and replayed for
  all 256 steps: the per-step scalars come from a device table row and the
  step's RNG word from a device word, the stochastic-conditioning choice is a
  device-to-device copy into the graph's static input before each replay;
* all b chains of a step condition on the same (record view, target view)
  poses and logSNR pair, so the conditioning is computed for the 2 distinct
  classes (cond / uncond) only -- 4 conditioning images instead of 4b -- and
  shared by the GN-FiLM kernels through a row -> class map
  (``XUNet.forward(shared_cond=)``; ``share_cond=False`` restores the
  per-example forward);
* D9 (noise skipped at t=0.5 where logsnr_next == 0) is opt-in via
  ``ref_quirk``; default adds noise on every step but the last.
"""
from __future__ import annotations

import math
import random
from typing import List, Optional, Tuple

import torch

from ..diffusion import logsnr_schedule_cosine, sampler_logsnrs, cfg_posterior

_M64 = (1 << 64) - 1
_GOLDEN = 0x9E3779B97F4A7C15


class RecordEntry:
    """One conditioning candidate: images [b,3,H,W] (per-chain), R [3,3], T [3]."""

    def __init__(self, img: torch.Tensor, R: torch.Tensor, T: torch.Tensor):
        self.img, self.R, self.T = img, R, T


class DiffusionSampler:
    def __init__(self, model: torch.nn.Module, timesteps: int = 256, ref_quirk: bool = False,
                 logsnr_min: float = -20.0, logsnr_max: float = 20.0, seed: int = 0, device=None,
                 chain_offset: int = 0, graph: Optional[bool] = None, share_cond: bool = True):
        """``chain_offset``: global index of this sampler's first chain (its
        rank's shard start).  ``graph``: replay the step from a HIP graph
        (default: on for the bf16 HIP path).  ``share_cond``: compute the
        conditioning once per class instead of once per chain in
        :meth:`sample` (identical result)."""
        self.share_cond = bool(share_cond)
        self.model = model
        self.T = timesteps
        self.ref_quirk = ref_quirk
        self.lmin, self.lmax = logsnr_min, logsnr_max
        self.device = device or next(model.parameters()).device
        self.seed_base = (int(seed) * 0x2545F4914F6CDD1D + 0x5DEECE66D) & _M64
        self.c0 = int(chain_offset)
        self.choice_rng = random.Random(seed)
        lam, lam_next = sampler_logsnrs(timesteps, logsnr_min, logsnr_max)
        self.lam, self.lam_next = lam.tolist(), lam_next.tolist()
        self.lam0 = float(logsnr_schedule_cosine(torch.zeros(()), logsnr_min=logsnr_min, logsnr_max=logsnr_max))
        self.graph = graph
        self._g = None

    # ------------------------------------------------------------ scalars
    def step_seed(self, k: int) -> int:
        return (self.seed_base + (k + 1) * _GOLDEN) & _M64

    def add_noise(self, k: int) -> bool:
        return (self.lam_next[k] != 0.0) if self.ref_quirk else (k < self.T - 1)

    def params(self, k: int) -> List[float]:
        """[lambda, alpha, sigma, alpha_next, c, sqrt(var), add_noise, lambda0]
        (the device block of sampler_inputs_k / sampler_step2_k)."""
        lam, lam_next = self.lam[k], self.lam_next[k]
        sig = lambda x: 1.0 / (1.0 + math.exp(-x))  # noqa: E731
        c = -math.expm1(lam - lam_next)
        return [lam, math.sqrt(sig(lam)), math.sqrt(sig(-lam)), math.sqrt(sig(lam_next)), c,
                math.sqrt(sig(-lam_next) * c), 1.0 if self.add_noise(k) else 0.0, self.lam0]

    def _hip(self, z: torch.Tensor) -> bool:
        from .. import ops
        return z.is_cuda and getattr(self.model, "compute_dtype", None) == torch.bfloat16 and \
            ops.use_hip(z, any_dtype=True)

    # ---------------------------------------------------- counter noise
    def _noise(self, key: int, k: Optional[int], shape, device) -> torch.Tensor:
        """N(0,1) [b, ...] for this sampler's chains: element (j, i) is
        normal01(seed ^ key, (c0 + j) * D + i)."""
        from ..ops import torch_impl as TI
        s = (self.seed_base if k is None else self.step_seed(k)) ^ key
        D = int(torch.Size(shape[1:]).numel())
        if device.type == "cuda":
            from .. import ops
            if ops.use_hip(torch.empty(0, device=device), any_dtype=True):
                from ..ops import hip_impl
                return hip_impl.randn_hash(shape, s, self.c0 * D, device)
        idx = torch.arange(int(torch.Size(shape).numel()), device=device, dtype=torch.int64) + self.c0 * D
        return TI.normal01(s, idx).reshape(shape)

    # ------------------------------------------------ shared conditioning
    @staticmethod
    def shared_cond(R1, T1, K1, logsnr: torch.Tensor, b: int) -> dict:
        """The 2 distinct conditioning examples of a CFG batch whose b chains
        share one pose pair: class 0 conditional, class 1 unconditional
        (rays masked).  R1 [2,3,3], T1 [2,3], K1 [3,3], logsnr [2,2] (or a
        view of any 2 rows of the batch's identical [lambda0, lambda] rows)."""
        dev = R1.device
        return {"R": R1[None].expand(2, 2, 3, 3), "t": T1[None].expand(2, 2, 3),
                "K": K1.reshape(1, 3, 3).expand(2, 3, 3), "logsnr": logsnr,
                "cond_mask": torch.tensor([True, False], device=dev),
                "example_class": torch.cat([torch.zeros(b, dtype=torch.int32, device=dev),
                                            torch.ones(b, dtype=torch.int32, device=dev)])}

    # ------------------------------------------------------- eager step
    @torch.no_grad()
    def denoise_eps(self, x_cond, z, R, T, K, logsnr: float, k: int = 0, shared: bool = False):
        """CFG pair in one forward: rows [0,b) conditional, [b,2b) unconditional
        (x replaced by the step-k counter-based noise, rays zeroed via
        cond_mask=False).  ``shared``: R/T/K are the same for every chain
        (as in :meth:`sample`): condition once per class."""
        from ..ops import torch_impl as TI
        b = z.shape[0]
        dev = z.device
        x_unc = self._noise(TI.K_XU, k, tuple(x_cond.shape), dev).to(x_cond.dtype)
        lam = torch.full((2 * b,), float(logsnr), device=dev)
        logsnr2 = torch.stack([torch.full_like(lam, self.lam0), lam], 1)
        batch = {"x": torch.cat([x_cond, x_unc]), "z": torch.cat([z, z])}
        if shared:
            eps = self.model(batch, shared_cond=self.shared_cond(R[0], T[0], K[0], logsnr2[:2], b)).float()
        else:
            batch.update({"logsnr": logsnr2, "R": torch.cat([R, R]), "t": torch.cat([T, T]),
                          "K": torch.cat([K, K])})
            mask = torch.cat([torch.ones(b, dtype=torch.bool, device=dev),
                              torch.zeros(b, dtype=torch.bool, device=dev)])
            eps = self.model(batch, cond_mask=mask).float()
        return eps[:b], eps[b:]

    @torch.no_grad()
    def step(self, z, x_cond, R, T, K, w, k: int, shared: bool = False):
        """One ancestral CFG step for b chains.  ``shared``: every chain has
        the same R/T/K (conditioning computed once per class)."""
        from ..ops import torch_impl as TI
        if self._hip(z):
            return self._hip_step(z, x_cond, R, T, K, w, k, shared)
        eps_c, eps_u = self.denoise_eps(x_cond, z, R, T, K, self.lam[k], k, shared)
        mean, var = cfg_posterior(z, eps_c, eps_u, w, torch.tensor(self.lam[k]), torch.tensor(self.lam_next[k]))
        if not self.add_noise(k):
            return mean
        return mean + var.sqrt() * self._noise(TI.K_NZ, k, tuple(z.shape), z.device)

    @torch.no_grad()
    def _hip_step(self, z, x_cond, R, T, K, w, k, shared=False):
        """Eager form of the graphed step (same kernels, host seed)."""
        from ..ops import hip_impl
        b, _, H, W = z.shape
        dev = z.device
        prm = torch.tensor(self.params(k), dtype=torch.float32).to(dev)
        xz = torch.empty(4 * b, H, W, 8, dtype=torch.bfloat16, device=dev)
        logsnr = torch.empty(2 * b, 2, dtype=torch.float32, device=dev)
        z = z.float().contiguous().clone()
        hip_impl.sampler_inputs(x_cond.float().contiguous(), z, prm, None, self.step_seed(k), self.c0, xz, logsnr)
        if shared:
            sc = self.shared_cond(R[0].float(), T[0].float(), K[0].float(), logsnr[:2], b)
            y = self.model({"xz": xz}, shared_cond=sc, head_nhwc=True)
        else:
            mask = torch.cat([torch.ones(b, dtype=torch.bool, device=dev),
                              torch.zeros(b, dtype=torch.bool, device=dev)])
            batch = {"xz": xz, "logsnr": logsnr, "R": torch.cat([R, R]), "t": torch.cat([T, T]),
                     "K": torch.cat([K, K])}
            y = self.model(batch, cond_mask=mask, head_nhwc=True)
        hip_impl.sampler_step2(z, y, w.float().contiguous(), prm, None, self.step_seed(k), self.c0)
        return z

    # ------------------------------------------------------ graph step
    def _graph_setup(self, b: int, H: int, W: int, K: torch.Tensor, w: torch.Tensor, target_R, target_T):
        from ..ops import hip_impl
        dev = self.device
        g = {"b": b, "H": H, "W": W}
        g["xc"] = torch.zeros(b, 3, H, W, device=dev)
        g["z"] = torch.zeros(b, 3, H, W, device=dev)
        shared = g["shared"] = self.share_cond
        nb = 1 if shared else 2 * b                 # pose rows the graph reads
        g["R"] = torch.zeros(nb, 2, 3, 3, device=dev)
        g["t"] = torch.zeros(nb, 2, 3, device=dev)
        g["R"][:, 1] = target_R.to(dev).float()
        g["t"][:, 1] = target_T.to(dev).float()
        g["K"] = K.to(dev).float().reshape(1, 3, 3).expand(nb, 3, 3).contiguous()
        g["w"] = w.to(dev).float().contiguous()
        g["prm_table"] = torch.tensor([self.params(k) for k in range(self.T)], dtype=torch.float32).to(dev)
        g["prm"] = g["prm_table"][0].clone()
        g["sd"] = torch.zeros(3, dtype=torch.int64, device=dev)
        g["xz"] = torch.empty(4 * b, H, W, 8, dtype=torch.bfloat16, device=dev)
        g["logsnr"] = torch.empty(2 * b, 2, dtype=torch.float32, device=dev)
        g["mask"] = torch.cat([torch.ones(b, dtype=torch.bool, device=dev),
                               torch.zeros(b, dtype=torch.bool, device=dev)])
        g["target"] = (target_R.detach().clone(), target_T.detach().clone(), K.detach().clone(), w.detach().clone())

        if shared:
            g["sc"] = self.shared_cond(g["R"][0], g["t"][0], g["K"][0], g["logsnr"][:2], b)

        def body():
            hip_impl.sampler_inputs(g["xc"], g["z"], g["prm"], g["sd"], self.seed_base, self.c0, g["xz"],
                                    g["logsnr"])
            if shared:
                y = self.model({"xz": g["xz"]}, shared_cond=g["sc"], head_nhwc=True)
            else:
                batch = {"xz": g["xz"], "logsnr": g["logsnr"], "R": g["R"], "t": g["t"], "K": g["K"]}
                y = self.model(batch, cond_mask=g["mask"], head_nhwc=True)
            hip_impl.sampler_step2(g["z"], y, g["w"], g["prm"], g["sd"], self.seed_base, self.c0)

        z_keep = g["z"].clone()
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.no_grad(), torch.cuda.stream(s):
            for _ in range(2):          # lazy init, weight caches, allocator warm-up
                body()
        torch.cuda.current_stream(dev).wait_stream(s)
        hip_impl.refresh_weights()
        torch.cuda.synchronize(dev)
        graph = torch.cuda.CUDAGraph()
        from .graphs import _gc_paused            # (no collection finalising old graphs mid-capture)
        with torch.no_grad(), _gc_paused(), torch.cuda.graph(graph):
            body()
        torch.cuda.synchronize(dev)
        g["z"].copy_(z_keep)
        g["graph"] = graph
        g["weights"] = self._weight_signature()
        self._g = g
        return g

    def _weight_signature(self):
        """The captured graph reads the cached bf16 weight operands by address:
        any out-of-place change (``load_state_dict`` / ``copy_`` bump the
        parameters' versions and the cache rebuilds the operand in a new
        buffer) must force a recapture."""
        from ..ops import hip_impl
        return (hip_impl._REV[0], tuple(p._version for p in self.model.parameters()))

    def _graph_ok(self, b, H, W, K, w, target_R, target_T) -> bool:
        g = self._g
        if g is None or g["b"] != b or g["H"] != H or g["W"] != W or g["shared"] != self.share_cond:
            return False
        if g["weights"] != self._weight_signature():
            return False
        tR, tT, tK, tw = g["target"]
        return bool(torch.equal(tK.to(K.device), K) and torch.equal(tw.to(w.device), w))

    # ----------------------------------------------------------- sample
    @torch.no_grad()
    def sample(self, record: List[RecordEntry], target_R: torch.Tensor, target_T: torch.Tensor,
               K: torch.Tensor, w: torch.Tensor, progress: bool = False) -> torch.Tensor:
        """Generate the view at (target_R, target_T) for each of the b chains;
        each step conditions on a random entry of ``record`` (stochastic
        conditioning, `sampling.py:137-145`)."""
        from ..ops import torch_impl as TI
        model_was_training = self.model.training
        self.model.eval()
        b = w.shape[0]
        dev = self.device
        H, W = record[0].img.shape[-2:]
        z = self._noise(TI.K_Z0, None, (b, 3, H, W), dev)
        Kb = K.to(dev).reshape(1, 3, 3).expand(b, 3, 3).contiguous()
        w = w.to(dev).float()
        it = range(self.T)
        if progress:
            try:
                from tqdm import tqdm
                it = tqdm(it, desc="diffusion", leave=False)
            except Exception:
                pass
        use_graph = self._hip(z) and (self.graph is None or self.graph)
        if use_graph:
            if not self._graph_ok(b, H, W, K.to(dev), w, target_R, target_T):
                self._graph_setup(b, H, W, K, w, target_R, target_T)
            g = self._g
            g["R"][:, 1] = target_R.to(dev).float()
            g["t"][:, 1] = target_T.to(dev).float()
            g["z"].copy_(z)
            for k in it:
                e = record[self.choice_rng.randrange(len(record))]
                g["xc"].copy_(e.img)
                g["R"][:, 0] = e.R.to(dev).float()
                g["t"][:, 0] = e.T.to(dev).float()
                g["prm"].copy_(g["prm_table"][k])
                g["sd"][0].fill_(k + 1)
                g["graph"].replay()
            z = g["z"].clone()
        else:
            for k in it:
                e = record[self.choice_rng.randrange(len(record))]
                R = torch.stack([e.R.to(dev), target_R.to(dev)], 0)[None].expand(b, 2, 3, 3).contiguous()
                T = torch.stack([e.T.to(dev), target_T.to(dev)], 0)[None].expand(b, 2, 3).contiguous()
                z = self.step(z, e.img.to(dev), R, T, Kb, w, k, shared=self.share_cond)
        if model_was_training:
            self.model.train()
        return z


def shard_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous, disjoint, covering split of n chains over ranks."""
    base, rem = divmod(n, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)
