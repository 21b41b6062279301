"""X-UNet denoiser (3DiM), MI355X-native NHWC execution.

Capability parity with the reference X-UNet (`xunet.py:355-536`): identical
module tree / parameter names / shapes / init (so `state_dict`s -- and the
reference's Adam state, indexed by ``model.parameters()`` order -- load
unchanged; Appendix A of SURVEY.md), identical math.  The execution is
re-designed:

* activations are ``[2B, H, W, C]`` (frames folded into the batch,
  channels-last) in the compute dtype (bf16 on MI355X), parameters stay fp32
  masters; every op goes through :mod:`..ops`, which dispatches to the gfx950
  HIP kernels (implicit-GEMM MFMA conv3x3, fused GN/SiLU, fused GN+FiLM+dropout,
  flash-style cross-view attention, on-device ray/posenc) or to the torch oracle;
* camera rays are generated on device (the reference round-trips through numpy
  on the host every forward, `xunet.py:311-318`);
* ``silu(logsnr_emb + pose_emb_i)`` is computed once per resolution level and
  shared by all FiLM layers of that level, whose projections run as one GEMM
  (the reference recomputes the SiLU in every FiLM, `xunet.py:84`);
* the output head runs on frame 1 only (the reference computes both frames and
  discards frame 0, `xunet.py:535-536`).
"""
from __future__ import annotations

import math
import os
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn as nn

from .. import ops
from ..config import ModelConfig

INV_SQRT2 = 1.0 / math.sqrt(2.0)


_COND_STREAM = os.environ.get("D3D_COND_STREAM", "1") != "0"
# AttnBlock: out_proj + the 1x1 `linear` as one merged map (ops.attn_out); 0: two layers
_ATTN_MERGE = os.environ.get("D3D_ATTN_MERGE", "1") != "0"
# conditioning stream: one FiLM GEMM + ready event per block instead of one per level
FILM_BLOCK_EVENTS = False        # measured -1.2 % at bs16 and bs128 (profiles/r3/ab_film_events_s64.txt)
_COND_STREAMS: Dict[int, "torch.cuda.Stream"] = {}
# (level, event): parameters outside the early update part become valid at
# `event` -- the trunk waits on it before encoder level `level` and the
# conditioning stream before that level's FiLM projections (deferred,
# overlapped optimizer step of the graph-replayed training step,
# engine/graphs.py).  Set only around that step's forward.
PARAM_FENCE: List = [None]


class GroupNorm(nn.Module):
    """GroupNorm(32) applied per (example, frame) image (`xunet.py:61-71`)."""

    def __init__(self, num_groups: int = 32, num_channels: int = 64):
        super().__init__()
        self.gn = nn.GroupNorm(num_groups=num_groups, num_channels=num_channels)

    def forward(self, h: torch.Tensor, silu: bool = False, res_slot=None) -> torch.Tensor:
        return ops.group_norm(h, self.gn.weight, self.gn.bias, self.gn.num_groups, self.gn.eps, silu, res_slot)


class FiLM(nn.Module):
    """FiLM projection ``dense(silu(emb)) -> [scale | shift]`` (`xunet.py:74-87`).
    ``forward`` takes the per-level (pre-activation) embedding and returns the
    packed ``[N, H, W, 2C]`` modulation; the modulation itself is fused into the
    GroupNorm kernel (:func:`ops.gn_film`).  The level-batched path
    (:func:`ops.film_batch`) runs every FiLM of a level as one GEMM."""

    def __init__(self, features: int, emb_ch: int = 1024):
        super().__init__()
        self.features = features
        self.dense = nn.Linear(emb_ch, 2 * features)

    def forward(self, emb: torch.Tensor) -> torch.Tensor:
        return ops.linear(ops.silu(emb), self.dense.weight, self.dense.bias)


class ResnetBlock(nn.Module):
    """BigGAN ResBlock over frames (`xunet.py:90-152`):
    ``GN0 -> SiLU -> conv3x3 -> GN1 -> FiLM -> dropout -> conv3x3 (+ 1x1 skip)
    -> /sqrt2 -> avgpool|nearest-up``."""

    def __init__(self, in_features: int, out_features: Optional[int] = None, dropout: float = 0.0,
                 resample: Optional[str] = None, emb_ch: int = 1024):
        super().__init__()
        out_features = in_features if out_features is None else out_features
        self.in_features = in_features
        self.features = out_features
        self.dropout_p = float(dropout)
        if resample not in (None, "up", "down"):
            raise ValueError(resample)
        self.resample = resample
        # Registration order mirrors the reference so parameters() order (and
        # therefore optimizer-state indices) is identical.
        self.groupnorm0 = GroupNorm(num_channels=in_features)
        self.groupnorm1 = GroupNorm(num_channels=out_features)
        self.conv1 = nn.Conv2d(in_features, out_features, kernel_size=3, stride=1, padding=1)
        self.film = FiLM(out_features, emb_ch)
        self.conv2 = nn.Conv2d(out_features, out_features, kernel_size=3, stride=1, padding=1)
        if in_features != out_features:
            self.dense = nn.Conv2d(in_features, out_features, kernel_size=1)
        nn.init.zeros_(self.conv2.weight)
        self._seed_slot = 0

    def forward(self, x, semb: torch.Tensor) -> torch.Tensor:
        skip = slot = None
        fused = None
        if isinstance(x, tuple):
            # decoder: x is the skip concatenation [h | hs] (xunet.py:521-531),
            # never materialised -- GN0 and the 1x1 skip read both halves
            a, b = x
            assert a.shape[-1] + b.shape[-1] == self.in_features and self.in_features != self.features
            h, skip = ops.cat_gn_silu_dense(a, b, self.groupnorm0.gn.weight, self.groupnorm0.gn.bias,
                                            self.dense.weight, self.dense.bias, self.groupnorm0.gn.num_groups,
                                            self.groupnorm0.gn.eps)
        else:
            N, H, W, C = x.shape
            assert C == self.in_features, (C, self.in_features)
            # x's two consumers here (GN0 and the residual / NIN branch) hand
            # their gradients over inside the GN0 backward kernel
            slot = ops.res_slot(x) if torch.is_grad_enabled() and x.requires_grad else None
            if slot is not None:
                # a decoder skip concat that also reads x deposits its gradient here (ops _CatGNDense)
                x._d3d_res_slot = slot
            # GN0 + SiLU inside conv1's input staging where the HIP conv takes it
            fused = ops.gn_silu_conv3x3(x, self.groupnorm0.gn.weight, self.groupnorm0.gn.bias, self.conv1.weight,
                                        self.conv1.bias, self.groupnorm0.gn.num_groups, self.groupnorm0.gn.eps,
                                        gn1_groups=self.groupnorm1.gn.num_groups, res_slot=slot)
            if fused is None:
                h = self.groupnorm0(x, silu=True, res_slot=slot)
        if fused is not None:
            h = fused
        else:
            # the conv epilogues also emit the partial statistics of the GroupNorm
            # that reads their output (GN1 here; the next block's GN0 below)
            h = ops.conv3x3(h, self.conv1.weight, self.conv1.bias, gn_groups=self.groupnorm1.gn.num_groups)
        ss = self.__dict__.pop("_ss", None)     # precomputed by the level-batched FiLM
        ev = self.__dict__.pop("_ss_event", None)
        if ev is not None:                      # ... on the conditioning stream: first read here
            torch.cuda.current_stream().wait_event(ev)
        if ss is None:
            ss = self.film(semb)
        # shared conditioning: ss holds one modulation per conditioning class,
        # image n reads class ss_map[n] (XUNet.forward(shared_cond=))
        ss_map = self.__dict__.get("_ss_map")
        h = ops.gn_film(h, self.groupnorm1.gn.weight, self.groupnorm1.gn.bias, ss,
                        self.groupnorm1.gn.num_groups, self.groupnorm1.gn.eps,
                        self.dropout_p, self.training, _next_seed(self), ss_map=ss_map)
        rslot = None
        if skip is not None:
            # decoder: conv2 deposits the skip's gradient in the NIN op's slot
            rslot = skip.__dict__.get("_d3d_out_slot")
        if skip is None:
            if self.in_features != self.features:
                skip = ops.linear(x, self.dense.weight, self.dense.bias, in_slot=slot)
            else:
                skip, rslot = x, slot
        h = ops.conv3x3(h, self.conv2.weight, self.conv2.bias, residual=skip, out_scale=INV_SQRT2,
                        gn_groups=self.groupnorm1.gn.num_groups if self.resample is None else 0, res_slot=rslot)
        if self.resample == "down":
            h = ops.avgpool2(h)
        elif self.resample == "up":
            h = ops.upsample2(h)
        return h


class AttnLayer(nn.Module):
    """Container of the reference's ``nn.MultiheadAttention`` parameters
    (`xunet.py:154-177`): packed ``in_proj`` and ``out_proj``."""

    def __init__(self, attn_heads: int = 4, in_channels: int = 32):
        super().__init__()
        self.in_channels = in_channels
        self.attn_heads = attn_heads
        self.attn = nn.MultiheadAttention(in_channels, attn_heads, batch_first=True)

    def core(self, hn: torch.Tensor, cross: bool) -> torch.Tensor:
        """q/k/v projection + multi-head attention, before out_proj."""
        qkv = ops.linear(hn, self.attn.in_proj_weight, self.attn.in_proj_bias)
        return ops.attention(qkv, self.attn_heads, cross)

    def forward(self, hn: torch.Tensor, cross: bool) -> torch.Tensor:
        return ops.linear(self.core(hn, cross), self.attn.out_proj.weight, self.attn.out_proj.bias)


class AttnBlock(nn.Module):
    """GN -> per-frame self / cross-frame MHA (shared weights for both frames)
    -> zero-init 1x1 -> (h + x)/sqrt2 (`xunet.py:179-220`)."""

    def __init__(self, attn_type: str, attn_heads: int = 4, in_channels: int = 32):
        super().__init__()
        if attn_type not in ("self", "cross"):
            raise NotImplementedError(attn_type)
        self.in_channels = in_channels
        self.attn_type = attn_type
        self.attn_heads = attn_heads
        self.groupnorm = GroupNorm(num_channels=in_channels)
        self.attn_layer = AttnLayer(attn_heads=attn_heads, in_channels=in_channels)
        self.linear = nn.Conv2d(in_channels, in_channels, kernel_size=1)
        nn.init.zeros_(self.linear.weight)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        N, H, W, C = x.shape
        assert C == self.in_channels
        slot = ops.res_slot(x) if torch.is_grad_enabled() and x.requires_grad else None
        hn = self.groupnorm(x, res_slot=slot).reshape(N, H * W, C)
        # the output feeds the next GroupNorm (the cross-attention block's, or
        # the next ResnetBlock's GN0): its statistics come out of this epilogue
        if _ATTN_MERGE:
            # out_proj and the 1x1 `linear` (no nonlinearity between them) as ONE map
            a = self.attn_layer.core(hn, cross=(self.attn_type == "cross"))
            op = self.attn_layer.attn.out_proj
            y = ops.attn_out(a, op.weight, op.bias, self.linear.weight, self.linear.bias,
                             residual=x.reshape(N, H * W, C), out_scale=INV_SQRT2, res_slot=slot,
                             gn_groups=self.groupnorm.gn.num_groups)
        else:
            o = self.attn_layer(hn, cross=(self.attn_type == "cross"))
            y = ops.linear(o, self.linear.weight, self.linear.bias, residual=x.reshape(N, H * W, C),
                           out_scale=INV_SQRT2, res_slot=slot, gn_groups=self.groupnorm.gn.num_groups)
        return ops.carry_gn_stats(y, y.reshape(N, H, W, C))


class XUNetBlock(nn.Module):
    """ResnetBlock [+ self-attn + cross-attn] (`xunet.py:222-256`)."""

    def __init__(self, in_channels: int, features: int, use_attn: bool = False, attn_heads: int = 4,
                 dropout: float = 0.0, emb_ch: int = 1024):
        super().__init__()
        self.in_channels = in_channels
        self.features = features
        self.use_attn = use_attn
        self.resnetblock = ResnetBlock(in_channels, features, dropout=dropout, emb_ch=emb_ch)
        if use_attn:
            self.attnblock_self = AttnBlock("self", attn_heads, features)
            self.attnblock_cross = AttnBlock("cross", attn_heads, features)

    def forward(self, x, semb: torch.Tensor) -> torch.Tensor:
        c = sum(t.shape[-1] for t in x) if isinstance(x, tuple) else x.shape[-1]
        assert c == self.in_channels, (c, self.in_channels)
        h = self.resnetblock(x, semb)
        if self.use_attn:
            h = self.attnblock_self(h)
            h = self.attnblock_cross(h)
        return h


class ConditioningProcessor(nn.Module):
    """logSNR embedding MLP + camera-ray conditioning (`xunet.py:259-352`).

    Returns the per-level embeddings ``logsnr_emb + pose_emb_i`` as
    ``[2B, H_i, W_i, emb_ch]`` tensors; FiLM applies the SiLU (`xunet.py:84`),
    fused into its projection's GEMM."""

    D = 144

    def __init__(self, emb_ch: int, H: int, W: int, num_resolutions: int, use_pos_emb: bool = True,
                 use_ref_pose_emb: bool = True, rescale_intrinsics: bool = False):
        super().__init__()
        self.emb_ch = emb_ch
        self.H, self.W = H, W
        self.num_resolutions = num_resolutions
        self.use_pos_emb = use_pos_emb
        self.use_ref_pose_emb = use_ref_pose_emb
        self.rescale_intrinsics = rescale_intrinsics
        D = self.D
        self.logsnr_emb_emb = nn.Sequential(nn.Linear(emb_ch, emb_ch), nn.SiLU(), nn.Linear(emb_ch, emb_ch))
        if use_pos_emb:
            self.pos_emb = nn.Parameter(torch.zeros(D, H, W))
            nn.init.normal_(self.pos_emb, std=1.0 / np.sqrt(D))
        if use_ref_pose_emb:
            self.first_emb = nn.Parameter(torch.zeros(1, 1, D, 1, 1))
            nn.init.normal_(self.first_emb, std=1.0 / np.sqrt(D))
            self.other_emb = nn.Parameter(torch.zeros(1, 1, D, 1, 1))
            nn.init.normal_(self.other_emb, std=1.0 / np.sqrt(D))
        self.convs = nn.ModuleList([
            nn.Conv2d(D, emb_ch, kernel_size=3, stride=2 ** i, padding=1) for i in range(num_resolutions)])

    def logsnr_embedding(self, logsnr: torch.Tensor, dtype: Optional[torch.dtype] = None) -> torch.Tensor:
        """[B, 2] logSNR -> [2B, emb_ch] fp32 (clip +-20, DDPM posenc x1000, MLP;
        one fused HIP op in bf16 GPU runs)."""
        l0, act, l1 = self.logsnr_emb_emb
        return ops.logsnr_mlp(logsnr, l0.weight, l0.bias, l1.weight, l1.bias, max_time=1.0, dtype=dtype)

    def learned_embedding_image(self, dtype: torch.dtype) -> Optional[torch.Tensor]:
        """The learned part of the 144-ch conditioning input, identical for
        every example of a given frame: ``[2, H, W, 144]`` with image f =
        pos_emb + (first_emb if f == 0 else other_emb) (`xunet.py:333-336`)."""
        e = None
        if self.use_pos_emb:
            e = self.pos_emb.permute(1, 2, 0)[None].expand(2, self.H, self.W, self.D)
        if self.use_ref_pose_emb:
            fe = torch.cat([self.first_emb, self.other_emb], dim=1).reshape(2, 1, 1, self.D)
            e = fe.expand(2, self.H, self.W, self.D) if e is None else e + fe
        return None if e is None else e.to(dtype).contiguous()

    def forward(self, batch: Dict[str, torch.Tensor], cond_mask: torch.Tensor,
                dtype: torch.dtype) -> List[torch.Tensor]:
        return list(self.levels(batch, cond_mask, dtype))

    def levels(self, batch: Dict[str, torch.Tensor], cond_mask: torch.Tensor, dtype: torch.dtype):
        """:meth:`forward` as a generator: yields the embedding of level 0, 1,
        ... as soon as each is computed (the shared parts come first)."""
        B = batch["logsnr"].shape[0]
        assert cond_mask.shape == (B,), (cond_mask.shape, B)
        logsnr_emb = self.logsnr_embedding(batch["logsnr"], dtype)
        # Data-dependent part: NeRF-encoded camera rays (masked), no gradient.
        # A pinhole ray's origin is the camera centre, identical for every
        # pixel, so the 93 origin channels form a constant image per frame:
        # only the 51 direction channels go through the spatial conv, the
        # origin half enters as per-image tap biases (ops.cond_conv).
        mask = cond_mask.to(batch["R"].device).bool()
        rays_dir, orig_pe = ops.ray_conditioning(batch["R"], batch["t"], batch["K"], self.H, self.W, mask,
                                                 rescale_from=128 if self.rescale_intrinsics else 0, out_dtype=dtype)
        # Convolution is linear, so conv(rays + emb) = conv(rays) + conv(emb):
        # the learned term is convolved once per FRAME (2 images) and added as
        # a batch-broadcast residual.  Its input gradient (for pos_emb /
        # first_emb / other_emb) is then a 2-image transposed conv instead of a
        # per-example one.
        emb_img = self.learned_embedding_image(dtype)
        for i, conv in enumerate(self.convs):
            s = 2 ** i
            e_emb = ops.conv3x3(emb_img, conv.weight, None, stride=s) if emb_img is not None else None
            e = ops.cond_conv(rays_dir, orig_pe, conv.weight, conv.bias, s, row_bias=logsnr_emb, residual=e_emb,
                              res_period=2 if e_emb is not None else 0, silu_out=True)
            yield e


class XUNet(nn.Module):
    """The 2-frame X-UNet (`xunet.py:355-536`).  ``forward(batch, cond_mask=)``
    takes the reference's batch dict ``{x, z: [B,3,H,W], logsnr: [B,2],
    R: [B,2,3,3], t: [B,2,3], K: [B,3,3]}`` and returns eps-hat for frame 1,
    ``[B,3,H,W]``."""

    def __init__(self, cfg: Optional[ModelConfig] = None, **kwargs):
        super().__init__()
        cfg = cfg or ModelConfig()
        for k, v in kwargs.items():
            if not hasattr(cfg, k):
                raise TypeError(f"unknown XUNet option {k}")
            setattr(cfg, k, v)
        self.cfg = cfg
        self.H, self.W = cfg.H, cfg.W
        self.ch = cfg.ch
        self.ch_mult = tuple(cfg.ch_mult)
        self.num_res_blocks = cfg.num_res_blocks
        self.attn_resolutions = tuple(cfg.attn_resolutions)
        L = len(self.ch_mult)
        assert cfg.H % (2 ** (L - 1)) == 0 and cfg.W % (2 ** (L - 1)) == 0, \
            f"image size must be a multiple of {2 ** (L - 1)}"
        self.num_resolutions = L
        self.compute_dtype: Optional[torch.dtype] = None

        self.conditioningprocessor = ConditioningProcessor(
            cfg.emb_ch, cfg.H, cfg.W, L, cfg.use_pos_emb, cfg.use_ref_pose_emb, cfg.rescale_intrinsics)
        self.conv = nn.Conv2d(3, cfg.ch, kernel_size=3, stride=1, padding=1)
        self.dim_in = [cfg.ch] + [cfg.ch * m for m in self.ch_mult[:-1]]
        self.dim_out = [cfg.ch * m for m in self.ch_mult]
        kw = dict(dropout=cfg.dropout, attn_heads=cfg.attn_heads, emb_ch=cfg.emb_ch)

        self.xunetblocks = nn.ModuleList()
        for i in range(L):
            level = nn.ModuleList()
            for j in range(cfg.num_res_blocks):
                level.append(XUNetBlock(self.dim_in[i] if j == 0 else self.dim_out[i], self.dim_out[i],
                                        use_attn=i in self.attn_resolutions, **kw))
            if i != L - 1:
                level.append(ResnetBlock(self.dim_out[i], self.dim_out[i], dropout=cfg.dropout,
                                         resample="down", emb_ch=cfg.emb_ch))
            self.xunetblocks.append(level)

        self.middle = XUNetBlock(self.dim_out[-1], self.dim_out[-1], use_attn=L in self.attn_resolutions, **kw)

        self.upsample = nn.ModuleDict()
        for i in reversed(range(L)):
            level = nn.ModuleList()
            for j in range(cfg.num_res_blocks + 1):
                if j == 0:
                    prev_h = self.dim_out[i + 1] if i + 1 < L else self.dim_out[i]
                    skip = self.dim_out[i]
                elif j == cfg.num_res_blocks:
                    prev_h, skip = self.dim_out[i], self.dim_in[i]
                else:
                    prev_h, skip = self.dim_out[i], self.dim_out[i]
                level.append(XUNetBlock(prev_h + skip, self.dim_out[i], use_attn=i in self.attn_resolutions, **kw))
            if i != 0:
                level.append(ResnetBlock(self.dim_out[i], self.dim_out[i], dropout=cfg.dropout,
                                         resample="up", emb_ch=cfg.emb_ch))
            self.upsample[str(i)] = level

        self.lastgn = GroupNorm(num_channels=cfg.ch)
        self.lastconv = nn.Conv2d(cfg.ch, 3, kernel_size=3, stride=1, padding=1)
        nn.init.zeros_(self.lastconv.weight)

        # deterministic per-block dropout seed slots
        for idx, m in enumerate(mm for mm in self.modules() if isinstance(mm, ResnetBlock)):
            m._seed_slot = idx
        self._dropout_seed = 0
        self.batch_film = True

    def _film_groups(self):
        """ResnetBlocks grouped by the conditioning level whose embedding
        their FiLM consumes (mirrors the routing in forward)."""
        if self.__dict__.get("_fg") is None:
            L = self.num_resolutions
            groups = [[] for _ in range(L)]
            for i in range(L):
                for blk in self.xunetblocks[i]:
                    groups[i].append(blk.resnetblock if isinstance(blk, XUNetBlock) else blk)
                for blk in self.upsample[str(i)]:
                    groups[i].append(blk.resnetblock if isinstance(blk, XUNetBlock) else blk)
            groups[L - 1].append(self.middle.resnetblock)
            self.__dict__["_fg"] = groups
        return self.__dict__["_fg"]

    # -- dropout seeding: every forward gets a fresh base seed (set by the
    # trainer from its step counter) so HIP dropout masks are reproducible and
    # regenerated (not stored) in backward.
    def set_dropout_seed(self, seed: int) -> None:
        for m in self.modules():
            if isinstance(m, ResnetBlock):
                m._base_seed = int(seed)

    def forward(self, batch: Dict[str, torch.Tensor], *, cond_mask: Optional[torch.Tensor] = None,
                head_nhwc: bool = False, shared_cond: Optional[Dict[str, torch.Tensor]] = None) -> torch.Tensor:
        """``batch``: the reference dict {x, z, logsnr, R, t, K} (`xunet.py:477`),
        or with ``xz`` -- the already stacked NHWC stem input [2B,H,W,C>=3]
        (frames interleaved; extra channels zero) drawn by
        ``ops.diffusion_inputs`` -- in place of x and z.  ``head_nhwc``: return
        the head conv's NHWC output (channel-padded on the HIP path) for
        ``ops.diff_loss_nhwc`` instead of eps [B,3,H,W].

        ``shared_cond`` (inference only): when many examples share the same
        conditioning -- CFG sampling, where all b chains use the same poses
        and logSNR pair and differ only in cond / uncond -- pass the Bc
        DISTINCT conditioning examples ``{"logsnr": [Bc,2], "R", "t", "K",
        "cond_mask": [Bc], "example_class": [B] int}`` instead of per-example
        R/t/K/logsnr: the conditioning processor and the FiLM projections run
        on 2Bc images instead of 2B and the GN-FiLM kernels read the
        modulation of class ``example_class[n]``.  Same result as the
        per-example forward; removes ~38 % of the sampler's FLOPs at b=8."""
        if shared_cond is not None:
            return self._forward_shared(batch, shared_cond, head_nhwc)
        xz = batch.get("xz")
        if xz is not None:
            B = xz.shape[0] // 2
            H, W = xz.shape[1], xz.shape[2]
            xdt = xz.dtype
        else:
            x, z = batch["x"], batch["z"]
            B, C, H, W = x.shape
            xdt = x.dtype
        for key, v in batch.items():
            if key != "xz":
                assert v.shape[0] == B, f"{key} should have batch size {B}, not {v.shape[0]}"
        assert cond_mask is not None and cond_mask.shape[0] == B
        assert (H, W) == (self.H, self.W), ((H, W), (self.H, self.W))
        dt = self.compute_dtype or xdt
        cs = self._cond_stream(batch.get("xz", batch.get("x")))
        if cs is not None:
            return self._trunk(batch, None, B, H, W, dt, head_nhwc, None,
                               cond=(cs, batch, cond_mask))
        sembs = self.conditioningprocessor(batch, cond_mask, dt)
        return self._trunk(batch, sembs, B, H, W, dt, head_nhwc, None)

    def update_parts(self):
        """Split of the parameters for an optimizer step overlapped with the
        next forward: ``(early, level)`` -- the parameters the forward reads
        before encoder level ``level`` (conditioning processor, stem, encoder
        levels below ``level`` and the FiLM projections of those levels,
        decoder blocks included since the level-batched FiLM runs up front);
        every other parameter can still be in flight until that level starts.
        None when the model is too shallow for a useful split."""
        L = self.num_resolutions
        if L < 3:
            return None
        level = 2
        early = []
        early += list(self.conditioningprocessor.parameters())
        early += list(self.conv.parameters())
        for i in range(level):
            early += list(self.xunetblocks[i].parameters())
        groups = self._film_groups()
        for i in range(level):
            for b in groups[i]:
                early += [b.film.dense.weight, b.film.dense.bias]
        seen, out = set(), []
        for p_ in early:
            if id(p_) not in seen:
                seen.add(id(p_))
                out.append(p_)
        return out, level

    def _cond_stream(self, ref: Optional[torch.Tensor]):
        """The conditioning side stream (HIP path, level-batched FiLM): the
        camera-ray / logSNR conditioning and the FiLM projections of every
        level depend only on the poses and logSNR, not on the trunk, so they
        run on their own HIP stream -- level 0 first -- while the trunk's stem
        and level-0 blocks run; the trunk waits on one event per level right
        before that level's first block.  Autograd runs their backward on the
        same stream.  D3D_COND_STREAM=0 keeps everything on one stream."""
        if not (self.batch_film and _COND_STREAM and ref is not None and ref.is_cuda
                and (self.compute_dtype or ref.dtype) == torch.bfloat16 and ops.use_hip(ref, any_dtype=True)):
            return None
        # measured gain at 64x64 (bs16 / bs128).  At 128x128 the EAGER step
        # (multi-GB conditioning tensors) ran 4.5x slower with the second
        # stream (profiles/ab_cond_stream_r2.txt): the caching allocator keeps
        # one block cache per stream, so the side stream's freed blocks were
        # unusable by the trunk and every step hit allocation retries (a full
        # cache flush + device sync each).  Inside a HIP-graph capture every
        # stream of the capture allocates from the graph's one private pool
        # and replays allocate nothing, so the side stream is safe there at
        # any size; eager steps above 64x64 keep one stream unless
        # D3D_COND_STREAM=2.
        if (self.H * self.W > 64 * 64 and os.environ.get("D3D_COND_STREAM", "1") != "2"
                and not torch.cuda.is_current_stream_capturing()):
            return None
        idx = ref.device.index if ref.device.index is not None else torch.cuda.current_device()
        st = _COND_STREAMS.get(idx)
        if st is None:
            st = _COND_STREAMS[idx] = torch.cuda.Stream(device=idx,
                                                        priority=0)
            from ..ops.gradsink import SINK
            SINK.add_compute_stream(st)
        return st

    def _forward_shared(self, batch, sc, head_nhwc):
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            raise RuntimeError("shared_cond is an inference path: run it under torch.no_grad()")
        xz = batch.get("xz")
        if xz is not None:
            B, H, W = xz.shape[0] // 2, xz.shape[1], xz.shape[2]
            xdt = xz.dtype
        else:
            B, _, H, W = batch["x"].shape
            xdt = batch["x"].dtype
        assert (H, W) == (self.H, self.W), ((H, W), (self.H, self.W))
        ecls = sc["example_class"]
        assert ecls.shape == (B,), (ecls.shape, B)
        Bc = sc["logsnr"].shape[0]
        for key in ("R", "t", "K", "cond_mask"):
            assert sc[key].shape[0] == Bc, (key, sc[key].shape, Bc)
        dt = self.compute_dtype or xdt
        sembs = self.conditioningprocessor(sc, sc["cond_mask"], dt)
        # image (example e, frame f) -> conditioning image (class of e, frame f)
        fr = torch.arange(2, device=ecls.device, dtype=torch.int32)
        ss_map = (2 * ecls.to(torch.int32)[:, None] + fr).reshape(-1)
        return self._trunk(batch, sembs, B, H, W, dt, head_nhwc, ss_map)

    def _trunk(self, batch, sembs, B, H, W, dt, head_nhwc, ss_map, cond=None):
        for blocks in self._film_groups():
            for b in blocks:
                b.__dict__["_ss_map"] = ss_map
        events = None
        if cond is not None:
            # conditioning + level-batched FiLM on the side stream, one event per level
            cs, cbatch, cond_mask = cond
            main = torch.cuda.current_stream()
            cs.wait_stream(main)
            for t in list(cbatch.values()) + [cond_mask]:
                if isinstance(t, torch.Tensor) and t.is_cuda:
                    t.record_stream(cs)
            sembs, events = [], []
            fence = PARAM_FENCE[0]
            with torch.cuda.stream(cs):
                for i, (semb, blocks) in enumerate(zip(self.conditioningprocessor.levels(cbatch, cond_mask, dt),
                                                       self._film_groups())):
                    if fence is not None and i == fence[0]:
                        cs.wait_event(fence[1])
                    outs = ops.film_batch(semb, [b.film.dense.weight for b in blocks],
                                          [b.film.dense.bias for b in blocks], block_events=FILM_BLOCK_EVENTS,
                                          split=len(self.xunetblocks[i]))
                    for o in outs:
                        o.record_stream(main)       # read by the trunk's GN-FiLM kernels
                    ev = torch.cuda.Event()
                    ev.record(cs)
                    for b, o in zip(blocks, outs):
                        b.__dict__["_ss"] = o
                        # the block waits right before its GN-FiLM, for its own slice when the
                        # projection ran per block
                        b.__dict__["_ss_event"] = getattr(o, "_d3d_ready", ev)
                    events.append(ev)
                    sembs.append(semb)
        elif ss_map is not None or self.batch_film:
            # every FiLM projection of a level reads the same embedding: run
            # them as one GEMM per level (ops.film_batch) and hand each
            # ResnetBlock its modulation slice
            fence = PARAM_FENCE[0]
            for i, blocks in enumerate(self._film_groups()):
                if fence is not None and i == fence[0]:
                    torch.cuda.current_stream().wait_event(fence[1])
                # (split: the encoder blocks lead the level's group, _film_groups;
                # the decoder blocks' FiLM weight gradients can start early)
                outs = ops.film_batch(sembs[i], [b.film.dense.weight for b in blocks],
                                      [b.film.dense.bias for b in blocks], split=len(self.xunetblocks[i]))
                for b, o in zip(blocks, outs):
                    b.__dict__["_ss"] = o
        xz = batch.get("xz")
        if xz is not None:
            h = xz.to(dt)
        else:
            x, z = batch["x"], batch["z"]
            C = x.shape[1]
            h = torch.stack([x, z], dim=1).reshape(2 * B, C, H, W).permute(0, 2, 3, 1).to(dt).contiguous()
        h = ops.conv3x3(h, self.conv.weight, self.conv.bias)

        L = self.num_resolutions
        hs = [h]
        fence = PARAM_FENCE[0]
        for i in range(L):
            if fence is not None and i == fence[0]:
                torch.cuda.current_stream().wait_event(fence[1])
            for j in range(self.num_res_blocks):
                h = self.xunetblocks[i][j](h, sembs[i])
                hs.append(h)
            if i != L - 1:
                h = self.xunetblocks[i][-1](h, sembs[i])
                hs.append(h)
        h = self.middle(h, sembs[-1])
        for i in reversed(range(L)):
            level = self.upsample[str(i)]
            for j in range(self.num_res_blocks + 1):
                h = level[j]((h, hs.pop()), sembs[i])       # skip concat, fused into the block entry
            if i != 0:
                h = level[-1](h, sembs[i])
        assert not hs
        # only frame 1 (the target view) is returned by the reference
        h1 = self.lastgn(h[1::2].contiguous(), silu=True)
        out = ops.conv3x3(h1, self.lastconv.weight, self.lastconv.bias, keep_pad=head_nhwc)
        if head_nhwc:
            return out
        return out.permute(0, 3, 1, 2)


_GOLDEN = 0x9E3779B97F4A7C15


def _next_seed(block: ResnetBlock) -> int:
    """64-bit dropout seed of one block: slot part + base * golden ratio.  The
    HIP mask kernels of a graph replay add ``device_word * golden`` to a baked
    slot part (base 0), so eager and replayed steps draw identical masks when
    the device word equals the eager base seed (engine/graphs.py)."""
    base = getattr(block, "_base_seed", 0)
    return (block._seed_slot * 7919 + 17 + base * _GOLDEN) & 0xFFFFFFFFFFFFFFFF


def count_params(model: nn.Module) -> int:
    return sum(p.numel() for p in model.parameters())
