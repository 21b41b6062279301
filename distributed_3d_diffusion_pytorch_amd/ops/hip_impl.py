"""Autograd bindings of the gfx950 HIP kernels (``libd3d_hip.so``).

Every function takes/returns NHWC bf16 activations on the current HIP stream
and fp32 master parameters; parameter gradients are produced in fp32.  No
host synchronisation, no allocation inside the kernels (workspaces come from
the torch caching allocator), so the whole step can be captured in a HIP
graph.
"""
from __future__ import annotations

import contextlib
import collections
import ctypes
import os
import math
from typing import Dict, Optional, Tuple

import torch
import torch.nn.functional as F

from ._backend import load_library
from . import torch_impl as _t
from .gradsink import SINK

_lib = load_library(required=True)
BF16 = torch.bfloat16
F32 = torch.float32

_ZERO_PAGE: Dict[int, torch.Tensor] = {}
# FiLM weight gradients: "tn" (the transposed-read split-K MFMA GEMM of
# wgrad_gemm.hip with the bias sums folded in), "blas" (hipBLASLt product +
# separate bias sums + segment scatter; profiles/ab_film_wgrad.txt) or "seg"
# (the 1x1 conv weight-gradient kernel)
_FILM_WGRAD = "tn"
# level-batched FiLM forward of the big levels on hipBLASLt (plain GEMM + bias)
_FILM_BLAS = os.environ.get("D3D_FILM_BLAS", "1") != "0"
# FiLM weight gradients of a level in two jobs: the decoder blocks' (complete
# early in the backward) as soon as their GN-FiLM backwards have written their
# d(scale|shift) columns, the encoder blocks' after the level's last block --
# instead of one level-wide job after that last block (the first encoder
# block: the 64x64 level's whole weight gradient, P = 1M rows, ran exposed at
# the very end of the backward).  Measured (profiles/r6/film_early_wgrad.txt):
# +0.7 % at bs16 (graph-captured step), -0.7 % at bs128 (eager step: its
# weight-gradient stream is saturated, so the earlier job only delays the
# conv weight gradients), and one job per BLOCK -3 % / -2 % (each re-reads the
# level's [P, 1024] silu(e) operand).  OFF by default: in the 1-rank RCCL
# graph step with a 32-job flush batch the early jobs leave NaN gradients in
# other parameters (4 of bucket 24 at the first replay; tools/
# diag_flush_nan_bisect.sh isolates it to this switch) and the cause is not
# found.  D3D_FILM_EARLY_WGRAD: 0 (default) never, 1 graph-captured steps,
# 2 always.
_FILM_EARLY = int(os.environ.get("D3D_FILM_EARLY_WGRAD", "0"))
# D3D_FILM_WGRAD_INLINE=1: the level's LAST FiLM weight-gradient job runs in
# place, on the stream the level-batched FiLM backward runs on (the
# conditioning stream), instead of queueing behind the conv weight gradients
# on the side stream, where the 64x64 level's ran with nothing beside it
# (bs128: ~4.6 ms/step of wgrad_tn_k "solo").  Measured -1.1 % at bs128 and
# +0.4 % (noise) at bs16 -- overlapping it only slows the kernels it joins --
# so off (profiles/r6/film_wgrad_inline.txt).
_FILM_INLINE = os.environ.get("D3D_FILM_WGRAD_INLINE", "0") == "1"


def set_conv_impl(impl: str) -> None:
    """'bufl' (default: buffer-descriptor LDS-DMA pipelined MFMA kernel),
    'glds' (flat-address LDS-DMA) or 'reg' (register-staged); the latter two
    are kept for A/B measurements and for operands beyond 2 GiB."""
    dev = torch.cuda.current_device()
    if dev not in _ZERO_PAGE:
        _ZERO_PAGE[dev] = torch.zeros(64, dtype=BF16, device="cuda")
    _chk(_lib.d3d_set_conv_impl({"reg": 0, "glds": 1, "bufl": 2, "bufl1": 3, "w8": 4, "w8w": 6, "w8n": 7, "halo": 8}[impl], _ZERO_PAGE[dev].data_ptr()), "set_conv_impl")


def set_conv_korder(korder: int) -> None:
    """glds conv k-step order (1: channel-chunk major, default; 0: tap major)."""
    _chk(_lib.d3d_set_conv_korder(int(korder)), "set_conv_korder")


_WGRAD_IMPLS = {"reg": 0, "glds": 1, "glds64x2": 1, "glds32x2": 2, "glds32x3": 3, "glds64x3": 4, "bufl": 5,
                "w8": 6}


def set_wgrad_impl(impl: str) -> None:
    """Weight-gradient kernel: 'reg' (register-staged, padded LDS rows) or a
    DMA-staged variant 'glds<pixels per stage>x<stages>'."""
    _chk(_lib.d3d_set_wgrad_impl(_WGRAD_IMPLS[impl]), "set_wgrad_impl")


_IMPL_SET = [False]


def _ensure_impl():
    if not _IMPL_SET[0]:
        import os
        set_conv_impl("halo")
        set_wgrad_impl("w8")
        _IMPL_SET[0] = True


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


def _st() -> int:
    return torch.cuda.current_stream().cuda_stream


# Launch-checking debug mode (the counterpart of
# CUDA_LAUNCH_BLOCKING for the native kernels): D3D_SYNC_CHECK=1 synchronises
# the device after every native launch outside graph capture, so an
# asynchronous fault (out-of-bounds access, trap) is reported at the op that
# caused it, and keeps a ring of the last launches for the post-mortem.
_SYNC_CHECK = os.environ.get("D3D_SYNC_CHECK", "0") == "1"
_RECENT = collections.deque(maxlen=64)


def set_sync_check(on: bool) -> None:
    global _SYNC_CHECK
    _SYNC_CHECK = bool(on)


def recent_launches() -> list:
    """Names of the last native launches (recorded with D3D_SYNC_CHECK=1)."""
    return list(_RECENT)


def _chk(rc: int, name: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{name} failed with hipError {rc}")
    if _SYNC_CHECK:
        _RECENT.append(name)
        if not torch.cuda.is_current_stream_capturing():
            try:
                torch.cuda.synchronize()
            except RuntimeError as e:
                raise RuntimeError(f"{name}: device fault after launch (recent: {list(_RECENT)[-8:]}): {e}") from e


def _need_bf16(*ts):
    for t in ts:
        if t is not None and t.dtype != BF16:
            raise TypeError(f"HIP kernels take bf16 activations, got {t.dtype}")


# Shapes a HIP kernel does not cover run the torch composition instead -- only
# with D3D_ALLOW_TORCH_FALLBACK=1 (the same switch that guards the library
# load, ops/_backend.py): otherwise such a shape is an error, so a GPU run can
# never silently leave the native path.  Each allowed (op, shape) is reported
# once on stderr and counted here; bench.py reports the count and the
# full-model / graph-step tests assert it stays empty.
FALLBACKS: Dict[str, int] = {}


class NativeFallbackError(RuntimeError):
    """A shape outside the HIP kernels' coverage while fallbacks are not allowed."""


def fallbacks_allowed() -> bool:
    return os.environ.get("D3D_ALLOW_TORCH_FALLBACK", "0") == "1"


def _fallback(op: str, why: str) -> None:
    key = f"{op}: {why}"
    if not fallbacks_allowed():
        raise NativeFallbackError(f"HIP {op} does not cover this shape ({why}); set D3D_ALLOW_TORCH_FALLBACK=1 "
                                  "to run the torch composition instead")
    if key not in FALLBACKS:
        import sys
        print(f"[d3d] HIP {op} falls back to the torch composition ({why})", file=sys.stderr, flush=True)
    FALLBACKS[key] = FALLBACKS.get(key, 0) + 1


def _up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


# --------------------------------------------------------------------------
# bf16 operand cache of the fp32 master weights.  Every entry keeps a
# descriptor; after the optimizer step ``refresh_weights()`` re-derives ALL
# entries in one kernel launch (instead of ~500 lazy per-layer packs).  Any
# other in-place change of a parameter bumps its version and rebuilds that
# entry alone.
_EPOCH = [0]
_WCACHE: Dict[Tuple, list] = {}          # key -> [tok, tensor, desc_tuple]
_DESC_TABLE = [None, None, -1, 0]        # descriptors, block->descriptor map, revision, total blocks
_REV = [0]


def invalidate_weight_cache() -> None:
    _EPOCH[0] += 1
    _WCACHE.clear()
    _CATBUF.clear()
    _REV[0] += 1


def _cached(p: torch.Tensor, kind: str, build, desc=None):
    if not isinstance(p, torch.nn.Parameter):
        return build()      # temporaries (e.g. channel-padded stem/head weights)
    key = (p.data_ptr(), kind, tuple(p.shape))
    tok = (p._version, _EPOCH[0])
    hit = _WCACHE.get(key)
    if hit is not None and hit[0] == tok:
        return hit[1]
    v = build()
    _WCACHE[key] = [tok, v, (p, desc)]
    _REV[0] += 1
    return v


def _pack_blocks(OC: int, OCp: int, ICp: int, mode: int) -> int:
    """Blocks of pack_all_k for one operand (must match its tiling): fwd pack
    = one output row x 256 input channels, transposed pack = 32 x 16 channel
    tiles, plain cast = 2048 elements."""
    if mode == 0:
        return OCp * ((ICp + 255) // 256)
    if mode == 1:
        return ((OCp + 31) // 32) * ((ICp + 15) // 16)
    return (OC + 2047) // 2048


def _desc_tensors(rows, blk):
    """Device descriptor table (conv.hip PackDesc rows) + block -> row map."""
    import numpy as np
    dt = np.dtype([("src", np.uint64), ("dst", np.uint64), ("OC", np.int32), ("IC", np.int32),
                   ("OCp", np.int32), ("ICp", np.int32), ("taps", np.int32), ("mode", np.int32),
                   ("blk0", np.int32), ("ICs", np.int32), ("ldd", np.int32), ("pad", np.int32)])
    arr = np.array(rows, dtype=dt)
    host = torch.from_numpy(arr.view(np.uint8).copy())
    counts = np.diff(np.append(arr["blk0"], blk))
    bmap = torch.from_numpy(np.repeat(np.arange(len(rows), dtype=np.int32), counts))
    return host.to("cuda"), bmap.to("cuda")


def refresh_weights() -> None:
    """After an optimizer update of the master weights: one launch repacks
    every cached operand; cache tokens advance to the new epoch."""
    _EPOCH[0] += 1
    if not _WCACHE:
        _attn_refresh()
        return
    if _DESC_TABLE[2] != _REV[0]:
        rows = []
        blk = 0
        for key, (tok, t, (p, desc)) in _WCACHE.items():
            if desc is None:
                continue
            OC, IC, OCp, ICp, taps, mode = desc[:6]
            src_off = desc[6] if len(desc) > 6 else 0        # byte offset (channel slice)
            ics = desc[7] if len(desc) > 7 else 0            # source IC stride
            ldd = desc[8] if len(desc) > 8 else 0            # destination row stride (transposed cat)
            rows.append((p.data_ptr() + src_off, t.data_ptr(), OC, IC, OCp, ICp, taps, mode, blk, ics, ldd, 0))
            blk += _pack_blocks(OC, OCp, ICp, mode)
        _DESC_TABLE[0], _DESC_TABLE[1] = _desc_tensors(rows, blk)
        _DESC_TABLE[2] = _REV[0]
        _DESC_TABLE[3] = blk
    _chk(_lib.d3d_pack_all(_DESC_TABLE[0].data_ptr(), _DESC_TABLE[1].data_ptr(), _DESC_TABLE[3], _st()), "pack_all")
    for ent in _WCACHE.values():
        p = ent[2][0]
        ent[0] = (p._version, _EPOCH[0])
    _attn_refresh()


def packed_weight(w: torch.Tensor, trans: bool, taps: int = 9) -> torch.Tensor:
    """[OC, IC(, kh, kw)] fp32 -> [OCp][taps][ICp] bf16 (trans: [ICp][taps][OCp])
    for the MFMA kernels; GEMM-M dims padded to 128 (block M), K chunks to 64."""
    OC, IC = w.shape[0], w.shape[1]

    def build():
        if not trans:
            OCp, ICp = _up(OC, 128), _up(IC, 64)
            out = torch.empty(OCp * taps * ICp, dtype=BF16, device=w.device)
        else:
            OCp, ICp = _up(OC, 64), _up(IC, 128)
            out = torch.empty(ICp * taps * OCp, dtype=BF16, device=w.device)
        _chk(_lib.d3d_pack_weight(w.data_ptr(), out.data_ptr(), OC, IC, OCp, ICp, int(trans), taps, _st()),
             "pack_weight")
        return out
    if not trans:
        desc = (OC, IC, _up(OC, 128), _up(IC, 64), taps, 0)
    else:   # kernel-side names: rows = IC (padded 128), K = OC (padded 64)
        desc = (OC, IC, _up(OC, 64), _up(IC, 128), taps, 1)
    return _cached(w, f"pack{taps}{'T' if trans else ''}", build, desc)


def packed_weight_slice(w: torch.Tensor, ic0: int, nic: int, ICp: int) -> torch.Tensor:
    """Forward-packed [OCp][9][ICp] bf16 operand of the input-channel slice
    w[:, ic0:ic0+nic] of a 3x3 weight (the ray-direction half of a
    conditioning conv), refreshed with every other cached operand."""
    OC, IC = w.shape[0], w.shape[1]
    OCp = _up(OC, 128)

    def build():
        v = w.detach()[:, ic0:ic0 + nic].reshape(OC, nic, 9).permute(0, 2, 1)
        out = torch.zeros(OCp, 9, ICp, dtype=BF16, device=w.device)
        out[:OC, :, :nic] = v.to(BF16)
        return out.reshape(-1)
    desc = (OC, nic, OCp, ICp, 9, 0, ic0 * 9 * 4, IC)
    return _cached(w, f"slice{ic0}_{nic}_{ICp}", build, desc)


def packed_conv_weight(w: torch.Tensor, trans: bool) -> torch.Tensor:
    return packed_weight(w, trans, 9)


_CATBUF: Dict[Tuple, torch.Tensor] = {}


def bf16_cat(params, kind: str) -> torch.Tensor:
    """bf16 copy of ``cat([p.reshape(p.shape[0], -1) for p in params])`` kept
    as ONE persistent buffer: every parameter's slice is a cache entry whose
    descriptor points into the buffer, so the batched repack after each
    optimizer step refreshes it in place and a forward never concatenates
    (the level-batched FiLM projection weights / biases)."""
    key = (kind,) + tuple((p.data_ptr(), tuple(p.shape)) for p in params)
    buf = _CATBUF.get(key)
    rows = [p.shape[0] for p in params]
    cols = params[0].numel() // params[0].shape[0]
    if buf is None:
        buf = torch.empty(sum(rows), cols, dtype=BF16, device=params[0].device)
        _CATBUF[key] = buf
    off = 0
    for p, r in zip(params, rows):
        view = buf[off: off + r]

        def build(p=p, view=view):
            view.copy_(p.detach().reshape(view.shape))
            return view
        _cached(p, f"{kind}@{buf.data_ptr()}", build, (p.numel(), 1, 1, 1, 1, 2))
        off += r
    return buf if cols > 1 else buf.reshape(-1)


def bf16_catT(params, kind: str) -> torch.Tensor:
    """bf16 ``cat([p for p in params]).t()`` ([K, sum rows], the input-gradient
    operand of a level-batched projection) kept as ONE persistent buffer:
    every parameter's column block is a cache entry of the transposed pack
    (mode 1, destination row stride = the total width), refreshed in the
    batched repack after each optimizer step."""
    key = (kind,) + tuple((p.data_ptr(), tuple(p.shape)) for p in params)
    rows = [p.shape[0] for p in params]
    K = params[0].shape[1]
    S = sum(rows)
    buf = _CATBUF.get(key)
    if buf is None:
        buf = torch.empty(K, S, dtype=BF16, device=params[0].device)
        _CATBUF[key] = buf
    off = 0
    for p, r in zip(params, rows):
        view = buf[:, off: off + r]

        def build(p=p, view=view):
            view.copy_(p.detach().t())
            return view
        _cached(p, f"{kind}@{buf.data_ptr()}", build, (r, K, r, K, 1, 1, 0, 0, S))
        off += r
    return buf


def bf16_weight(w: torch.Tensor) -> torch.Tensor:
    desc = (w.numel(), 1, 1, 1, 1, 2)
    if w.dim() == 1:
        return _cached(w, "bf16", lambda: w.detach().to(BF16), desc)
    return _cached(w, "bf16", lambda: w.detach().reshape(w.shape[0], -1).to(BF16), desc)


# Per-step seed block on the device (graph replay: a captured kernel cannot
# see a new Python seed): int64 [dropout word, input-draw word, example
# offset].  The mask kernels add word 0 (x golden) to their baked seed, the
# input draw adds word 1 and offsets its example index by word 2.  None in
# eager mode.
_SEED_DEV = [None]


def set_device_seed(t: Optional[torch.Tensor]) -> None:
    assert t is None or (t.dtype == torch.int64 and t.is_cuda and t.numel() >= 3)
    _SEED_DEV[0] = t


# ------------------------------------------------------------ GroupNorm ----
def _gn_plan(N, P, C):
    a, b = ctypes.c_int(), ctypes.c_int()
    _lib.d3d_gn_plan(N, P, C, ctypes.byref(a), ctypes.byref(b))
    return a.value, b.value


def _gn_stats(x, G, eps):
    N, H, W, C = x.shape
    P = H * W
    nch, _ = _gn_plan(N, P, C)
    part = torch.empty(N * nch * G * 2, dtype=F32, device=x.device)
    stats = torch.empty(N * G * 2, dtype=F32, device=x.device)
    _chk(_lib.d3d_gn_stats(x.data_ptr(), N, P, C, G, eps, part.data_ptr(), stats.data_ptr(), None, 0, _st()),
         "gn_stats")
    return stats


# Whole-image GroupNorm kernels (norm.hip gn_img_*): images of at most this
# many pixels (the 16x16 / 8x8 levels) run each GroupNorm pass as ONE launch
# that keeps an (image, channel slab) in registers -- statistics and backward
# reductions inside the block.  D3D_GN_IMG=<max pixels> (0: off).  Batches
# of 64..128 images also take it at the 32x32 level (norm.hip img_plan;
# D3D_GN_IMG_WIDE=<lo>:<hi> images, "0" off).
if os.environ.get("D3D_GN_IMG"):
    _lib.d3d_gn_img_cfg(int(os.environ["D3D_GN_IMG"]))
if os.environ.get("D3D_GN_IMG_WIDE"):
    _w = os.environ["D3D_GN_IMG_WIDE"]
    _lo, _hi = (int(v) for v in _w.split(":")) if ":" in _w else (1 << 30, 0)
    _lib.d3d_gn_img_wide_cfg(_lo, _hi)
_GN_IMG_OK: Dict[Tuple[int, ...], bool] = {}


def gn_img_ok(P: int, C: int, G: int, N: int = 0) -> bool:
    """True when a GroupNorm over N images of P pixels runs on the
    whole-image kernels (the same answer for its forward, backward and the
    producer that would otherwise emit its statistics)."""
    key = (P, C, G, N, _lib.d3d_gn_img_cfg(-1), _lib.d3d_gn_img_wide_cfg(-1, 0))
    v = _GN_IMG_OK.get(key)
    if v is None:
        v = _GN_IMG_OK[key] = bool(_lib.d3d_gn_img_ok_n(N, P, C, G))
    return v


def _gn_fwd(mode, x, w, b, G, eps, ss=None, ssld=0, p=0.0, seed=0, x2=None, ss_map=None):
    """Statistics pass + fused finalize/apply (mode 0 GN, 1 GN+SiLU, 2 GN+FiLM):
    two launches (one when the producing epilogue made the statistics, or for
    small images: the whole-image kernel); returns (y, stats) with stats =
    per-(image, group) mean/rstd.  With x2, the input is the virtual channel
    concat [x | x2]."""
    N, H, W, C1 = x.shape
    C = C1 + (x2.shape[-1] if x2 is not None else 0)
    P = H * W
    stats = torch.empty(N * G * 2, dtype=F32, device=x.device)
    if gn_img_ok(P, C, G, N):
        y = torch.empty(N, H, W, C, dtype=x.dtype, device=x.device)
        _chk(_lib.d3d_gn_img_fwd(mode, x.data_ptr(), stats.data_ptr(), w.data_ptr(), b.data_ptr(), _ptr(ss),
                                 y.data_ptr(), N, P, C, G, float(eps), float(p), int(seed), int(ssld),
                                 _ptr(_SEED_DEV[0]) if mode == 2 else None, _ptr(x2), C1, _ptr(ss_map), _st()),
             "gn_img_fwd")
        return y, stats
    fused = getattr(x, "_d3d_gnpart", None) if x2 is None else None
    if fused is not None and fused[1] == G:
        part, conv_parts = fused[0], fused[2]       # statistics came out of the producing conv's epilogue
    else:
        nch, _ = _gn_plan(N, P, C)
        part = torch.empty(N * nch * G * 2, dtype=F32, device=x.device)
        conv_parts = 0
        _chk(_lib.d3d_gn_stats(x.data_ptr(), N, P, C, G, eps, part.data_ptr(), None, _ptr(x2), C1, _st()),
             "gn_stats")
    y = torch.empty(N, H, W, C, dtype=x.dtype, device=x.device)
    _chk(_lib.d3d_gn_apply2(mode, x.data_ptr(), part.data_ptr(), stats.data_ptr(), w.data_ptr(), b.data_ptr(),
                            _ptr(ss), y.data_ptr(), N, P, C, G, float(eps), float(p), int(seed), int(ssld),
                            _ptr(_SEED_DEV[0]) if mode == 2 else None, _ptr(x2), C1, int(conv_parts),
                            _ptr(ss_map), _st()),
         "gn_apply2")
    return y, stats


class ResGradSlot:
    """Hand-off of the gradient of a tensor x between its two consumers in a
    block: a GroupNorm (GN0 / the attention GN) and the block's residual
    branch (the conv2 / out-projection residual, or the 1x1 NIN skip's input).
    The residual branch's backward -- which autograd runs before the
    GroupNorm's, since the GroupNorm output feeds it -- deposits its gradient
    here instead of returning it, and the GroupNorm backward adds it inside
    its apply kernel: no bf16 autograd add over x's gradient.  If the
    GroupNorm backward ran first after all, the branch returns its gradient
    normally (``consumed``), so any order stays correct.  The deposit is
    ``scale * g`` kept unscaled (the kernel applies the scale), so the
    branch's own backward never materialises its scaled output gradient."""
    __slots__ = ("g", "scale", "g2", "scale2", "consumed")

    def __init__(self):
        self.g = self.g2 = None
        self.scale = self.scale2 = 1.0
        self.consumed = False

    def deposit(self, g: torch.Tensor, scale: float = 1.0) -> bool:
        """Two deposits ride into the kernel (a block's residual branch and a
        decoder skip consumer of the same tensor); a third is folded in fp32."""
        if self.consumed:
            return False
        if self.g is None:
            self.g, self.scale = g, float(scale)
        elif self.g2 is None:
            self.g2, self.scale2 = g, float(scale)
        else:
            self.g, self.scale = (self.g.float() * self.scale + g.float() * scale).to(g.dtype), 1.0
        return True

    def take(self):
        r = (self.g, self.scale, self.g2, self.scale2)
        self.g = self.g2 = None
        self.scale = self.scale2 = 1.0
        self.consumed = True
        return r


def _gn_bwd(mode, x, dy, ss, stats, w, b, G, p, seed, dss=None, ssld=0, x2=None, dres=None, dres_scale=1.0,
            dres2=None, dres2_scale=1.0):
    N, H, W, C1 = x.shape
    C = C1 + (x2.shape[-1] if x2 is not None else 0)
    P = H * W
    if gn_img_ok(P, C, G, N):
        return _gn_bwd_img(mode, x, dy, ss, stats, w, b, G, p, seed, dss, ssld, x2, dres, dres_scale, dres2,
                           dres2_scale)
    nch, _ = _gn_plan(N, P, C)
    dev = x.device
    dx = torch.empty_like(x)
    dx2 = torch.empty_like(x2) if x2 is not None else None
    if dss is None and ss is not None:
        dss = torch.empty_like(ss)
    tg, tb = SINK.target(w), SINK.target(b)
    direct = tg is not None and tb is not None
    dg = tg if direct else torch.empty(C, dtype=F32, device=dev)
    db = tb if direct else torch.empty(C, dtype=F32, device=dev)
    cp = torch.empty(N * nch * C * 2, dtype=F32, device=dev)
    gp = torch.empty(N * nch * G * 2 + N * 2 * C + 64 * 2 * C, dtype=F32, device=dev)
    coef = torch.empty(N * G * 2, dtype=F32, device=dev)
    _chk(_lib.d3d_gn_bwd2(mode, x.data_ptr(), dy.data_ptr(), _ptr(ss), stats.data_ptr(), w.data_ptr(),
                          b.data_ptr(), N, P, C, G, float(p), int(seed), dx.data_ptr(), _ptr(dss), dg.data_ptr(),
                          db.data_ptr(), cp.data_ptr(), gp.data_ptr(), coef.data_ptr(), int(direct), int(ssld),
                          _ptr(_SEED_DEV[0]) if mode == 2 else None, _ptr(x2), _ptr(dx2), C1, _ptr(dres),
                          float(dres_scale), _ptr(dres2), float(dres2_scale), _st()),
         "gn_bwd")
    if x2 is not None:
        dx = (dx, dx2)
    if direct:
        SINK.done(w)
        SINK.done(b)
        return dx, dss, None, None
    return dx, dss, dg, db


def _gn_bwd_img(mode, x, dy, ss, stats, w, b, G, p, seed, dss, ssld, x2, dres, dres_scale, dres2, dres2_scale):
    """Whole-image GroupNorm backward: ONE launch on the compute stream (dx,
    dss) plus the fold of its per-image dgamma / dbeta rows -- a parameter
    gradient nothing downstream waits for, so it runs as a sink job on the
    weight-gradient stream when the parameters are sink-managed."""
    N, H, W, C1 = x.shape
    C = C1 + (x2.shape[-1] if x2 is not None else 0)
    P = H * W
    dev = x.device
    dx = torch.empty_like(x)
    dx2 = torch.empty_like(x2) if x2 is not None else None
    if dss is None and ss is not None:
        dss = torch.empty_like(ss)
    chan = torch.empty(N * 2 * C + 64 * 2 * C, dtype=F32, device=dev)     # [N][C][2] rows + colsum workspace
    _chk(_lib.d3d_gn_img_bwd(mode, x.data_ptr(), dy.data_ptr(), _ptr(ss), stats.data_ptr(), w.data_ptr(),
                             b.data_ptr(), N, P, C, G, float(p), int(seed), dx.data_ptr(), _ptr(dss), chan.data_ptr(),
                             int(ssld), _ptr(_SEED_DEV[0]) if mode == 2 else None, _ptr(x2), _ptr(dx2), C1,
                             _ptr(dres), float(dres_scale), _ptr(dres2), float(dres2_scale), _st()),
         "gn_img_bwd")
    if x2 is not None:
        dx = (dx, dx2)
    tg, tb = SINK.target(w), SINK.target(b)
    ws = chan[N * 2 * C:]
    if tg is not None and tb is not None:
        def job():
            _chk(_lib.d3d_colsum(chan.data_ptr(), N, 2 * C, ws.data_ptr(), tg.data_ptr(), tb.data_ptr(), 1, _st()),
                 "gn_img_dgb")
        # the column sums of a flush run as one batched launch (sink_group_run)
        spec = _ColJob(chan.data_ptr(), tg.data_ptr(), tb.data_ptr(), N, 2 * C, 1, 0) if _COLSUM_GROUP else None
        SINK.submit(dev, job, (chan,), (w, b), spec=spec)
        return dx, dss, None, None
    dg = torch.empty(C, dtype=F32, device=dev)
    db = torch.empty(C, dtype=F32, device=dev)
    _chk(_lib.d3d_colsum(chan.data_ptr(), N, 2 * C, ws.data_ptr(), dg.data_ptr(), db.data_ptr(), 0, _st()),
         "gn_img_dgb")
    return dx, dss, dg, db


class _GroupNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, groups, eps, silu, slot=None):
        x = x.contiguous()
        N, H, W, C = x.shape
        y, stats = _gn_fwd(1 if silu else 0, x, weight, bias, groups, eps)
        ctx.save_for_backward(x, weight, bias, stats)
        ctx.cfg = (groups, 1 if silu else 0)
        ctx.slot = slot
        SINK.use(weight, ctx.needs_input_grad[1])
        SINK.use(bias, ctx.needs_input_grad[2])
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, b, stats = ctx.saved_tensors
        G, mode = ctx.cfg
        dres, rsc, dres2, rsc2 = ctx.slot.take() if ctx.slot is not None else (None, 1.0, None, 1.0)
        if dres is not None:
            dres = dres.reshape(x.shape).contiguous()
        if dres2 is not None:
            dres2 = dres2.reshape(x.shape).contiguous()
        dy = dy.contiguous()
        dx, _, dg, db = _gn_bwd(mode, x, dy, None, stats, w, b, G, 0.0, 0, dres=dres, dres_scale=rsc,
                                dres2=dres2, dres2_scale=rsc2)
        return dx, dg, db, None, None, None, None




# decoder NIN skip as ONE GEMM over [h | skip] when both halves have the same
# width (12 of the 16 decoder blocks); D3D_CAT_GEMM=0: two GEMMs
_CAT_GEMM = os.environ.get("D3D_CAT_GEMM", "1") != "0"
# conv2 hands the skip's gradient to the NIN op through a slot with its 1/sqrt2
# (no scaled copy of dy per decoder block); D3D_SKIP_SLOT=0: returned scaled
_SKIP_SLOT = os.environ.get("D3D_SKIP_SLOT", "1") != "0"


class _CatGNDense(torch.autograd.Function):
    """Decoder ResnetBlock entry on the virtual concat x = [h | skip]
    (`xunet.py:521-531` + `xunet.py:139-150`): returns silu(GN0(x)) and the
    1x1 NIN skip dense(x) without materialising x: the GroupNorm kernels read
    both halves in place, the dense is two accumulating GEMMs, and the backward
    writes the two input gradients directly (no concat / split copies, no
    accumulation of the two branches' gradients)."""

    @staticmethod
    def forward(ctx, a, b, gw, gb, dw, db, groups, eps):
        a, b = a.contiguous(), b.contiguous()
        N, H, W, C1 = a.shape
        C2 = b.shape[-1]
        y, stats = _gn_fwd(1, a, gw, gb, groups, eps, x2=b)
        wb = bf16_weight(dw)                                    # [OC, C1 + C2]
        OC = wb.shape[0]
        a2, b2 = a.reshape(-1, C1), b.reshape(-1, C2)
        C = C1 + C2
        skip = None
        if C1 == C2 and _CAT_GEMM:
            # one GEMM over the virtual concat (gemm.hip F_CAT: the B operand
            # switches tensors at K = C1)
            skip = torch.empty(a2.shape[0], OC, dtype=BF16, device=a.device)
            bias = db.detach() if db is not None else None
            if _lib.d3d_gemm_cat(wb.data_ptr(), a2.data_ptr(), b2.data_ptr(), C1, skip.data_ptr(), _ptr(bias), OC,
                                 a2.shape[0], C, C, OC, 1.0, 1.0, _st()) < 0:
                skip = None
        if skip is not None:
            pass
        elif _gemm_ok(OC, a2.shape[0], C1, C, C1, a2, wb) and _gemm_ok(OC, b2.shape[0], C2, C, C2, b2, wb[:, C1:]):
            # two GEMMs over the halves; the second accumulates through its residual epilogue
            skip = torch.empty(a2.shape[0], OC, dtype=BF16, device=a.device)
            gemm_nt(wb, a2, skip, OC, a2.shape[0], C1, C, C1, OC, bias=db.detach() if db is not None else None)
            gemm_nt(wb[:, C1:], b2, skip, OC, b2.shape[0], C2, C, C2, OC, res=skip)
        else:
            _fallback("cat_gn_silu_dense", f"C1={C1} C2={C2} OC={OC} (library GEMM)")
            skip = torch.addmm(bf16_weight(db), a2, wb[:, :C1].t()) if db is not None else \
                torch.mm(a2, wb[:, :C1].t())
            skip.addmm_(b2, wb[:, C1:].t())
        ctx.save_for_backward(a, b, gw, gb, stats, dw)
        ctx.cfg = (groups, db is not None)
        ctx.params = (dw, db)
        # the skip's other consumer (the next encoder block's GroupNorm, whose
        # backward runs after this one) takes b's gradient inside its apply
        # kernel: no autograd bf16 add of the two gradients
        ctx.bslot = getattr(b, "_d3d_res_slot", None)
        SINK.use(gw, ctx.needs_input_grad[2])
        SINK.use(gb, ctx.needs_input_grad[3])
        SINK.use(dw, ctx.needs_input_grad[4])
        SINK.use(db, ctx.needs_input_grad[5])
        # the skip's consumer (conv2's residual, out = s * (conv + skip)) may
        # deposit its unscaled gradient and s here instead of returning a
        # scaled copy (models.xunet.ResnetBlock); s rides on the GEMM alphas
        # and the weight-gradient job
        ctx.oslot = ResGradSlot() if _SKIP_SLOT else None
        ctx.set_materialize_grads(False)
        skip = skip.view(N, H, W, OC)
        if ctx.oslot is not None:
            skip._d3d_out_slot = ctx.oslot
        return y, skip

    @staticmethod
    def backward(ctx, dy, dskip):
        a, b, gw, gb, stats, dw = ctx.saved_tensors
        G, has_db = ctx.cfg
        N, H, W, C1 = a.shape
        C2 = b.shape[-1]
        dwp, dbp = ctx.params
        OC = dwp.shape[0]
        if dy is None:
            dy = torch.zeros(N, H, W, C1 + C2, dtype=BF16, device=a.device)
        dy = dy.contiguous()
        (da, db_in), _, dgw, dgb = _gn_bwd(1, a, dy, None, stats, gw, gb, G, 0.0, 0, x2=b)
        # the skip's gradient: returned by autograd, or deposited (unscaled,
        # with its scale) by conv2's backward into the output slot
        gs = 1.0
        g = dskip
        if ctx.oslot is not None:
            d1, s1, d2, s2 = ctx.oslot.take()
            if d1 is not None:
                if d2 is not None:
                    d1, s1 = (d1.float() * s1 + d2.float() * s2).to(BF16), 1.0
                if g is not None:
                    d1, s1 = (d1.float() * s1 + g.float()).to(BF16), 1.0
                g, gs = d1, s1
        if g is None:
            g = torch.zeros(N, H, W, OC, dtype=BF16, device=a.device)
        g = g.contiguous()
        g2 = g.reshape(-1, OC)
        rows = g2.shape[0]
        C = C1 + C2
        gW = gB = None
        tw = SINK.target(dwp)
        tb = SINK.target(dbp) if has_db else None
        direct = tw is not None and (not has_db or tb is not None)
        dWt = tw.view(OC, C) if direct else torch.zeros(OC, C, dtype=F32, device=g.device)
        dbt = (tb if direct else torch.zeros(OC, dtype=F32, device=g.device)) if has_db else None
        spec = wgrad_job(g2, a, OC, C, rows, 1, 1, 1, dWt, dbt, gs, x2=b, C1=C1) if direct else None
        if gs != 1.0 and spec is None:
            # the per-job weight-gradient path takes no scale: a scaled copy
            gsc = torch.empty_like(g2)
            _chk(_lib.d3d_add_scale(g2.data_ptr(), None, gsc.data_ptr(), float(gs), g2.numel(), _st()), "scale")
            g2, gs = gsc, 1.0
        OCp = _up(OC, 64)
        rows_ = g2.shape[0]
        if g2.is_contiguous() and _gemm_ok(C1, rows_, OC, OCp, OC, g2, da, db_in) and \
                _gemm_ok(C2, rows_, OC, OCp, OC, g2, da, db_in):
            pk = packed_weight(dw, True, 1)                      # [ICp][OCp]: rows = input channels
            d2a, d2b = da.view(-1, C1), db_in.view(-1, C2)
            gemm_nt(pk, g2, d2a, C1, rows_, OC, OCp, OC, C1, res=d2a, alpha=gs)
            gemm_nt(pk[C1 * OCp:], g2, d2b, C2, rows_, OC, OCp, OC, C2, res=d2b, alpha=gs)
        else:
            wb = bf16_weight(dw)
            da.view(-1, C1).addmm_(g2, wb[:, :C1], alpha=gs)
            db_in.view(-1, C2).addmm_(g2, wb[:, C1:], alpha=gs)
        # one weight-gradient GEMM over the virtual concat (the kernel picks
        # the source per 128-channel tile); two GEMMs when it cannot
        _ensure_impl()
        def job():
            sp, pps = ctypes.c_int(), ctypes.c_int()
            _lib.d3d_conv_wgrad_plan2(rows, 1, 1, OC, C, 1, ctypes.byref(sp), ctypes.byref(pps))
            ws = torch.empty(sp.value * OC * C + 2 * sp.value * OC, dtype=F32, device=g.device)
            rc = _lib.d3d_conv_wgrad_cat(g2.data_ptr(), a.data_ptr(), b.data_ptr(), C1, ws.data_ptr(), dWt.data_ptr(),
                                         _ptr(dbt), rows, C, OC, sp.value, pps.value, 1, _st())
            if rc < 0:
                g4 = g2.reshape(rows, 1, 1, OC)
                dW1, dbias = _wgrad(g4, a.reshape(rows, 1, 1, C1), OC, C1, rows, 1, 1, 1, 1, 1, 1, want_bias=has_db)
                dW2, _ = _wgrad(g4, b.reshape(rows, 1, 1, C2), OC, C2, rows, 1, 1, 1, 1, 1, 1)
                dWt[:, :C1].add_(dW1.view(OC, C1))
                dWt[:, C1:].add_(dW2.view(OC, C2))
                if has_db:
                    dbt.add_(dbias)
            else:
                _chk(rc, "wgrad_cat")
        if direct:
            SINK.submit(g.device, job, (g2, a, b), (dwp, dbp if has_db else None), spec=spec)
        else:
            job()
            gW = dWt.view(dwp.shape)
            gB = dbt
        if ctx.bslot is not None and ctx.bslot.deposit(db_in):
            db_in = None
        return da, db_in, dgw, dgb, gW, gB, None, None


def cat_gn_silu_dense(a, b, gw, gb, dw, db, groups=32, eps=1e-5):
    _need_bf16(a, b)
    C1, C2 = a.shape[-1], b.shape[-1]
    if C1 % 8 or C2 % 8 or (C1 + C2) // groups > 1024:
        x = torch.cat([a, b], -1)
        return group_norm(x, gw, gb, groups, eps, True), linear(x, dw, db)
    return _CatGNDense.apply(a, b, gw, gb, dw, db, groups, eps)


def group_norm(x, weight, bias, groups=32, eps=1e-5, silu=False, res_slot=None):
    _need_bf16(x)
    return _GroupNorm.apply(x, weight, bias, groups, eps, silu, res_slot)


def _ss_layout(ss: torch.Tensor, C: int):
    """Row stride of a FiLM modulation [N,H,W,2C]: 2C when contiguous, or the
    parent width when ss is a channel slice of a level-batched projection."""
    N, H, W, C2 = ss.shape
    ld = ss.stride(2)
    if C2 == 2 * C and ss.stride(3) == 1 and ss.stride(1) == W * ld and ss.stride(0) == H * W * ld and ld >= C2:
        return ss, ld
    return ss.contiguous(), 2 * C


class _GNFiLM(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, ss, groups, eps, p, seed, ss_map=None):
        x = x.contiguous()
        N, H, W, C = x.shape
        slot = getattr(ss, "_d3d_slot", None)
        ss, ld = _ss_layout(ss, C)
        if ss_map is not None:
            assert ss_map.dtype == torch.int32 and ss_map.is_contiguous() and ss_map.shape == (N,), \
                (ss_map.dtype, ss_map.shape, N)
            assert ss.shape[1:3] == (H, W), (ss.shape, x.shape)
        y, stats = _gn_fwd(2, x, weight, bias, groups, eps, ss, ld, p, seed, ss_map=ss_map)
        ctx.save_for_backward(x, weight, bias, ss, stats)
        ctx.cfg = (groups, p, seed, ld)
        ctx.slot = slot if ld != 2 * C or slot is not None else None
        SINK.use(weight, ctx.needs_input_grad[1])
        SINK.use(bias, ctx.needs_input_grad[2])
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, b, ss, stats = ctx.saved_tensors
        G, p, seed, ld = ctx.cfg
        dss = None
        into_slot = ctx.slot is not None and ctx.needs_input_grad[3] and ctx.slot[0].width == ld
        if into_slot:
            # write d(scale|shift) straight into the level's shared dY buffer
            # so the batched FiLM backward runs one GEMM with no gather (the
            # kernel reads ss and writes dss with ONE row stride: only when
            # the forward modulation has the buffer's width)
            holder, off = ctx.slot
            dss = holder.grad_slice(off, x.shape[-1])
        dx, dss, dg, db = _gn_bwd(2, x, dy.contiguous(), ss, stats, w, b, G, p, seed, dss=dss, ssld=ld)
        if into_slot:
            ctx.slot[0].block_ready(ctx.slot[1])      # this block's FiLM weight gradient can start
        return dx, dg, db, dss, None, None, None, None, None


def gn_film(x, weight, bias, ss, groups=32, eps=1e-5, dropout_p=0.0, training=False, seed=0, ss_map=None):
    _need_bf16(x, ss)
    p = float(dropout_p) if training else 0.0
    if ss_map is not None and torch.is_grad_enabled() and \
            any(t is not None and t.requires_grad for t in (x, weight, bias, ss)):
        raise RuntimeError("gn_film(ss_map=) is inference-only")
    return _GNFiLM.apply(x, weight, bias, ss, groups, eps, p, int(seed) & 0xFFFFFFFFFFFFFFFF, ss_map)


# ----------------------------------------------------------------- conv ----
if os.environ.get("D3D_GEMM_TUNE"):     # A/B knob "cfg,gm,grid" (gemm.hip d3d_gemm_tune; 0 keeps a value)
    _lib.d3d_gemm_tune(*[int(v) for v in os.environ["D3D_GEMM_TUNE"].split(",")])
if os.environ.get("D3D_HALO_AU"):        # A/B knob: halo conv with unrolled taps / precomputed offsets (1) or not (0)
    _lib.d3d_conv_halo_cfg(int(os.environ["D3D_HALO_AU"]))
if os.environ.get("D3D_GEMM_SMALL_K"):   # A/B knob: 128x128 tiles for short-K 256-768-channel GEMMs (1) or not (0)
    _lib.d3d_gemm_small_k(int(os.environ["D3D_GEMM_SMALL_K"]))
if os.environ.get("D3D_CONV_HSM"):      # A/B knob: small-image halo conv (conv_small.hip conv_hsm_k) on (1) / off (0)
    _lib.d3d_conv_hsm_cfg(int(os.environ["D3D_CONV_HSM"]))
if os.environ.get("D3D_GN_CFG"):        # A/B knob "blocks,red_u,app_u": GroupNorm launch shapes
    _lib.d3d_gn_cfg(*[int(v) for v in os.environ["D3D_GN_CFG"].split(",")])
if os.environ.get("D3D_GN_CFG_SMALL"):  # "max_images,blocks": blocks per launch for small batches ("0,0" off)
    _lib.d3d_gn_cfg_small(*[int(v) for v in os.environ["D3D_GN_CFG_SMALL"].split(",")])


def _conv_fwd(x, wp, bias, row_bias, res, out, N, H, W, IC, ICp, OH, OW, OC, ldo, stride, trans, scale, res_nmod=0,
              taps=9, gn_groups=0, silu_out=None):
    """Launch the conv; with gn_groups > 0 the epilogue may also emit the
    GroupNorm partial statistics of ``out``: returns (part, nparts) when it
    did (the consuming GroupNorm then skips its statistics pass), else None.
    ``silu_out``: also write silu(out) there -- from the epilogue when the
    chosen kernel can, else by the SiLU pass."""
    _ensure_impl()
    ns = _lib.d3d_conv_plan(N, OH, OW, OC, ICp, taps) if ldo == OC else 1
    ws = torch.empty(ns * N * OH * OW * OC, dtype=F32, device=x.device) if ns > 1 else None
    gnp = None
    if gn_groups and (OH * OW) % 64 == 0:
        gnp = torch.empty(N * gn_groups * (OH * OW // 64) * 2, dtype=F32, device=x.device)
    done = ctypes.c_int(0)
    sdone = ctypes.c_int(0)
    _chk(_lib.d3d_conv3(x.data_ptr(), wp.data_ptr(), _ptr(bias), _ptr(row_bias), _ptr(res), out.data_ptr(), N, H, W,
                        IC, ICp, OH, OW, OC, ldo, stride, int(trans), float(scale), int(res_nmod), taps, _ptr(ws), ns,
                        _ptr(gnp), int(gn_groups), ctypes.byref(done), _ptr(silu_out), ctypes.byref(sdone), _st()),
         "conv")
    if silu_out is not None and not sdone.value:
        _chk(_lib.d3d_silu(out.data_ptr(), silu_out.data_ptr(), out.numel(), _st()), "silu")
    return (gnp, OH * OW // 64) if done.value else None


def _wgrad(g, x, OC, IC, N, H, W, OH, OW, stride, taps=9, want_bias=False, dW=None, db=None, accumulate=False,
           scale=1.0):
    """Split-K weight gradient (+ fused bias column sums).  Writes into the
    given dW/db (accumulating when asked) or into fresh fp32 tensors."""
    _ensure_impl()
    if _WGRAD_DIRECT_HALO and stride == 1 and (OH, OW) == (H, W) and taps == 9 and x.dtype == BF16:
        # the all-taps halo tile when it takes the shape (one grouped launch of one job)
        dW_ = dW if dW is not None else torch.empty(OC, IC, taps, dtype=F32, device=x.device)
        db_ = db if (db is not None or not want_bias) else torch.empty(OC, dtype=F32, device=x.device)
        j = wgrad_job(g, x, OC, IC, N, H, W, taps, dW_, db_, scale, accumulate) if g.is_contiguous() and \
            x.is_contiguous() else None
        if j is not None and _lib.d3d_wgrad_group_engine(ctypes.byref(j)) == 1:
            wgrad_group_run([j])
            return dW_, db_
    s, pps = ctypes.c_int(), ctypes.c_int()
    _lib.d3d_conv_wgrad_plan3(N, H, W, OH, OW, OC, IC, taps, stride, ctypes.byref(s), ctypes.byref(pps))
    extra = 2 * s.value * OC if (want_bias or db is not None) else 0
    ws = torch.empty(s.value * OC * taps * IC + extra, dtype=F32, device=x.device)
    if dW is None:
        dW = torch.empty(OC, IC, taps, dtype=F32, device=x.device)
    if want_bias and db is None:
        db = torch.empty(OC, dtype=F32, device=x.device)
    _chk(_lib.d3d_conv_wgrad3(g.data_ptr(), x.data_ptr(), ws.data_ptr(), dW.data_ptr(), _ptr(db), N, H, W, IC, OH,
                              OW, OC, stride, s.value, pps.value, int(accumulate), taps, float(scale), _st()),
         "conv_wgrad")
    return dW, db


# ------------------------------------------------- grouped weight gradients
class _WgJob(ctypes.Structure):
    """One weight-gradient job of a grouped launch (wgrad_group.hip
    WgJobDesc): dW[co][ci][tap] (+)= scale * sum_p dY[p][co] X[p+shift][ci],
    db[co] (+)= scale * sum_p dY[p][co]; X may be the virtual concat [x | x2]
    split at channel C1."""
    _fields_ = [("dy", ctypes.c_void_p), ("x", ctypes.c_void_p), ("x2", ctypes.c_void_p),
                ("dw", ctypes.c_void_p), ("db", ctypes.c_void_p),
                ("N", ctypes.c_int), ("H", ctypes.c_int), ("W", ctypes.c_int), ("OC", ctypes.c_int),
                ("IC", ctypes.c_int), ("C1", ctypes.c_int), ("taps", ctypes.c_int), ("acc", ctypes.c_int),
                ("scale", ctypes.c_float), ("pad_", ctypes.c_int)]


assert ctypes.sizeof(_WgJob) == 80
# 1: weight-gradient jobs deferred inside graph capture run grouped, one
# launch (+ one slab reduce) per sink flush; 0: one launch pair per job
_WGRAD_GROUP = os.environ.get("D3D_WGRAD_GROUP", "1") != "0"
# direct (non-sink) weight gradients -- the conditioning conv's -- on the halo tile when it takes the shape
_WGRAD_DIRECT_HALO = _WGRAD_GROUP and os.environ.get("D3D_WGRAD_DIRECT_HALO", "1") != "0"
if os.environ.get("D3D_WGRAD_GROUP_BLOCKS"):           # planner target (A/B knob): blocks per grouped launch
    _lib.d3d_wgrad_group_cfg(int(os.environ["D3D_WGRAD_GROUP_BLOCKS"]), 0, 0)
if os.environ.get("D3D_WGRAD_GROUP_NS"):               # A/B knob: LDS ring stages (2-4)
    _lib.d3d_wgrad_group_stages(int(os.environ["D3D_WGRAD_GROUP_NS"]))
if os.environ.get("D3D_WGRAD_HALO"):                   # A/B knob "on[,blocks[,stages]]": all-taps halo tiles
    _hv = [int(v) for v in os.environ["D3D_WGRAD_HALO"].split(",")] + [0, 0]
    _lib.d3d_wgrad_group_halo(_hv[0], _hv[1], _hv[2])
if os.environ.get("D3D_WGRAD_HALO_BIG"):               # A/B knob "blocks,lg2": halo target of the big flushes
    _lib.d3d_wgrad_group_halo_big(*[int(v) for v in os.environ["D3D_WGRAD_HALO_BIG"].split(",")])
if os.environ.get("D3D_ATTN_FWD_ALL_MIN"):             # A/B knob: min (image, head) pairs for the
    _lib.d3d_attn_fwd_cfg(int(os.environ["D3D_ATTN_FWD_ALL_MIN"]))   # one-workgroup-per-head forward
if os.environ.get("D3D_ATTN_WIDE_MIN"):               # A/B knob: (image, head) pairs from which one workgroup owns
    _lib.d3d_attn_bwd_cfg(int(os.environ["D3D_ATTN_WIDE_MIN"]))   # all keys of an attention backward (L <= 256)
if os.environ.get("D3D_WGRAD_HALO_PK"):                # A/B knob: pixels per halo K-step (32 / 64, the latter at W >= 64)
    _lib.d3d_wgrad_group_halo_pk(int(os.environ["D3D_WGRAD_HALO_PK"]))


def wgrad_job(dy, x, OC, IC, N, H, W, taps, dw, db=None, scale=1.0, accumulate=True, x2=None, C1=0):
    """A grouped weight-gradient job over contiguous bf16 dY [P, OC] and X
    [P, IC] (or [P, C1] + x2 [P, IC - C1]), or None when the grouped kernel
    cannot take it (the caller keeps its per-job path)."""
    if not _WGRAD_GROUP or dw is None:
        return None
    for t in (dy, x, x2):
        if t is not None and (t.dtype != BF16 or not t.is_contiguous()):
            return None
    j = _WgJob(dy.data_ptr(), x.data_ptr(), _ptr(x2), dw.data_ptr(), _ptr(db), int(N), int(H), int(W), int(OC),
               int(IC), int(C1 if x2 is not None else IC), int(taps), int(bool(accumulate)), float(scale), 0)
    return j if _lib.d3d_wgrad_group_ok(ctypes.byref(j)) == 0 else None


def wgrad_group_run(jobs) -> None:
    """Run grouped weight-gradient jobs on the current stream: at most 16 per
    launch and never two writing the same gradient in one launch (the
    unsplit epilogue accumulates in place)."""
    dev = torch.device("cuda", torch.cuda.current_device())
    batch, seen = [], set()

    def go(b):
        arr = (_WgJob * len(b))(*b)
        need = _lib.d3d_wgrad_group(arr, len(b), None, 0, None)
        if need < 0:
            raise RuntimeError(f"d3d_wgrad_group plan failed ({need})")
        ws = torch.empty(max(int(need), 1), dtype=F32, device=dev)
        rc = _lib.d3d_wgrad_group(arr, len(b), ws.data_ptr(), int(need), _st())
        if rc != 0:
            raise RuntimeError(f"d3d_wgrad_group failed ({rc})")
        if _SYNC_CHECK:
            _chk(0, "wgrad_group")

    for j in jobs:
        keys = {j.dw} | ({j.db} if j.db else set())
        if len(batch) == 16 or keys & seen:
            go(batch)
            batch, seen = [], set()
        batch.append(j)
        seen |= keys
    if batch:
        go(batch)


class _ColJob(ctypes.Structure):
    """reduce.hip ColJob: one [R][Cc] column sum (interleaved pairs -> two outputs)."""
    _fields_ = [("inp", ctypes.c_void_p), ("out0", ctypes.c_void_p), ("out1", ctypes.c_void_p), ("R", ctypes.c_int),
                ("Cc", ctypes.c_int), ("acc", ctypes.c_int), ("blk0", ctypes.c_int)]


assert ctypes.sizeof(_ColJob) == 40
_COLSUM_GROUP = os.environ.get("D3D_COLSUM_GROUP", "1") != "0"


def colsum_group_run(jobs) -> None:
    """Run batched column-sum jobs on the current stream, 16 per launch, never
    two accumulating into the same output in one launch."""
    batch, seen = [], set()

    def go(b):
        arr = (_ColJob * len(b))(*b)
        _chk(_lib.d3d_colsum_jobs(arr, len(b), _st()), "colsum_jobs")

    for j in jobs:
        keys = {j.out0, j.out1}
        if len(batch) == 16 or keys & seen:
            go(batch)
            batch, seen = [], set()
        batch.append(j)
        seen |= keys
    if batch:
        go(batch)


def sink_group_run(specs) -> None:
    """The sink's grouped launch: weight-gradient specs as grouped wgrad
    launches, column-sum specs as batched column sums (issue order kept per kind)."""
    wg = [s_ for s_ in specs if not isinstance(s_, _ColJob)]
    cs = [s_ for s_ in specs if isinstance(s_, _ColJob)]
    if wg:
        wgrad_group_run(wg)
    if cs:
        colsum_group_run(cs)


SINK.group_fn = sink_group_run


def _chansum(g, per_image: bool):
    N, OH, OW, C = g.shape
    P = OH * OW
    nch = max(1, min(64, (2048 + N - 1) // N, (P + 63) // 64))
    part = torch.empty((nch + 1) * N * C + 64 * C, dtype=F32, device=g.device)
    per = torch.empty(N, C, dtype=F32, device=g.device) if per_image else None
    tot = torch.empty(C, dtype=F32, device=g.device)
    _chk(_lib.d3d_chansum(g.data_ptr(), part.data_ptr(), _ptr(per), tot.data_ptr(), N, P, C, nch, _st()), "chansum")
    return per, tot


class _Conv(torch.autograd.Function):
    """Implicit-GEMM conv (taps=9: 3x3 pad 1 stride s; taps=1: per-pixel
    linear) with fused bias / per-image bias / residual / scale epilogue.
    Backward: input grad via the same kernel in transposed mode, weight grad
    via the split-K transpose-read kernel, bias grads via channel sums."""

    @staticmethod
    def forward(ctx, x, weight, bias, stride, residual, out_scale, row_bias, res_period, taps, gn=None, res_slot=None):
        x = x.contiguous()
        N, H, W, IC = x.shape
        OC = weight.shape[0]
        assert weight.shape[1] == IC and IC % 8 == 0 and OC % 8 == 0, (tuple(weight.shape), IC, OC)
        if taps == 9:
            OH, OW = (H - 1) // stride + 1, (W - 1) // stride + 1
        else:
            assert stride == 1
            OH, OW = H, W
        wp = packed_weight(weight, False, taps)
        out = torch.empty(N, OH, OW, OC, dtype=BF16, device=x.device)
        res = residual.contiguous() if residual is not None else None
        rb = row_bias.contiguous().float() if row_bias is not None else None
        parts = _conv_fwd(x, wp, bias, rb, res, out, N, H, W, IC, _up(IC, 64), OH, OW, OC, OC, stride, False,
                          out_scale, res_period, taps, gn["groups"] if gn is not None else 0)
        if gn is not None and parts is not None:
            gn["part"] = parts
        ctx.save_for_backward(x, weight)
        ctx.cfg = (stride, out_scale, residual is not None, row_bias is not None, bias is not None, res_period, taps)
        ctx.bias_param = bias
        ctx.res_slot = res_slot
        SINK.use(weight, ctx.needs_input_grad[1])
        SINK.use(bias, ctx.needs_input_grad[2])
        return out

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        stride, scale, has_res, has_rb, has_b, res_period, taps = ctx.cfg
        N, H, W, IC = x.shape
        OC = weight.shape[0]
        dy = dy.contiguous()
        _, OH, OW, _ = dy.shape
        bias = ctx.bias_param
        need_w, need_b = ctx.needs_input_grad[1], has_b and ctx.needs_input_grad[2]
        # out = scale * (conv + residual): the gradient of both is scale * dy.
        # Fold the scale into the kernels (dgrad epilogue, wgrad reduction,
        # the GroupNorm that takes the residual's share) instead of writing a
        # scaled copy of dy, whenever every consumer can take it that way.
        slot = ctx.res_slot
        lazy = scale != 1.0 and not has_rb and not res_period and (need_w or not need_b) and \
            (not has_res or not ctx.needs_input_grad[4] or (slot is not None and not slot.consumed))
        if scale != 1.0 and not lazy:
            g = torch.empty_like(dy)
            _chk(_lib.d3d_add_scale(dy.data_ptr(), None, g.data_ptr(), float(scale), dy.numel(), _st()), "scale")
            ks = 1.0
        else:
            g, ks = dy, scale
        dx = None
        if ctx.needs_input_grad[0]:
            wt = packed_weight(weight, True, taps)
            dx = torch.empty_like(x)
            _conv_fwd(g, wt, None, None, None, dx, N, OH, OW, OC, _up(OC, 64), H, W, IC, IC, stride, True, ks, 0,
                      taps)
        dW = db = drb = None
        tw = SINK.target(weight) if need_w else None
        tb = SINK.target(bias) if need_b else None
        if has_rb:
            # per-image bias gradient (conditioning convs) -> channel sums
            per, tot = _chansum(g, True)
            drb = per
            if need_b:
                if tb is not None:
                    tb.add_(tot)
                    SINK.done(bias)
                else:
                    db = tot
            need_b = False
        if need_w:
            direct = tw is not None and (not need_b or tb is not None)
            if direct:
                def job(g=g, x=x, tw=tw, tb=tb if need_b else None, ks=ks):
                    _wgrad(g, x, OC, IC, N, H, W, OH, OW, stride, taps, dW=tw.view(OC, IC, taps), db=tb,
                           accumulate=True, scale=ks)
                spec = wgrad_job(g, x, OC, IC, N, H, W, taps, tw, tb if need_b else None, ks) \
                    if stride == 1 and (OH, OW) == (H, W) else None
                SINK.submit(g.device, job, (g, x), (weight, bias if need_b else None), spec=spec)
            else:
                dW, db2 = _wgrad(g, x, OC, IC, N, H, W, OH, OW, stride, taps, want_bias=need_b, scale=ks)
                dW = dW.reshape(weight.shape)
                if need_b:
                    db = db2
        elif need_b:
            gg = g if taps == 9 else g.reshape(1, N * OH * OW, 1, OC)
            db = _chansum(gg, False)[1]
        dres = None
        if has_res and ctx.needs_input_grad[4]:
            if res_period:
                dres = _period_sum(g, res_period)
            elif slot is None or not slot.deposit(g, ks):
                assert ks == 1.0            # (lazy only when the slot takes it)
                dres = g
        return dx, dW, db, None, dres, None, drb, None, None, None, None


# ResnetBlock GN0 + SiLU folded into conv1's halo staging (conv.hip
# conv_halo_k GNA) where that conv runs on the 256-pixel halo tiles (the
# 32x32 level at 16 examples per GPU).  Measured -1.1 % at bs16
# (profiles/r6/gn_conv_fusion.txt), so off by default; D3D_GN_CONV=1 enables it.
_GN_CONV = os.environ.get("D3D_GN_CONV", "0") == "1"


def gn_silu_conv_ok(x: torch.Tensor, OC: int, groups: int) -> bool:
    """True when :func:`gn_silu_conv3x3` takes this shape (chunked GroupNorm
    and the halo conv's 256-pixel tiles)."""
    if not _GN_CONV or x.dtype != BF16 or x.dim() != 4:
        return False
    _ensure_impl()
    N, H, W, C = x.shape
    return not gn_img_ok(H * W, C, groups, N) and bool(_lib.d3d_conv3_gn_ok(N, H, W, C, OC))


class _GNSiLUConv(torch.autograd.Function):
    """conv3x3(silu(GroupNorm(x))) with the GroupNorm + SiLU applied to the
    conv's input halo in LDS (`xunet.py:114-131`'s GN0 -> SiLU -> conv1): the
    normalised activation h is never written in the forward.  Backward: the
    conv's input gradient dh as usual, the GroupNorm backward on (x, dh) (with
    the residual-gradient hand-off of x's other consumer), and the conv's
    weight gradient on h rematerialised from x by the same arithmetic, inside
    the weight-gradient job (side stream)."""

    @staticmethod
    def forward(ctx, x, gw, gb, cw, cb, groups, eps, gn1_groups, slot, info):
        x = x.contiguous()
        N, H, W, C = x.shape
        OC = cw.shape[0]
        P = H * W
        fused = getattr(x, "_d3d_gnpart", None)
        if fused is not None and fused[1] == groups:
            part, conv_parts = fused[0], fused[2]
        else:
            nch, _ = _gn_plan(N, P, C)
            part = torch.empty(N * nch * groups * 2, dtype=F32, device=x.device)
            conv_parts = 0
            _chk(_lib.d3d_gn_stats(x.data_ptr(), N, P, C, groups, eps, part.data_ptr(), None, None, C, _st()),
                 "gn_stats")
        stats = torch.empty(N * groups * 2, dtype=F32, device=x.device)
        ab = torch.empty(N * C * 2, dtype=F32, device=x.device)
        _chk(_lib.d3d_gn_ab(part.data_ptr(), stats.data_ptr(), gw.data_ptr(), gb.data_ptr(), ab.data_ptr(), N, P, C,
                            groups, float(eps), int(conv_parts), _st()), "gn_ab")
        wp = packed_weight(cw, False, 9)
        out = torch.empty(N, H, W, OC, dtype=BF16, device=x.device)
        gnp = torch.empty(N * gn1_groups * (P // 64) * 2, dtype=F32, device=x.device) \
            if gn1_groups and P % 64 == 0 else None
        done = ctypes.c_int(0)
        rc = _lib.d3d_conv3_gn(x.data_ptr(), wp.data_ptr(), _ptr(cb), out.data_ptr(), N, H, W, C, _up(C, 64), OC,
                               _ptr(gnp), int(gn1_groups), ctypes.byref(done), ab.data_ptr(), _st())
        if rc == -2:
            raise RuntimeError("gn_silu_conv3x3: shape not taken (check gn_silu_conv_ok first)")
        _chk(rc, "conv3_gn")
        ctx.save_for_backward(x, gw, gb, stats, ab, cw)
        ctx.cfg = (groups, cb is not None)
        ctx.slot = slot
        ctx.cb = cb
        if done.value:
            info["part"] = (gnp, P // 64)
        for i, p_ in ((1, gw), (2, gb), (3, cw), (4, cb)):
            SINK.use(p_, ctx.needs_input_grad[i])
        return out

    @staticmethod
    def backward(ctx, dy):
        x, gw, gb, stats, ab, cw = ctx.saved_tensors
        G, has_b = ctx.cfg
        cb = ctx.cb
        N, H, W, C = x.shape
        OC = cw.shape[0]
        dy = dy.contiguous()
        dev = x.device
        # conv input gradient dh
        wt = packed_weight(cw, True, 9)
        dh = torch.empty_like(x)
        _conv_fwd(dy, wt, None, None, None, dh, N, H, W, OC, _up(OC, 64), H, W, C, C, 1, True, 1.0, 0, 9)
        # conv weight / bias gradients on h = silu(x * A + B), rematerialised
        dW = dB = None
        need_w, need_b = ctx.needs_input_grad[3], has_b and ctx.needs_input_grad[4]
        if need_w or need_b:
            tw = SINK.target(cw) if need_w else None
            tb = SINK.target(cb) if need_b else None

            def remat():
                h = torch.empty_like(x)
                _chk(_lib.d3d_gn_ab_silu(x.data_ptr(), ab.data_ptr(), h.data_ptr(), N, H * W, C, _st()), "gn_ab_silu")
                return h
            if need_w and tw is not None and (not need_b or tb is not None):
                def job(dy=dy, tw=tw, tb=tb):
                    _wgrad(dy, remat(), OC, C, N, H, W, H, W, 1, 9, dW=tw.view(OC, C, 9), db=tb, accumulate=True)
                SINK.submit(dev, job, (dy, x, ab), (cw, cb if need_b else None))
            else:
                dW, dB = _wgrad(dy, remat(), OC, C, N, H, W, H, W, 1, 9, want_bias=need_b)
                dW = dW.reshape(cw.shape) if need_w else None
        # GroupNorm + SiLU backward on (x, dh), with x's other consumer's gradient
        dres, rsc, dres2, rsc2 = ctx.slot.take() if ctx.slot is not None else (None, 1.0, None, 1.0)
        if dres is not None:
            dres = dres.reshape(x.shape).contiguous()
        if dres2 is not None:
            dres2 = dres2.reshape(x.shape).contiguous()
        dx, _, dg, db = _gn_bwd(1, x, dh, None, stats, gw, gb, G, 0.0, 0, dres=dres, dres_scale=rsc, dres2=dres2,
                                dres2_scale=rsc2)
        return dx, dg, db, dW, dB, None, None, None, None, None


def gn_silu_conv3x3(x, gw, gb, cw, cb, groups=32, eps=1e-5, gn1_groups=0, res_slot=None):
    """``conv3x3(silu(group_norm(x)), cw, cb)`` with the GroupNorm + SiLU in
    the conv's input staging (see :func:`gn_silu_conv_ok`).  ``gn1_groups``:
    the output's GroupNorm partial statistics from the epilogue, as
    :func:`conv3x3`'s ``gn_groups``."""
    _need_bf16(x)
    OC = cw.shape[0]
    if gn1_groups and gn_img_ok(x.shape[1] * x.shape[2], OC, int(gn1_groups), x.shape[0]):
        gn1_groups = 0
    info = {}
    y = _GNSiLUConv.apply(x, gw, gb, cw, cb, int(groups), float(eps), int(gn1_groups), res_slot, info)
    if "part" in info:
        y._d3d_gnpart = (info["part"][0], int(gn1_groups), info["part"][1])
    return y


def conv3x3(x, weight, bias, stride=1, residual=None, out_scale=1.0, row_bias=None, res_period=0, gn_groups=0,
            res_slot=None, keep_pad=False):
    """3x3 conv.  gn_groups > 0: the output feeds a GroupNorm with that many
    groups -- the conv epilogue then also emits the GroupNorm's partial
    statistics when its kernel can (attached to the output as ``_d3d_gnpart``
    and consumed by :func:`group_norm` / :func:`gn_film`)."""
    _need_bf16(x, residual)
    OC, IC = weight.shape[0], weight.shape[1]
    if IC % 8 == 0 and OC % 8 == 0:
        if gn_groups:
            OH, OW = (x.shape[1] - 1) // stride + 1, (x.shape[2] - 1) // stride + 1
            if gn_img_ok(OH * OW, OC, int(gn_groups), x.shape[0]):
                gn_groups = 0           # the consumer's whole-image kernel makes its own statistics
        gn = {"groups": int(gn_groups)} if gn_groups else None
        y = _Conv.apply(x, weight, bias, stride, residual, out_scale, row_bias, res_period, 9, gn, res_slot)
        if gn is not None and "part" in gn:
            y._d3d_gnpart = (gn["part"][0], int(gn_groups), gn["part"][1])
        return y
    # stem (IC=3) / head (OC=3): zero-pad channels to a multiple of 8 so every
    # access stays 16-byte vectorised; the padding costs < 0.1 % of FLOPs.
    ICe, OCe = _up(IC, 8), _up(OC, 8)
    xe = F.pad(x, (0, ICe - x.shape[-1])) if x.shape[-1] != ICe else x      # (the fused input draw is pre-padded)
    we = F.pad(weight, (0, 0, 0, 0, 0, ICe - IC, 0, OCe - OC))
    be = F.pad(bias, (0, OCe - OC)) if bias is not None else None
    re = F.pad(residual, (0, OCe - OC)) if residual is not None else None
    rbe = F.pad(row_bias, (0, OCe - OC)) if row_bias is not None else None
    y = _Conv.apply(xe, we, be, stride, re, out_scale, rbe, res_period, 9)
    return y[..., :OC].contiguous() if (OCe != OC and not keep_pad) else y


# ------------------------------------------------- conditioning conv ------
_TAPCOEF: Dict[Tuple, torch.Tensor] = {}


def _tap_coef(IH, IW, OH, OW, stride, device):
    """[9, 9] matrix M with dU[n, t] = sum_k M[t, k] * stats[n, k] over
    stats = [image total, first row, last row, first col, last col, corners
    (0,0) (0,W-1) (H-1,0) (H-1,W-1)]: the sum of dy over the pixels where tap t
    reads inside the image, by inclusion-exclusion (built once per geometry,
    eagerly, so graph capture never sees the host copy)."""
    key = (IH, IW, OH, OW, stride, str(device))
    m = _TAPCOEF.get(key)
    if m is None:
        rows = []
        for t in range(9):
            kh, kw = t // 3, t % 3
            top = kh - 1 < 0
            bot = (OH - 1) * stride + kh - 1 >= IH
            left = kw - 1 < 0
            right = (OW - 1) * stride + kw - 1 >= IW
            rows.append([1.0, -top, -bot, -left, -right, top and left, top and right, bot and left, bot and right])
        m = torch.tensor(rows, dtype=F32).to(device)
        _TAPCOEF[key] = m
    return m


def _period_sum(g: torch.Tensor, period: int) -> torch.Tensor:
    """Gradient of a residual broadcast over the batch with the given period:
    [N, ...] -> [period, ...], summed over the N / period repeats (bf16, fp32
    accumulation; elementwise.hip period_sum_k)."""
    g = g.contiguous()
    N = g.shape[0]
    out = torch.empty((period,) + tuple(g.shape[1:]), dtype=g.dtype, device=g.device)
    qm = out.numel()
    if g.dtype != BF16 or qm % 8 or N % period:
        return g.reshape(N // period, period, *g.shape[1:]).sum(0, dtype=F32).to(g.dtype)
    _chk(_lib.d3d_period_sum(g.data_ptr(), out.data_ptr(), N // period, qm, _st()), "period_sum")
    return out


def _sgemm(A, B, C, M, N, K, batch, sa, sb, sc, alpha: float = 1.0, beta: float = 0.0) -> None:
    """C_b = alpha A_b B_b + beta C_b over fp32 element-strided views
    (small_gemm.hip); s* = (batch, row, column) strides of each operand."""
    for t in (A, B, C):
        if t.dtype != F32 or not t.is_cuda:
            raise ValueError("_sgemm: fp32 device tensors")
    _chk(_lib.d3d_sgemm_strided(A.data_ptr(), B.data_ptr(), C.data_ptr(), M, N, K, batch, *sa, *sb, *sc, alpha, beta,
                                _st()), "sgemm_strided")


class _CondConv(torch.autograd.Function):
    """Conditioning conv (`xunet.py:292-299,340-350`) on the split ray input:
    MFMA conv over the 51 direction channels (padded to 64) + the constant
    origin half as per-image tap biases (cond.hip).  Same result as the
    144-channel conv; 3x fewer conv FLOPs and half the weight-gradient tiles."""

    @staticmethod
    def forward(ctx, rays_dir, orig_pe, weight, bias, row_bias, residual, stride, res_period, aux=None):
        N, H, W, ICd = rays_dir.shape
        OC, IC = weight.shape[0], weight.shape[1]
        no = orig_pe.shape[1]
        nd = IC - no
        OH, OW = (H - 1) // stride + 1, (W - 1) // stride + 1
        wp = packed_weight_slice(weight, no, nd, ICd)
        # U[n, t, o] = sum_k pe[n, k] W[o, k, t] (origin channels k < no)     [N, 9, OC] fp32
        U = torch.empty(N, 9, OC, dtype=F32, device=rays_dir.device)
        _sgemm(orig_pe, weight.detach(), U, N, OC, no, 9, (0, no, 1), (1, 9, IC * 9), (OC, 9 * OC, 1))
        rb = U.sum(1)
        if row_bias is not None:
            rb = rb + row_bias.float()
        out = torch.empty(N, OH, OW, OC, dtype=BF16, device=rays_dir.device)
        res = residual.contiguous() if residual is not None else None
        # aux: also produce silu(out) -- the FiLM projections' GEMM operand
        # (xunet.py:84) -- from the conv epilogue + the border correction,
        # instead of a separate SiLU pass over the level embedding
        so = torch.empty_like(out) if aux is not None else None
        _conv_fwd(rays_dir, wp, bias, rb.contiguous(), res, out, N, H, W, ICd, ICd, OH, OW, OC, OC, stride, False,
                  1.0, res_period, 9, silu_out=so)
        _chk(_lib.d3d_border_fix(out.data_ptr(), U.data_ptr(), N, H, W, OH, OW, OC, stride, _ptr(so), _st()),
             "border_fix")
        if aux is not None:
            aux["silu"] = so
        ctx.save_for_backward(rays_dir, orig_pe, weight)
        ctx.cfg = (stride, residual is not None, row_bias is not None, bias is not None, res_period)
        ctx.bias_param = bias
        SINK.use(weight, ctx.needs_input_grad[2])
        SINK.use(bias, ctx.needs_input_grad[3])
        return out

    @staticmethod
    def backward(ctx, dy):
        rays_dir, orig_pe, weight = ctx.saved_tensors
        stride, has_res, has_rb, has_b, res_period = ctx.cfg
        g = dy.contiguous()
        N, OH, OW, OC = g.shape
        _, H, W, ICd = rays_dir.shape
        IC, no = weight.shape[1], orig_pe.shape[1]
        nd = IC - no
        bias = ctx.bias_param
        need_w, need_b = ctx.needs_input_grad[2], has_b and ctx.needs_input_grad[3]
        per, tot = _chansum(g, True)                                        # [N, OC], [OC]
        dW = db = None
        if need_w:
            dWd, _ = _wgrad(g, rays_dir, OC, ICd, N, H, W, OH, OW, stride, 9)   # [OC, ICd, 9]
            S = torch.empty(N, 8, OC, dtype=F32, device=g.device)
            _chk(_lib.d3d_border_sums(g.data_ptr(), S.data_ptr(), N, OH, OW, OC, _st()), "border_sums")
            stats = torch.cat([per[:, None], S], 1)                         # [N, 9, OC]
            # dU[n, t, o] = sum_k M[t, k] stats[n, k, o]
            dU = torch.empty(N, 9, OC, dtype=F32, device=g.device)
            _sgemm(_tap_coef(H, W, OH, OW, stride, g.device), stats, dU, 9, OC, 9, N, (0, 9, 1), (9 * OC, OC, 1),
                   (9 * OC, OC, 1))
            # dW[o, k, t] (+)= sum_n dU[n, t, o] pe[n, k]: straight into the gradient
            tw = SINK.target(weight)
            if tw is not None:
                tv = tw.view(OC, IC, 9)
                _sgemm(dU, orig_pe, tv, OC, no, N, 9, (OC, 1, 9 * OC), (0, no, 1), (1, IC * 9, 9), beta=1.0)
                tv[:, no:].add_(dWd[:, :nd])
                SINK.done(weight)
            else:
                dWo = torch.empty(OC, no, 9, dtype=F32, device=g.device)
                _sgemm(dU, orig_pe, dWo, OC, no, N, 9, (OC, 1, 9 * OC), (0, no, 1), (1, no * 9, 9))
                dW = torch.cat([dWo, dWd[:, :nd]], 1).reshape(weight.shape)
        if need_b:
            tb = SINK.target(bias)
            if tb is not None:
                tb.add_(tot)
                SINK.done(bias)
            else:
                db = tot
        drb = per if has_rb else None
        dres = None
        if has_res:
            dres = g if not res_period else _period_sum(g, res_period)
        return None, None, dW, db, drb, dres, None, None, None


def cond_conv(rays_dir, orig_pe, weight, bias, stride, row_bias=None, residual=None, res_period=0, silu_out=False):
    """``silu_out``: the output carries ``_d3d_silu`` = silu(output), produced
    with it (consumed by :func:`film_batch` instead of its SiLU pass)."""
    _need_bf16(rays_dir, residual)
    aux = {} if silu_out else None
    y = _CondConv.apply(rays_dir, orig_pe.float().contiguous(), weight, bias, row_bias, residual, stride,
                        res_period, aux)
    if aux is not None:
        y._d3d_silu = aux["silu"]
    return y


def ray_posenc_dir(R, t, K, H, W, cond_mask, rescale_from=0, ld=64):
    B = R.shape[0]
    Kd = K.to(torch.float64)
    if rescale_from:
        Kd = torch.cat([Kd[:, 0:1] * (W / rescale_from), Kd[:, 1:2] * (H / rescale_from), Kd[:, 2:3]], 1)
    Kinv = _inv3x3(Kd).float().contiguous()
    Rf = R.float().reshape(B * 2, 9).contiguous()
    mask = cond_mask.to(torch.uint8).contiguous()
    out = torch.empty(B * 2, H, W, ld, dtype=BF16, device=R.device)
    _chk(_lib.d3d_ray_dir(Rf.data_ptr(), Kinv.data_ptr(), mask.data_ptr(), out.data_ptr(), B, H, W, ld, _st()),
         "ray_dir")
    return out


def ray_conditioning(R, t, K, H, W, cond_mask, rescale_from=0, ld=64):
    """(direction image [2B,H,W,ld] bf16, origin posenc [2B,93] fp32): the
    inverse intrinsics, mask and origin posenc come from one prep launch
    (rays.hip cond_prep_k), the direction image from ray_dir_k."""
    B = R.shape[0]
    dev = R.device
    Kf = K.float().reshape(B, 9).contiguous()
    tf = t.float().reshape(B * 2, 3).contiguous()
    cm = cond_mask.to(torch.bool).contiguous()
    sx = W / rescale_from if rescale_from else 1.0
    sy = H / rescale_from if rescale_from else 1.0
    Kinv = torch.empty(B, 9, dtype=F32, device=dev)
    mask = torch.empty(B, dtype=torch.uint8, device=dev)
    ope = torch.empty(B * 2, 93, dtype=F32, device=dev)
    _chk(_lib.d3d_cond_prep(Kf.data_ptr(), tf.data_ptr(), cm.data_ptr(), B, float(sx), float(sy), Kinv.data_ptr(),
                            mask.data_ptr(), ope.data_ptr(), _st()), "cond_prep")
    Rf = R.float().reshape(B * 2, 9).contiguous()
    out = torch.empty(B * 2, H, W, ld, dtype=BF16, device=dev)
    _chk(_lib.d3d_ray_dir(Rf.data_ptr(), Kinv.data_ptr(), mask.data_ptr(), out.data_ptr(), B, H, W, ld, _st()),
         "ray_dir")
    return out, ope


# --------------------------------------------------------------- linear ----
def _mm_f32(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    try:
        return torch.mm(a, b, out_dtype=F32)
    except (RuntimeError, TypeError):
        return torch.mm(a, b).float()


def _gemm_ok(M: int, N: int, K: int, lda: int, ldb: int, *ops: Optional[torch.Tensor], res=None) -> bool:
    """Shapes csrc/gemm.hip takes (K % 64 == 0 and >= 128, M % 8 == 0, 16-byte
    rows), and -- for the operand / output tensors given -- the pointer
    conditions d3d_gemm checks at launch (16-byte aligned operands and output,
    8-byte aligned residual), so an odd view takes the caller's library
    fallback instead of failing the launch."""
    if not _lib.d3d_gemm_nt_ok(M, N, K, lda, ldb):
        return False
    if any(t is not None and t.data_ptr() % 16 for t in ops):
        return False
    return res is None or res.data_ptr() % 8 == 0


def gemm_nt(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor, M: int, N: int, K: int, lda: int, ldb: int, ldo: int,
            bias: Optional[torch.Tensor] = None, res: Optional[torch.Tensor] = None, ldr: int = 0,
            alpha: float = 1.0, scale: float = 1.0, gnp: Optional[torch.Tensor] = None, gn_groups: int = 0,
            gn_hw: int = 0, dsilu_of: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out[n][m] = (alpha * sum_k a[m][k] b[n][k] + bias[m] + res[n][m]) * scale on
    the gfx950 GEMM (csrc/gemm.hip; bf16 operands / output, fp32 or bf16 bias).
    ``gnp``: the output's GroupNorm partial statistics (groups ``gn_groups``
    over images of ``gn_hw`` rows) from the same epilogue.  ``dsilu_of``
    (row stride ``ldr``): instead out = alpha * acc * dsilu(dsilu_of[n][m]) --
    an input gradient through a SiLU whose pre-activation is dsilu_of."""
    if bias is not None:
        assert bias.dtype in (F32, BF16) and bias.is_contiguous()
    epi = 0 if dsilu_of is None else 1
    r = res if dsilu_of is None else dsilu_of
    _chk(_lib.d3d_gemm(a.data_ptr(), b.data_ptr(), out.data_ptr(), _ptr(bias),
                       int(bias is not None and bias.dtype == BF16), _ptr(r), M, N, K, lda, ldb, ldo, ldr or ldo,
                       float(alpha), float(scale), _ptr(gnp), int(gn_groups), int(gn_hw), epi, _st()), "gemm")
    return out


class _Linear(torch.autograd.Function):
    """Per-pixel dense layer on the gfx950 GEMM: forward with the bias /
    residual / scale (+ GroupNorm statistics) epilogue, input gradient against
    the cached transposed weight, weight gradient on the split-K MFMA kernel
    (the reduction runs over every pixel of the batch)."""

    @staticmethod
    def forward(ctx, x, weight, bias, residual, out_scale, res_slot=None, in_slot=None, gn=None):
        shp = x.shape
        x2 = x.reshape(-1, shp[-1])
        P, IC = x2.shape
        OC = weight.shape[0]
        L = shp[1] if len(shp) == 3 else 0
        r = residual.reshape(P, OC).contiguous() if residual is not None else None
        if x2.is_contiguous() and _gemm_ok(OC, P, IC, IC, IC, x2, res=r):
            gnp = None
            if gn is not None and L and L % 64 == 0 and OC % gn["groups"] == 0 and \
                    OC // gn["groups"] in (4, 8, 16, 32):
                gnp = torch.empty((P // L) * gn["groups"] * (L // 64) * 2, dtype=F32, device=x.device)
            y = torch.empty(P, OC, dtype=BF16, device=x.device)
            gemm_nt(bf16_weight(weight), x2, y, OC, P, IC, IC, IC, OC,
                    bias=bias.detach() if bias is not None else None, res=r, scale=float(out_scale), gnp=gnp,
                    gn_groups=gn["groups"] if gnp is not None else 0, gn_hw=L)
            if gnp is not None:
                gn["part"] = (gnp, L // 64)
        else:
            _fallback("linear", f"P={P} IC={IC} OC={OC} (library GEMM)")
            wb = bf16_weight(weight)
            y = torch.addmm(bf16_weight(bias), x2, wb.t()) if bias is not None else torch.mm(x2, wb.t())
            if residual is not None or out_scale != 1.0:
                _chk(_lib.d3d_add_scale(y.data_ptr(), _ptr(r), y.data_ptr(), float(out_scale), y.numel(), _st()),
                     "add_scale")
        ctx.save_for_backward(x2, weight)
        ctx.cfg = (shp, out_scale, residual is not None, bias is not None)
        ctx.bias_param = bias
        ctx.slots = (res_slot, in_slot)
        if shp[-1] % 8 == 0 and OC % 8 == 0:
            SINK.use(weight, ctx.needs_input_grad[1])
            SINK.use(bias, ctx.needs_input_grad[2])
        return y.reshape(*shp[:-1], OC)

    @staticmethod
    def backward(ctx, dy):
        x2, weight = ctx.saved_tensors
        shp, scale, has_res, has_b = ctx.cfg
        g = dy.reshape(-1, dy.shape[-1])
        OC, IC = g.shape[-1], x2.shape[-1]
        rows = g.shape[0]
        dW = db = None
        bias = ctx.bias_param
        need_w, need_b = ctx.needs_input_grad[1], has_b and ctx.needs_input_grad[2]
        res_slot, in_slot = ctx.slots
        # gradient of out = scale * (x W^T + b + residual) is scale * dy: the
        # scale rides on the GEMM alpha, the wgrad reduction and the residual
        # hand-off instead of a scaled copy of dy (same rule as _Conv)
        mma = IC % 8 == 0 and OC % 8 == 0
        lazy = scale != 1.0 and mma and need_w and \
            (not has_res or not ctx.needs_input_grad[3] or (res_slot is not None and not res_slot.consumed))
        ks = 1.0
        if scale != 1.0 and not lazy:
            gs = torch.empty_like(g)
            _chk(_lib.d3d_add_scale(g.contiguous().data_ptr(), None, gs.data_ptr(), float(scale), g.numel(), _st()),
                 "scale")
            g = gs
        elif lazy:
            ks = scale
        if ctx.needs_input_grad[0]:
            OCp = _up(OC, 64)
            if g.is_contiguous() and _gemm_ok(IC, rows, OC, OCp, OC, g):
                dx = torch.empty(rows, IC, dtype=g.dtype, device=g.device)
                gemm_nt(packed_weight(weight, True, 1), g, dx, IC, rows, OC, OCp, OC, IC, alpha=float(ks))
            else:
                _fallback("linear dgrad", f"P={rows} IC={IC} OC={OC} (library GEMM)")
                dx = torch.empty(rows, IC, dtype=g.dtype, device=g.device).addmm_(g, bf16_weight(weight), beta=0.0,
                                                                                   alpha=ks)
            dx = dx.reshape(shp)
        else:
            dx = None
        if mma and need_w:
            g = g.contiguous()
            g4, x4 = g.reshape(rows, 1, 1, OC), x2.contiguous().reshape(rows, 1, 1, IC)
            tw = SINK.target(weight)
            tb = SINK.target(bias) if need_b else None
            if tw is not None and (not need_b or tb is not None):
                def job(g4=g4, x4=x4, tw=tw, tb=tb, ks=ks):
                    _wgrad(g4, x4, OC, IC, rows, 1, 1, 1, 1, 1, 1, dW=tw.view(OC, IC, 1), db=tb, accumulate=True,
                           scale=ks)
                spec = wgrad_job(g4, x4, OC, IC, rows, 1, 1, 1, tw, tb, ks)
                SINK.submit(g.device, job, (g4, x4), (weight, bias if need_b else None), spec=spec)
            else:
                dW, db = _wgrad(g4, x4, OC, IC, rows, 1, 1, 1, 1, 1, 1, want_bias=need_b, scale=ks)
                dW = dW.reshape(weight.shape)
        elif mma:
            if need_b:
                db = _chansum(g.contiguous().reshape(1, rows, 1, OC), False)[1]
        else:
            if ctx.needs_input_grad[1]:
                dW = _mm_f32(g.t(), x2).reshape(weight.shape)
            if has_b and ctx.needs_input_grad[2]:
                db = g.float().sum(0)
        dres = None
        if has_res and ctx.needs_input_grad[3] and (res_slot is None or not res_slot.deposit(g, ks)):
            assert ks == 1.0
            dres = g.reshape(*shp[:-1], OC)
        if dx is not None and in_slot is not None and in_slot.deposit(dx):
            dx = None
        return dx, dW, db, dres, None, None, None, None


# Explicit split-K of the hipBLASLt FiLM weight-gradient product: the pixel
# reduction (K up to 1M rows at bs128) as a batch of ``nsl`` GEMMs whose fp32
# partial products the scatter kernel sums while it writes the parameter
# gradients (no separate sum pass).  hipBLASLt's own choice for the single
# mixed-precision GEMM runs 640-950 TF/s on these shapes; 8 (4 for the
# smallest level) slabs run 910-1160 TF/s (profiles/film_wgrad_split_r2.txt).
def wgrad_tn(dy: torch.Tensor, x: torch.Tensor, splits: int = 0):
    """Split-K weight-gradient GEMM (wgrad_gemm.hip): ``dy [P, M]`` (row
    stride ``dy.stride(0)``) and ``x [P, N]`` bf16 -> ``(ws [used, M, N],
    bws [used, M], used)`` fp32 partials whose sums over the first axis are
    ``dy^T @ x`` and the column sums of ``dy`` (bws: ``2 cdiv(N, 256)`` partial
    rows per split)."""
    P, M = dy.shape
    N = x.shape[1]
    ldy, ldx = dy.stride(0), x.stride(0)
    if dy.stride(1) != 1 or x.stride(1) != 1 or x.shape[0] != P:
        raise ValueError("wgrad_tn: row-major [P, C] operands")
    if not splits:
        splits = _lib.d3d_wgrad_tn_plan(M, N, P, ldy, ldx)
    if splits <= 0:
        raise ValueError(f"wgrad_tn: unsupported shape P={P} M={M} N={N}")
    bpr = 2 * ((N + 255) // 256)                 # bias partial rows per split
    buf = torch.empty(splits * M * N + splits * bpr * M, dtype=F32, device=dy.device)
    ws, bws = buf[: splits * M * N], buf[splits * M * N:]
    used = _lib.d3d_wgrad_tn(dy.data_ptr(), x.data_ptr(), ws.data_ptr(), bws.data_ptr(), M, N, P, ldy, ldx, splits,
                             _st())
    if used <= 0:
        raise RuntimeError(f"d3d_wgrad_tn failed ({used})")
    return ws.view(splits, M, N)[:used], bws.view(splits * bpr, M)[: used * bpr], used


def _film_wgrad_product(dy: torch.Tensor, x2: torch.Tensor):
    """``dy^T @ x2`` in fp32 as ``nsl`` stacked partial products."""
    rows, S = dy.shape
    K = x2.shape[1]
    nsl = 8 if rows >= 32768 else 4 if rows >= 8192 else 1
    if nsl > 1 and rows % nsl == 0:
        try:
            a = dy.view(nsl, rows // nsl, S).transpose(1, 2)
            return torch.bmm(a, x2.view(nsl, rows // nsl, K), out_dtype=F32), nsl
        except (RuntimeError, TypeError):
            pass
    return _mm_f32(dy.t(), x2), 1


class _FiLMSlot:
    """Shared gradient buffer of one level-batched FiLM projection: each
    GN-FiLM backward deposits its d(scale|shift) into its column slice."""

    def __init__(self, shape, width, device, want_events=False):
        self.shape, self.width, self.device = tuple(shape), width, device
        self.buf = None
        self.want_events = want_events      # forward: one GEMM + ready event per block (film_batch)
        self.events = []
        self.x2 = None                      # silu(e) [P, K]: the weight gradients' second operand
        self.blocks = {}                    # column offset -> (weight, bias, width): early weight gradients
        self.groups = []                    # block offsets per weight-gradient job (contiguous columns)
        self.ready = set()                  # offsets whose d(scale|shift) is written
        self.early = set()                  # offsets whose weight gradient is submitted

    def grad_slice(self, off: int, C: int) -> torch.Tensor:
        if self.buf is None:
            self.buf = torch.empty(*self.shape, self.width, dtype=BF16, device=self.device)
        return self.buf[..., off: off + 2 * C]

    def block_ready(self, off: int) -> None:
        """The GN-FiLM backward of the block at column ``off`` has written its
        d(scale|shift) slice of :attr:`buf`: once every block of its group
        has, submit the group's weight gradient (it overlaps the rest of the
        backward)."""
        if off not in self.blocks or self.buf is None:
            return
        self.ready.add(off)
        for grp in self.groups:
            if grp[0] not in self.early and all(o in self.ready for o in grp):
                if _film_group_wgrad(self.buf.view(-1, self.width), grp, self.blocks, self.x2):
                    self.early.update(grp)


def _film_group_wgrad(dy: torch.Tensor, grp, blocks, x2: torch.Tensor, inline: bool = False) -> bool:
    """The weight / bias gradients of FiLM blocks ``grp`` (column offsets of
    contiguous blocks of the level's [P, S] d(scale|shift) buffer ``dy``) as
    ONE sink job: split-K MFMA GEMM over their columns against ``x2`` =
    silu(e), then the reduction scatters rows into each block's gradients.
    False when a parameter is not sink-managed or the GEMM cannot take the
    shape (the level-wide job then covers the blocks)."""
    ps = [blocks[o] for o in grp]
    tw = [SINK.target(w) for w, _, _ in ps]
    tb = [SINK.target(b) for _, b, _ in ps]
    if any(t is None for t in tw + tb):
        return False
    c0, c1 = grp[0], grp[-1] + ps[-1][2]
    cols = dy[:, c0:c1]
    rows, K = x2.shape
    sp = _lib.d3d_wgrad_tn_plan(c1 - c0, K, rows, cols.stride(0), K)
    if sp <= 0:
        return False
    n = len(grp)

    def job(cols=cols, x2=x2, tw=tw, tb=tb, sp=sp):
        ws, bws, used = wgrad_tn(cols, x2, sp)
        row0 = (ctypes.c_int * n)(*[o - c0 for o in grp])
        wdst = (ctypes.c_void_p * n)(*[t.data_ptr() for t in tw])
        bdst = (ctypes.c_void_p * n)(*[t.data_ptr() for t in tb])
        _chk(_lib.d3d_wgrad_scatter(ws.data_ptr(), c1 - c0, K, used, 1, bws.data_ptr(), bws.shape[0], n, row0, wdst,
                                    bdst, _st()), "film_group_wgrad")
    params = [p for w, b, _ in ps for p in (w, b)]
    if inline:
        job()
        for p_ in params:
            SINK.done(p_)
    else:
        SINK.submit(x2.device, job, (cols, x2), params, work=2.0 * rows * (c1 - c0) * K)
    return True


class _FiLMBatch(torch.autograd.Function):
    """All FiLM projections that read one level's conditioning embedding
    (`xunet.py:74-87`, ``dense(silu(emb))`` per ResnetBlock) as ONE GEMM
    ``silu(e)[P, emb_ch] x [emb_ch, sum 2C_i]``: the 1024-channel embedding is
    read once instead of once per block.  Backward: the input gradient is one
    GEMM over the concatenated d(scale|shift) whose epilogue applies the SiLU
    derivative of the pre-activation ``e`` (no separate dsilu pass, no
    d(silu(e)) tensor); the weight gradient is one split-K launch whose
    reduction scatters rows into each block's parameter gradient."""

    @staticmethod
    def forward(ctx, e, slot, n, se, split, *wb):
        Ws, Bs = wb[:n], wb[n:]
        shp = e.shape
        K = shp[-1]
        e2 = e.reshape(-1, K)
        P = e2.shape[0]
        if se is not None:
            x2 = se.reshape(-1, K)                          # silu(e) from the producing conv's epilogue
        else:
            x2 = torch.empty_like(e2)                       # silu(e): the GEMM operand, kept for the wgrad
            _chk(_lib.d3d_silu(e2.data_ptr(), x2.data_ptr(), e2.numel(), _st()), "silu")
        wcat = bf16_cat(Ws, "filmW")
        bcat = bf16_cat(list(Bs), "filmB")
        S = wcat.shape[0]
        y = torch.empty(P, S, dtype=BF16, device=e.device)
        if _gemm_ok(S, P, K, K, K, x2) and slot.want_events:
            # one GEMM per block's column slice, each followed by an event:
            # the trunk's block i waits for its own modulation only, so the
            # conditioning stream computes slice i + 1 while block i runs
            # (the whole-level GEMM made level 0 wait ~4 ms at bs128)
            off = 0
            slot.events = []
            for wd in [w.shape[0] for w in Ws]:
                gemm_nt(wcat[off:off + wd], x2, y[:, off:], wd, P, K, K, K, S, bias=bcat[off:off + wd])
                ev = torch.cuda.Event()
                ev.record()
                slot.events.append(ev)
                off += wd
        elif _FILM_BLAS and P * S * K >= (1 << 37) and x2.is_contiguous():
            # the big level projections (a plain GEMM + bias): hipBLASLt's
            # kernels run these 8-17 % faster than gemm_fw_k's 256 x 256 tile
            # (tools/kbench_gemm.py "film fwd"; profiles/r5/ab_gemm_small_k.txt)
            torch.addmm(bcat, x2, wcat.t(), out=y)
        elif _gemm_ok(S, P, K, K, K, x2):
            gemm_nt(wcat, x2, y, S, P, K, K, K, S, bias=bcat)
        else:
            _fallback("film_batch", f"P={P} K={K} S={S} (library GEMM)")
            torch.addmm(bcat, x2, wcat.t(), out=y)
        ctx.save_for_backward(x2, e2)
        ctx.n, ctx.slot, ctx.shp = n, slot, shp
        ctx.params = (Ws, Bs)
        ctx.widths = [w.shape[0] for w in Ws]
        early_on = _FILM_EARLY == 2 or (_FILM_EARLY == 1 and torch.cuda.is_current_stream_capturing())
        if early_on and _FILM_WGRAD == "tn" and 0 < split < n and all(ctx.needs_input_grad[5:5 + 2 * n]) and \
                all(SINK.managed(p) for p in wb):
            slot.x2 = x2
            offs = [0]
            for w, b, wd in zip(Ws, Bs, ctx.widths):
                slot.blocks[offs[-1]] = (w, b, wd)
                offs.append(offs[-1] + wd)
            slot.groups = [offs[:split], offs[split:n]]
        for i, (w, b) in enumerate(zip(Ws, Bs)):
            SINK.use(w, ctx.needs_input_grad[5 + i])
            SINK.use(b, ctx.needs_input_grad[5 + n + i])
        y = y.view(*shp[:-1], S)
        outs, off = [], 0
        for wd in ctx.widths:
            outs.append(y[..., off: off + wd])
            off += wd
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gs):
        x2, e2 = ctx.saved_tensors
        n, slot, shp = ctx.n, ctx.slot, ctx.shp
        Ws, Bs = ctx.params
        S = sum(ctx.widths)
        buf = slot.buf
        offs = [0]
        for wd in ctx.widths:
            offs.append(offs[-1] + wd)
        ok = buf is not None
        if ok:
            for g, o in zip(gs, offs):
                if g is None or g.data_ptr() != buf.data_ptr() + 2 * o or g.stride(-2) != S:
                    ok = False
                    break
        if ok:
            dy = buf.view(-1, S)
            # written by the GN-FiLM backwards (trunk stream), read here -- on
            # the conditioning stream when that is on (models/xunet.py)
            buf.record_stream(torch.cuda.current_stream())
        else:
            dy = torch.zeros(x2.shape[0], S, dtype=BF16, device=x2.device)
            for g, o, wd in zip(gs, offs, ctx.widths):
                if g is not None:
                    dy[:, o: o + wd].copy_(g.reshape(-1, wd))
        early, blocks, groups = slot.early, slot.blocks, slot.groups
        slot.buf, slot.x2, slot.blocks, slot.groups, slot.ready, slot.early = None, None, {}, [], set(), set()
        rows, K = x2.shape
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(rows, K, dtype=BF16, device=x2.device)
            if _gemm_ok(K, rows, S, S, S, dy, e2):
                # d e = (dy @ Wcat) * dsilu(e), the SiLU derivative in the epilogue
                gemm_nt(bf16_catT(Ws, "filmWT"), dy, dx, K, rows, S, S, S, K, dsilu_of=e2, ldr=K)
            else:
                _fallback("film_batch dgrad", f"P={rows} K={K} S={S} (library GEMM)")
                ds = torch.mm(dy, bf16_cat(Ws, "filmW"))
                _chk(_lib.d3d_dsilu(e2.data_ptr(), ds.data_ptr(), dx.data_ptr(), dx.numel(), _st()), "dsilu")
            dx = dx.view(shp)
        grads_w, grads_b = [None] * n, [None] * n
        need_w = any(ctx.needs_input_grad[5: 5 + n])
        if need_w and early:
            # a group's weight gradients were submitted by its GN-FiLM
            # backwards (_FiLMSlot.block_ready); the rest go one job per group
            for grp in groups:
                if grp[0] not in early and not _film_group_wgrad(dy, grp, blocks, x2, inline=_FILM_INLINE):
                    raise RuntimeError("FiLM weight gradient: early and level-wide jobs mixed")
            need_w = False
        if need_w:
            tw = [SINK.target(w) for w in Ws]
            tb = [SINK.target(b) for b in Bs]
            direct = all(t is not None for t in tw + tb)
            if not direct:
                tw = [torch.zeros(w.shape, dtype=F32, device=x2.device) for w in Ws]
                tb = [torch.zeros(b.shape, dtype=F32, device=x2.device) for b in Bs]
            _ensure_impl()
            sp_tn = _lib.d3d_wgrad_tn_plan(S, K, rows, S, K) if _FILM_WGRAD == "tn" else 0

            def job():
                row0 = (ctypes.c_int * n)(*offs[:n])
                wd = (ctypes.c_void_p * n)(*[t.data_ptr() for t in tw])
                bd = (ctypes.c_void_p * n)(*[t.data_ptr() for t in tb])
                if sp_tn:
                    # fp32 split slabs + bias partials from one MFMA launch, then the
                    # reduction scatters rows into each block's parameter gradients
                    ws, bws, used = wgrad_tn(dy, x2, sp_tn)
                    _chk(_lib.d3d_wgrad_scatter(ws.data_ptr(), S, K, used, 1, bws.data_ptr(), bws.shape[0], n, row0,
                                                wd, bd, _st()), "film_wgrad_scatter")
                elif _FILM_WGRAD == "blas":
                    # wide FiLM weight gradients ([S, 1024] over every pixel of the
                    # level): the fp32 [S, K] product (stacked split-K slabs) and
                    # the bias column sums are scattered into the parameters'
                    # gradients in one launch
                    prod, nsl = _film_wgrad_product(dy, x2)
                    nimg = 64 if rows % 64 == 0 else 1
                    _, bsum = _chansum(dy.view(nimg, rows // nimg, 1, S), False)
                    _chk(_lib.d3d_wgrad_scatter(prod.data_ptr(), S, K, nsl, 1, bsum.data_ptr(), 1, n, row0, wd, bd,
                                                _st()), "film_wgrad_scatter")
                else:
                    sp, pps = ctypes.c_int(), ctypes.c_int()
                    _lib.d3d_conv_wgrad_plan3(rows, 1, 1, 1, 1, S, K, 1, 1, ctypes.byref(sp), ctypes.byref(pps))
                    ws = torch.empty(sp.value * S * K + 2 * sp.value * S, dtype=F32, device=x2.device)
                    _chk(_lib.d3d_conv_wgrad_seg(dy.data_ptr(), x2.data_ptr(), ws.data_ptr(), rows, 1, 1, K, 1, 1, S,
                                                 1, sp.value, pps.value, 1, 1, n, row0, wd, bd, _st()), "film_wgrad")
            if direct and _FILM_INLINE:
                job()
                for p_ in [p for wb in zip(Ws, Bs) for p in wb]:
                    SINK.done(p_)
            elif direct:
                SINK.submit(x2.device, job, (dy, x2), [p for wb in zip(Ws, Bs) for p in wb], work=2.0 * rows * S * K)
            else:
                job()
                grads_w = [t.view(w.shape) for t, w in zip(tw, Ws)]
                grads_b = tb
        return (dx, None, None, None, None, *grads_w, *grads_b)


def film_batch(emb, weights, biases, block_events=False, split=0):
    """Level-batched FiLM projections ``dense_i(silu(emb))`` of the per-level
    pre-activation embedding -> tuple of ``[N,H,W,2C_i]`` modulations (column
    slices of one GEMM output; GN-FiLM reads them strided).  ``block_events``:
    one GEMM per block with a ready event attached to each output as
    ``_d3d_ready`` (consumers on another stream wait per block).  ``split``:
    the weight gradients of blocks ``[split:]`` (the decoder's, done first in
    the backward) run as their own job as soon as those blocks' backwards
    are through; 0: one job for the level."""
    _need_bf16(emb)
    K = emb.shape[-1]
    widths = [w.shape[0] for w in weights]
    if K % 8 or any(wd % 8 for wd in widths) or len(weights) > 16:
        _fallback("film_batch", f"K={K} widths={widths}")
        se = silu(emb)
        return tuple(linear(se, w, b) for w, b in zip(weights, biases))
    slot = _FiLMSlot(emb.shape[:-1], sum(widths), emb.device, want_events=bool(block_events))
    se = getattr(emb, "_d3d_silu", None)          # silu(emb) written by the conditioning conv (cond_conv)
    if se is not None and (se.shape != emb.shape or not se.is_contiguous() or not emb.is_contiguous()):
        se = None
    outs = _FiLMBatch.apply(emb.contiguous(), slot, len(weights), se, int(split), *weights, *biases)
    off = 0
    for i, (o, wd) in enumerate(zip(outs, widths)):
        o._d3d_slot = (slot, off)
        if slot.events:
            o._d3d_ready = slot.events[i]
        off += wd
    slot.events = []
    return outs


_EPI_GN_STATS = True     # GroupNorm statistics from the producing epilogue


def linear(x, weight, bias, residual=None, out_scale=1.0, res_slot=None, in_slot=None, gn_groups=0):
    """Per-pixel dense layer on the gfx950 GEMM (fused bias / residual / scale
    epilogue; input gradient on the same kernel, weight gradient -- a
    reduction over every pixel of the batch -- on the split-K MFMA kernel).
    ``gn_groups`` (x of shape [N, L, C]): the epilogue also emits the partial
    statistics of the GroupNorm that reads the output (attached as
    ``_d3d_gnpart``; see :func:`carry_gn_stats` across reshapes)."""
    _need_bf16(x, residual)
    if gn_groups and x.dim() == 3 and gn_img_ok(x.shape[1], weight.shape[0], int(gn_groups), x.shape[0]):
        gn_groups = 0                   # the consumer's whole-image kernel makes its own statistics
    gn = {"groups": int(gn_groups)} if (gn_groups and _EPI_GN_STATS) else None
    y = _Linear.apply(x, weight, bias, residual, out_scale, res_slot, in_slot, gn)
    if gn is not None and "part" in gn:
        y._d3d_gnpart = (gn["part"][0], int(gn_groups), gn["part"][1])
    return y


# ------------------------------------- attention output map (merged) ----
# AttnBlock: out_proj (inside nn.MultiheadAttention, `xunet.py:175`) is
# followed by the zero-init 1x1 `linear` (`xunet.py:190,217`) with nothing in
# between: y = (a W_out^T + b_out) W_lin^T + b_lin = a W^T + b with
# W = W_lin W_out, b = W_lin b_out + b_lin.  The forward runs ONE GEMM with the
# merged operand and the input gradient ONE GEMM against W^T: the trunk's
# critical path loses one GEMM each way per attention block.  The weight
# gradients need the layers' own intermediates: o = a W_out^T + b_out and
# do = dy W_lin are recomputed by two GEMMs inside the weight-gradient job,
# i.e. on the weight-gradient stream, off the critical path -- or, when the
# pixel count is large against C (rows >= D3D_ATTN_SPLIT x C, bs128's 16x16
# level), from ONE reduction M = dy^T a (+ colsum dy) split back onto the two
# layers by C x C products (cheaper than two rows x C x C GEMMs there; at bs16
# the fp32 products, latency-bound at ~125 us per block, measured -5..-7 %):
#     dW_out = W_lin^T M,   db_out = W_lin^T colsum,
#     dW_lin = M W_out^T + colsum b_out^T,   db_lin = colsum.
# W / W^T / b are derived operands: recomputed for every registered block by
# one table launch (small_gemm.hip sgemm_jobs_k) after each optimizer update
# (captured into the update graphs like the operand repack) or lazily when a
# parameter changed.
class _SgJob(ctypes.Structure):
    _fields_ = [("A", ctypes.c_void_p), ("B", ctypes.c_void_p), ("C", ctypes.c_void_p), ("Cb", ctypes.c_void_p),
                ("CbT", ctypes.c_void_p), ("u", ctypes.c_void_p), ("v", ctypes.c_void_p),
                ("sam", ctypes.c_long), ("sak", ctypes.c_long), ("sbk", ctypes.c_long), ("sbn", ctypes.c_long),
                ("scm", ctypes.c_long), ("scn", ctypes.c_long), ("M", ctypes.c_int), ("N", ctypes.c_int),
                ("K", ctypes.c_int), ("ldb", ctypes.c_int), ("ldbt", ctypes.c_int), ("tile0", ctypes.c_int),
                ("alpha", ctypes.c_float), ("beta", ctypes.c_float)]


assert ctypes.sizeof(_SgJob) == 136


def _sg(A=None, B=None, C=None, Cb=None, CbT=None, u=None, v=None, sam=0, sak=0, sbk=0, sbn=0, scm=0, scn=0,
        M=1, N=1, K=1, ldb=0, ldbt=0, alpha=1.0, beta=0.0) -> dict:
    return dict(A=A, B=B, C=C, Cb=Cb, CbT=CbT, u=u, v=v, sam=sam, sak=sak, sbk=sbk, sbn=sbn, scm=scm, scn=scn, M=M,
                N=N, K=K, ldb=ldb, ldbt=ldbt, alpha=alpha, beta=beta)


class _SgTable:
    """A device-resident job table for d3d_sgemm_jobs (built eagerly, before
    any capture; the tensors it points at must outlive it)."""

    def __init__(self, jobs):
        arr = (_SgJob * len(jobs))()
        tile = 0
        for i, j in enumerate(jobs):
            r = arr[i]
            for k, val in j.items():
                if k in ("A", "B", "C", "Cb", "CbT", "u", "v"):
                    setattr(r, k, val.data_ptr() if val is not None else None)
                else:
                    setattr(r, k, val)
            r.tile0 = tile
            tile += ((j["M"] + 63) // 64) * ((j["N"] + 63) // 64)
        host = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
        self.dev = host.to("cuda")
        self.n, self.tiles = len(jobs), tile

    def run(self):
        _chk(_lib.d3d_sgemm_jobs(self.dev.data_ptr(), self.n, self.tiles, _st()), "sgemm_jobs")


class _AttnPair:
    """Derived operands and gradient scratch of one AttnBlock's merged map."""

    def __init__(self, W_out, b_out, W_lin, b_lin):
        C = W_out.shape[0]
        dev = W_out.device
        self.params = (W_out, b_out, W_lin, b_lin)
        self.C = C
        self.Wm = torch.empty(C, C, dtype=BF16, device=dev)       # merged weight (forward A operand)
        self.WmT = torch.empty(C, C, dtype=BF16, device=dev)      # its transpose (input-gradient A operand)
        self.bm = torch.empty(C, dtype=F32, device=dev)
        self.M = self.dcol = None                                    # dy^T a, colsum dy (split backward)
        self.tok = None
        self.bwd = {}                                                # (grad target ptrs) -> _SgTable
        self.scratch = None          # persistent gradient targets when the sink does not own the parameters

    def token(self):
        return (_EPOCH[0],) + tuple(p._version for p in self.params)

    def fwd_jobs(self):
        W_out, b_out, W_lin, b_lin = self.params
        C = self.C
        wl = W_lin.detach().reshape(C, C)
        return [_sg(A=wl, B=W_out.detach(), Cb=self.Wm, CbT=self.WmT, sam=C, sak=1, sbk=C, sbn=1, M=C, N=C, K=C,
                    ldb=C, ldbt=C),
                _sg(A=wl, B=b_out.detach(), C=self.bm, u=b_lin.detach(), sam=C, sak=1, sbk=1, sbn=0, scm=1, scn=0,
                    M=C, N=1, K=C)]

    def bwd_table(self, tw_out, tb_out, tw_lin, tb_lin, cache=True):
        key = (tw_out.data_ptr(), tb_out.data_ptr(), tw_lin.data_ptr(), tb_lin.data_ptr())
        t = self.bwd.get(key) if cache else None
        if t is None:
            W_out, b_out, W_lin, b_lin = self.params
            C = self.C
            if self.M is None:
                self.M = torch.empty(C, C, dtype=F32, device=W_out.device)
                self.dcol = torch.empty(C, dtype=F32, device=W_out.device)
            wl = W_lin.detach().reshape(C, C)
            t = _SgTable([
                # dW_out += W_lin^T M ; db_out += W_lin^T colsum
                _sg(A=wl, B=self.M, C=tw_out, sam=1, sak=C, sbk=C, sbn=1, scm=C, scn=1, M=C, N=C, K=C, beta=1.0),
                _sg(A=wl, B=self.dcol, C=tb_out, sam=1, sak=C, sbk=1, sbn=0, scm=1, scn=0, M=C, N=1, K=C, beta=1.0),
                # dW_lin += M W_out^T + colsum b_out^T ; db_lin += colsum
                _sg(A=self.M, B=W_out.detach(), C=tw_lin, u=self.dcol, v=b_out.detach(), sam=C, sak=1, sbk=1, sbn=C,
                    scm=C, scn=1, M=C, N=C, K=C, beta=1.0),
                _sg(C=tb_lin, u=self.dcol, scm=1, scn=0, M=C, N=1, K=0, beta=1.0)])
            if cache:
                self.bwd[key] = t
        return t



# split backward (one dy^T a reduction + C x C products) when rows >= this x C
_ATTN_SPLIT = int(os.environ.get("D3D_ATTN_SPLIT", "64"))
# below that, merge with the recomputing backward (measured neutral at bs16) or
# keep the two layers (default)
_ATTN_SMALL = os.environ.get("D3D_ATTN_MERGE_SMALL", "0") == "1"
# ... or from this many rows per channel (32: the 8x8 level at 256 images,
# measured +0.2-0.3 % at bs128 -- the size of the A/A ordering bias of the
# same runs, so off by default; profiles/r6/knob_sweep_b128.txt)
_ATTN_SMALL_MIN = int(os.environ.get("D3D_ATTN_MERGE_SMALL_MIN", str(1 << 30)))
_ATTN_PAIRS: Dict[Tuple[int, int], _AttnPair] = {}
_ATTN_TABLE = [None, -1]         # forward-refresh table over every registered pair, its registry size


def _attn_refresh() -> None:
    """Recompute every registered block's merged operands (one launch)."""
    if not _ATTN_PAIRS:
        return
    if _ATTN_TABLE[1] != len(_ATTN_PAIRS):
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("attention merge table built inside a graph capture")
        _ATTN_TABLE[0] = _SgTable([j for pr in _ATTN_PAIRS.values() for j in pr.fwd_jobs()])
        _ATTN_TABLE[1] = len(_ATTN_PAIRS)
    _ATTN_TABLE[0].run()
    for pr in _ATTN_PAIRS.values():
        pr.tok = pr.token()


def _attn_pair(W_out, b_out, W_lin, b_lin) -> _AttnPair:
    key = (W_out.data_ptr(), W_lin.data_ptr())
    pr = _ATTN_PAIRS.get(key)
    if pr is None or pr.params[0] is not W_out or pr.params[2] is not W_lin:
        pr = _ATTN_PAIRS[key] = _AttnPair(W_out, b_out, W_lin, b_lin)
    if pr.tok != pr.token() and not torch.cuda.is_current_stream_capturing():
        _attn_refresh()
    return pr


class _AttnOut(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, W_out, b_out, W_lin, b_lin, residual, out_scale, res_slot, gn):
        pr = _attn_pair(W_out, b_out, W_lin, b_lin)
        N_, L, C = a.shape
        a2 = a.reshape(-1, C)
        P = a2.shape[0]
        r = residual.reshape(P, C).contiguous() if residual is not None else None
        gnp = None
        if gn is not None and L % 64 == 0 and C % gn["groups"] == 0 and C // gn["groups"] in (4, 8, 16, 32):
            gnp = torch.empty((P // L) * gn["groups"] * (L // 64) * 2, dtype=F32, device=a.device)
        y = torch.empty(P, C, dtype=BF16, device=a.device)
        gemm_nt(pr.Wm, a2, y, C, P, C, C, C, C, bias=pr.bm, res=r, scale=float(out_scale), gnp=gnp,
                gn_groups=gn["groups"] if gnp is not None else 0, gn_hw=L)
        if gnp is not None:
            gn["part"] = (gnp, L // 64)
        ctx.save_for_backward(a2)
        ctx.pr, ctx.scale, ctx.has_res, ctx.res_slot, ctx.shp = pr, float(out_scale), residual is not None, \
            res_slot, a.shape
        for i, p_ in enumerate((W_out, b_out, W_lin, b_lin)):
            SINK.use(p_, ctx.needs_input_grad[1 + i])
        return y.view(N_, L, C)

    @staticmethod
    def backward(ctx, dy):
        (a2,) = ctx.saved_tensors
        pr, scale, slot = ctx.pr, ctx.scale, ctx.res_slot
        C = pr.C
        g = dy.reshape(-1, C).contiguous()
        rows = g.shape[0]
        # the scale of out = scale * (...) rides on the GEMM alpha, the reduction
        # and the residual hand-off (as _Linear); a scaled copy only when the
        # residual's gradient must be returned to autograd
        lazy = not ctx.has_res or not ctx.needs_input_grad[5] or (slot is not None and not slot.consumed)
        if scale != 1.0 and not lazy:
            gs = torch.empty_like(g)
            _chk(_lib.d3d_add_scale(g.data_ptr(), None, gs.data_ptr(), scale, g.numel(), _st()), "scale")
            g, ks = gs, 1.0
        else:
            ks = scale
        da = None
        if ctx.needs_input_grad[0]:
            da = torch.empty(rows, C, dtype=BF16, device=g.device)
            gemm_nt(pr.WmT, g, da, C, rows, C, C, C, C, alpha=ks)
            da = da.view(ctx.shp)
        grads = [None] * 4
        if any(ctx.needs_input_grad[1:5]):
            W_out, b_out, W_lin, b_lin = pr.params
            ps = (W_out, b_out, W_lin, b_lin)
            tgt = [SINK.target(p_) for p_ in ps]
            direct = all(t is not None for t in tgt)
            split = rows >= _ATTN_SPLIT * C
            if not direct and split:
                # persistent targets: the split table (a device job table, built by
                # a host-to-device copy) is built once for them, never per backward
                # (nor inside a graph capture); the results leave as copies
                if pr.scratch is None or pr.scratch[0].device != g.device:
                    pr.scratch = [torch.zeros(p_.shape, dtype=F32, device=g.device) for p_ in ps]
                tgt = pr.scratch
                for t_ in tgt:
                    t_.zero_()
            elif not direct:
                tgt = [torch.zeros(p_.shape, dtype=F32, device=g.device) for p_ in ps]
            tw_out, tb_out, tw_lin, tb_lin = tgt
            if split:
                tab = pr.bwd_table(tw_out.view(C, C), tb_out, tw_lin.view(C, C), tb_lin)
                g4, x4 = g.reshape(rows, 1, 1, C), a2.reshape(rows, 1, 1, C)
                spec = wgrad_job(g4, x4, C, C, rows, 1, 1, 1, pr.M.view(C, C, 1), pr.dcol, ks, accumulate=False)

                def job(g4=g4, x4=x4, ks=ks):
                    _wgrad(g4, x4, C, C, rows, 1, 1, 1, 1, 1, 1, dW=pr.M.view(C, C, 1), db=pr.dcol,
                           accumulate=False, scale=ks)

                if direct:
                    # M = ks dy^T a (+ colsum) as a grouped weight-gradient job, then the C x C split
                    # onto the two layers' gradients -- both on the weight-gradient stream, in order
                    SINK.submit(g.device, job, (g4, x4), (), spec=spec)
                    SINK.submit(g.device, tab.run, (), ps)
                else:
                    job()
                    tab.run()
                    grads = [t_.clone() for t_ in tgt]
            else:
                def job(g=g, a2=a2, ks=ks):
                    # the layers' intermediates, recomputed off the critical path
                    o = torch.empty(rows, C, dtype=BF16, device=g.device)
                    gemm_nt(bf16_weight(W_out), a2, o, C, rows, C, C, C, C, bias=b_out.detach())
                    do = torch.empty(rows, C, dtype=BF16, device=g.device)
                    gemm_nt(packed_weight(W_lin, True, 1), g, do, C, rows, C, C, C, C, alpha=ks)
                    pairs = [(t_.reshape(rows, 1, 1, C), u_.reshape(rows, 1, 1, C), tw_.view(C, C, 1), tb_, sc_)
                             for t_, u_, tw_, tb_, sc_ in ((g, o, tw_lin, tb_lin, ks), (do, a2, tw_out, tb_out, 1.0))]
                    jobs = [wgrad_job(d4, x4, C, C, rows, 1, 1, 1, tw_, tb_, sc_) for d4, x4, tw_, tb_, sc_ in pairs]
                    if all(j is not None for j in jobs):
                        wgrad_group_run(jobs)
                    else:
                        for d4, x4, tw_, tb_, sc_ in pairs:
                            _wgrad(d4, x4, C, C, rows, 1, 1, 1, 1, 1, 1, dW=tw_, db=tb_, accumulate=True, scale=sc_)

                if direct:
                    SINK.submit(g.device, job, (g, a2), ps)
                else:
                    job()
                    grads = tgt
        dres = None
        if ctx.has_res and ctx.needs_input_grad[5] and (slot is None or not slot.deposit(g, ks)):
            assert ks == 1.0
            dres = g.view(ctx.shp)
        return (da, *grads, dres, None, None, None)


def attn_out(a, W_out, b_out, W_lin, b_lin, residual=None, out_scale=1.0, res_slot=None, gn_groups=0):
    """The attention block's output map ``linear(out_proj(a))`` (+ residual,
    x out_scale, + fused GroupNorm statistics) as ONE merged GEMM forward and
    backward (see _AttnPair).  ``a`` [N, L, C]."""
    _need_bf16(a, residual)
    C = a.shape[-1]
    rows = a.numel() // C
    if C % 64 or W_lin.reshape(W_lin.shape[0], -1).shape != (C, C) or tuple(W_out.shape) != (C, C) or \
            b_out is None or b_lin is None or \
            (rows < _ATTN_SPLIT * C and not _ATTN_SMALL and rows < _ATTN_SMALL_MIN * C):
        o = linear(a, W_out, b_out)
        return linear(o, W_lin, b_lin, residual, out_scale, res_slot, None, gn_groups)
    if gn_groups and gn_img_ok(a.shape[1], C, int(gn_groups), a.shape[0]):
        gn_groups = 0                   # the consumer's whole-image kernel makes its own statistics
    gn = {"groups": int(gn_groups)} if (gn_groups and _EPI_GN_STATS) else None
    y = _AttnOut.apply(a.contiguous(), W_out, b_out, W_lin, b_lin, residual, out_scale, res_slot, gn)
    if gn is not None and "part" in gn:
        y._d3d_gnpart = (gn["part"][0], int(gn_groups), gn["part"][1])
    return y


def carry_gn_stats(src: torch.Tensor, dst: torch.Tensor) -> torch.Tensor:
    """Keep fused GroupNorm partials on a reshaped view of the same data."""
    part = getattr(src, "_d3d_gnpart", None)
    if part is not None:
        dst._d3d_gnpart = part
    return dst


# ------------------------------------------------------------ attention ----
class _Attention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, heads, cross):
        qkv = qkv.contiguous()
        N, L, C3 = qkv.shape
        C = C3 // 3
        out = torch.empty(N, L, C, dtype=BF16, device=qkv.device)
        lse = torch.empty(N, heads, L, dtype=F32, device=qkv.device)
        scale = 1.0 / math.sqrt(C // heads)
        _chk(_lib.d3d_attn_fwd(qkv.data_ptr(), out.data_ptr(), lse.data_ptr(), N, L, C, heads, int(cross), scale,
                               _st()), "attn_fwd")
        ctx.save_for_backward(qkv, out, lse)
        ctx.cfg = (heads, cross, scale)
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse = ctx.saved_tensors
        heads, cross, scale = ctx.cfg
        N, L, C3 = qkv.shape
        C = C3 // 3
        dout = dout.contiguous()
        # one fp32 dQ slab per 64-key block, summed in fixed order
        # (deterministic); a single key block (L <= 64), or one workgroup
        # owning all keys (L <= 256 at head dim 64, enough (image, head)
        # pairs), writes dQ directly; a ragged last block (L % 64 != 0) is
        # masked in the kernels
        slabs = _lib.d3d_attn_bwd_slabs(N, L, C, heads)
        dq = torch.empty(slabs, N, L, C, dtype=F32, device=qkv.device) if slabs else None
        dqkv = torch.empty_like(qkv)
        _chk(_lib.d3d_attn_bwd(qkv.data_ptr(), out.data_ptr(), dout.data_ptr(), lse.data_ptr(), _ptr(dq),
                               dqkv.data_ptr(), N, L, C, heads, int(cross), scale, _st()), "attn_bwd")
        return dqkv, None, None


def attention(qkv, heads, cross):
    _need_bf16(qkv)
    N, L, C3 = qkv.shape
    D = C3 // 3 // heads
    if D not in (64, 128) or (cross and N % 2):
        _fallback("attention", f"L={L} head_dim={D} N={N} cross={cross}")
        return _t.attention(qkv, heads, cross)
    return _Attention.apply(qkv, heads, cross)


# --------------------------------------------------- logSNR embedding ----
class _LogSNRMLP(torch.autograd.Function):
    """posenc_ddpm + Linear-SiLU-Linear of the logSNR embedding
    (`xunet.py:273-277,305-308`) on ``csrc/mlp.hip``: posenc, two
    split-K fp32 GEMMs with bias / SiLU-on-load epilogues; backward is one
    input-gradient GEMM with the dSiLU epilogue and two weight-gradient
    launches that deposit straight into the gradient sink."""

    @staticmethod
    def forward(ctx, logsnr, w1, b1, w2, b2, tscale):
        l = logsnr.reshape(-1).float().contiguous()
        R, E = l.numel(), w1.shape[0]
        dev = l.device
        pe = torch.empty(R, E, dtype=F32, device=dev)
        a1 = torch.empty(R, E, dtype=F32, device=dev)
        out = torch.empty(R, E, dtype=F32, device=dev)
        ws = torch.empty(max(int(_lib.d3d_mlp_ws(R, E, E)), 1), dtype=F32, device=dev)
        _chk(_lib.d3d_mlp_pe(l.data_ptr(), R, E, float(tscale), pe.data_ptr(), _st()), "mlp_pe")
        _chk(_lib.d3d_mlp_mm(pe.data_ptr(), w1.detach().contiguous().data_ptr(), R, E, E, 0, 0, 0, _ptr(b1), None,
                             ws.data_ptr(), a1.data_ptr(), _st()), "mlp_mm1")
        _chk(_lib.d3d_mlp_mm(a1.data_ptr(), w2.detach().contiguous().data_ptr(), R, E, E, 1, 0, 0, _ptr(b2), None,
                             ws.data_ptr(), out.data_ptr(), _st()), "mlp_mm2")
        ctx.save_for_backward(pe, a1, w2)
        ctx.params = (w1, b1, w2, b2)
        for i, p in enumerate(ctx.params):
            SINK.use(p, ctx.needs_input_grad[1 + i])
        return out

    @staticmethod
    def backward(ctx, dout):
        pe, a1, w2 = ctx.saved_tensors
        w1p, b1p, w2p, b2p = ctx.params
        g = dout.float().contiguous()
        R, E = g.shape
        dev = g.device
        ws = torch.empty(max(int(_lib.d3d_mlp_ws(R, E, E)), 1), dtype=F32, device=dev)
        da1 = torch.empty(R, E, dtype=F32, device=dev)
        # da1 = (dout @ W2) * dsilu(a1)
        _chk(_lib.d3d_mlp_mm(g.data_ptr(), w2.detach().contiguous().data_ptr(), R, E, E, 0, 1, 1, None, a1.data_ptr(),
                             ws.data_ptr(), da1.data_ptr(), _st()), "mlp_dgrad")
        targets = [SINK.target(p) for p in ctx.params]
        if all(t is not None for t in targets):
            tw1, tb1, tw2, tb2 = targets

            def job(g=g, a1=a1, da1=da1, pe=pe):
                _chk(_lib.d3d_mlp_wgrad(g.data_ptr(), a1.data_ptr(), R, E, E, 1, tw2.data_ptr(), tb2.data_ptr(), 1,
                                        _st()), "mlp_wgrad2")
                _chk(_lib.d3d_mlp_wgrad(da1.data_ptr(), pe.data_ptr(), R, E, E, 0, tw1.data_ptr(), tb1.data_ptr(), 1,
                                        _st()), "mlp_wgrad1")
            SINK.submit(dev, job, (g, a1, da1, pe), ctx.params)
            return None, None, None, None, None, None
        dw1 = torch.empty(E, E, dtype=F32, device=dev)
        dw2 = torch.empty(E, E, dtype=F32, device=dev)
        db1 = torch.empty(E, dtype=F32, device=dev)
        db2 = torch.empty(E, dtype=F32, device=dev)
        _chk(_lib.d3d_mlp_wgrad(g.data_ptr(), a1.data_ptr(), R, E, E, 1, dw2.data_ptr(), db2.data_ptr(), 0, _st()),
             "mlp_wgrad2")
        _chk(_lib.d3d_mlp_wgrad(da1.data_ptr(), pe.data_ptr(), R, E, E, 0, dw1.data_ptr(), db1.data_ptr(), 0, _st()),
             "mlp_wgrad1")
        return None, dw1, db1, dw2, db2, None


def logsnr_mlp(logsnr, w1, b1, w2, b2, max_time=1.0):
    E = w1.shape[0]
    if tuple(w1.shape) != (E, E) or tuple(w2.shape) != (E, E) or E % 64 or b1 is None or b2 is None:
        _fallback("logsnr_mlp", f"E={E}")
        return _t.logsnr_mlp(logsnr, w1, b1, w2, b2, max_time)
    return _LogSNRMLP.apply(logsnr, w1, b1, w2, b2, 1000.0 / max_time)


# -------------------------------------------------------- elementwise ----
class _SiLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        y = torch.empty_like(x)
        _chk(_lib.d3d_silu(x.data_ptr(), y.data_ptr(), x.numel(), _st()), "silu")
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        dx = torch.empty_like(x)
        _chk(_lib.d3d_dsilu(x.data_ptr(), dy.contiguous().data_ptr(), dx.data_ptr(), x.numel(), _st()), "dsilu")
        return dx


def silu(x):
    _need_bf16(x)
    return _SiLU.apply(x)


class _AvgPool2(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        N, H, W, C = x.shape
        y = torch.empty(N, H // 2, W // 2, C, dtype=x.dtype, device=x.device)
        _chk(_lib.d3d_avgpool2(x.data_ptr(), y.data_ptr(), N, H, W, C, 0, _st()), "avgpool2")
        ctx.shape = x.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        N, H, W, C = ctx.shape
        dx = torch.empty(N, H, W, C, dtype=dy.dtype, device=dy.device)
        _chk(_lib.d3d_avgpool2(dy.contiguous().data_ptr(), dx.data_ptr(), N, H, W, C, 1, _st()), "avgpool2_bwd")
        return dx


class _Upsample2(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        N, H, W, C = x.shape
        y = torch.empty(N, 2 * H, 2 * W, C, dtype=x.dtype, device=x.device)
        _chk(_lib.d3d_upsample2(x.data_ptr(), y.data_ptr(), N, H, W, C, 0, _st()), "upsample2")
        ctx.shape = x.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        N, H, W, C = ctx.shape
        dx = torch.empty(N, H, W, C, dtype=dy.dtype, device=dy.device)
        _chk(_lib.d3d_upsample2(dy.contiguous().data_ptr(), dx.data_ptr(), N, H, W, C, 1, _st()), "upsample2_bwd")
        return dx


def avgpool2(x):
    _need_bf16(x)
    return _AvgPool2.apply(x)


def upsample2(x):
    _need_bf16(x)
    return _Upsample2.apply(x)


# ------------------------------------------------------------- rays ------
def _inv3x3(m: torch.Tensor) -> torch.Tensor:
    """Batched 3x3 inverse by the adjugate: pure elementwise kernels, no
    host synchronisation (torch.linalg.inv reads its error flags back to the
    host, which a graph capture forbids)."""
    a, b, c = m[:, 0, 0], m[:, 0, 1], m[:, 0, 2]
    d, e, f = m[:, 1, 0], m[:, 1, 1], m[:, 1, 2]
    g, h, i = m[:, 2, 0], m[:, 2, 1], m[:, 2, 2]
    A, B_, C = e * i - f * h, -(d * i - f * g), d * h - e * g
    det = a * A + b * B_ + c * C
    adj = torch.stack([A, -(b * i - c * h), b * f - c * e,
                       B_, a * i - c * g, -(a * f - c * d),
                       C, -(a * h - b * g), a * e - b * d], 1).reshape(-1, 3, 3)
    return adj / det[:, None, None]



class _RayPosenc(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pos_emb, first_emb, other_emb, R, t, K, H, W, cond_mask, rescale_from):
        B = R.shape[0]
        Kd = K.to(torch.float64)
        if rescale_from:
            Kd = torch.cat([Kd[:, 0:1] * (W / rescale_from), Kd[:, 1:2] * (H / rescale_from), Kd[:, 2:3]], 1)
        Kinv = _inv3x3(Kd).float().contiguous()
        Rf = R.float().reshape(B * 2, 9).contiguous()
        tf = t.float().reshape(B * 2, 3).contiguous()
        mask = cond_mask.to(torch.uint8).contiguous()
        out = torch.empty(B * 2, H, W, 144, dtype=BF16, device=R.device)
        pe = pos_emb.contiguous() if pos_emb is not None else None
        fe = first_emb.reshape(-1).contiguous() if first_emb is not None else None
        oe = other_emb.reshape(-1).contiguous() if other_emb is not None else None
        _chk(_lib.d3d_ray_posenc(Rf.data_ptr(), tf.data_ptr(), Kinv.data_ptr(), mask.data_ptr(), _ptr(pe), _ptr(fe),
                                 _ptr(oe), out.data_ptr(), B, H, W, _st()), "ray_posenc")
        ctx.has = (pos_emb is not None, first_emb is not None)
        ctx.B = B
        return out

    @staticmethod
    def backward(ctx, g):
        has_pe, has_fe = ctx.has
        B = ctx.B
        N, H, W, D = g.shape
        gf = g.float()
        dpe = gf.sum(0).permute(2, 0, 1).contiguous() if has_pe else None
        dfe = doe = None
        if has_fe:
            fsum = gf.reshape(B, 2, H * W, D).sum((0, 2))
            dfe = fsum[0].reshape(1, 1, D, 1, 1)
            doe = fsum[1].reshape(1, 1, D, 1, 1)
        return dpe, dfe, doe, None, None, None, None, None, None, None


def ray_posenc(R, t, K, H, W, cond_mask, pos_emb, first_emb, other_emb, rescale_from=0, out_dtype=BF16):
    if out_dtype != BF16:
        return _t.ray_posenc(R, t, K, H, W, cond_mask, pos_emb, first_emb, other_emb, rescale_from).to(out_dtype)
    return _RayPosenc.apply(pos_emb, first_emb, other_emb, R, t, K, H, W, cond_mask, rescale_from)


# ------------------------------------------------------------ optimizer --
def adam_flat(p, g, m, v, ema, lr, b1, b2, eps, wd, step_size, bc2_sqrt, grad_scale, ema_decay):
    _chk(_lib.d3d_adam(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), _ptr(ema), p.numel(), b1, b2, eps, wd,
                       step_size, bc2_sqrt, grad_scale, ema_decay, _st()), "adam")
    refresh_weights()


# Fused optimizer step + operand repack (adam.hip d3d_adam_fused).  Tables
# (built on the host when the weight cache changes, never inside a capture):
#   tiles  -- weights whose cached MFMA operands are plain forward / transposed
#             packs: their Adam runs tile by tile and writes the packs from the
#             updated tile (the repack never re-reads their fp32 masters);
#   ranges -- every other span of the flat buffer: plain vectorised Adam;
#   rest   -- the remaining cached operands (bf16 casts, channel slices):
#             repacked by pack_all after both.
_FUSED = {}


def _fused_tables(flat, only=None, key=None, take_unowned=True):
    """``only``: restrict the update to these parameter indices (one part of
    a split update, :func:`prepare_update_parts`); ``key``: its cache key;
    ``take_unowned``: this part also repacks cached operands of tensors that
    are not flat parameters."""
    import numpy as np
    key = id(flat) if key is None else key
    ent = _FUSED.get(key)
    if ent is not None and ent["rev"] == _REV[0] and ent["flat"] is flat:
        return ent
    pidx = {id(p): i for i, p in enumerate(flat.params)}
    per = {}                                   # param index -> {"0": (t, desc), "1": (t, desc)}
    absorbed = set()
    for ckey, (tok, t, (p, desc)) in _WCACHE.items():
        i = pidx.get(id(p))
        if i is None or desc is None or len(desc) > 6 or desc[5] not in (0, 1):
            continue
        if only is not None and i not in only:
            absorbed.add(ckey)                 # another part's weight: neither tiled nor repacked here
            continue
        OC, IC, OCp, ICp, taps, mode = desc[:6]
        if p.shape[0] != OC or p.numel() != OC * IC * taps or taps > 9:
            continue
        slot = per.setdefault(i, {})
        if str(mode) in slot:
            continue
        slot[str(mode)] = (t, desc)
        absorbed.add(ckey)
    # tile table
    trows, tblk = [], 0
    for i, slot in sorted(per.items()):
        prm = flat.params[i]
        t0 = slot.get("0")
        t1 = slot.get("1")
        d = (t0 or t1)[1]
        OC, IC, taps = d[0], d[1], d[4]
        trows.append((flat.offsets[i], t0[0].data_ptr() if t0 else 0, t1[0].data_ptr() if t1 else 0, OC, IC, taps,
                      t0[1][3] if t0 else 0, t1[1][2] if t1 else 0, tblk))
        tblk += ((OC + 31) // 32) * ((IC + 15) // 16)
    # range table: the complement of the tile weights' spans (of this part's
    # parameters when split)
    rrows, rblk = [], 0
    if only is None:
        tiled = sorted((flat.offsets[i], flat.span(i)[1]) for i in per)
        pos = 0
        for a, b in tiled + [(flat.numel, flat.numel)]:
            if a > pos:
                rrows.append((pos, a - pos, rblk, 0))
                rblk += (a - pos + 4095) // 4096
            pos = max(pos, b)
    else:
        spans = sorted(flat.span(i) for i in only if i not in per)
        merged = []
        for a, b in spans:
            if merged and a <= merged[-1][1]:
                merged[-1][1] = max(merged[-1][1], b)
            else:
                merged.append([a, b])
        for a, b in merged:
            rrows.append((a, b - a, rblk, 0))
            rblk += (b - a + 4095) // 4096
    dev = flat.data.device
    tdt = np.dtype([("off", np.int64), ("dst0", np.uint64), ("dst1", np.uint64), ("OC", np.int32),
                    ("IC", np.int32), ("taps", np.int32), ("ICp0", np.int32), ("OCp1", np.int32), ("blk0", np.int32)])
    rdt = np.dtype([("start", np.int64), ("len", np.int64), ("blk0", np.int32), ("pad", np.int32)])

    def table(rows, dt, nblk):
        if not rows:
            return None, None
        arr = np.array(rows, dtype=dt)
        counts = np.diff(np.append(arr["blk0"], nblk))
        bmap = np.repeat(np.arange(len(rows), dtype=np.int32), counts)
        return (torch.from_numpy(arr.view(np.uint8).copy()).to(dev), torch.from_numpy(bmap).to(dev))
    tt, tb = table(trows, tdt, tblk)
    rt, rb = table(rrows, rdt, rblk)
    rest_rows, rest_blk = [], 0
    for ckey, (tok, t, (p, desc)) in _WCACHE.items():
        if desc is None or ckey in absorbed:
            continue
        if only is not None:
            owner = pidx.get(id(p))
            if (owner is None and not take_unowned) or (owner is not None and owner not in only):
                continue
        OC, IC, OCp, ICp, taps, mode = desc[:6]
        src_off = desc[6] if len(desc) > 6 else 0
        ics = desc[7] if len(desc) > 7 else 0
        ldd = desc[8] if len(desc) > 8 else 0
        rest_rows.append((p.data_ptr() + src_off, t.data_ptr(), OC, IC, OCp, ICp, taps, mode, rest_blk, ics, ldd, 0))
        rest_blk += _pack_blocks(OC, OCp, ICp, mode)
    rd, rm = _desc_tensors(rest_rows, rest_blk) if rest_rows else (None, None)
    ent = {"rev": _REV[0], "flat": flat, "tiles": (tt, tb, tblk), "ranges": (rt, rb, rblk),
           "rest": (rd, rm, rest_blk)}
    _FUSED[key] = ent
    return ent


def prepare_fused_update(flat) -> None:
    """Build the fused-update tables now (host work; call before a capture)."""
    _fused_tables(flat)


def prepare_update_parts(flat, parts) -> None:
    """Build the fused-update tables of a split update: ``parts`` is a list of
    parameter-index sets covering ``flat.params`` (host work; before a
    capture).  :func:`adam_update_part` then updates one part."""
    attn = {id(p_) for pr in _ATTN_PAIRS.values() for p_ in pr.params}
    for k, only in enumerate(parts):
        ent = _fused_tables(flat, set(only), key=(id(flat), "part", k), take_unowned=k == 0)
        ent["attn"] = any(id(flat.params[i]) in attn for i in only)


def adam_update_part(flat, m, v, ema, hp, k, zero_g=False) -> None:
    """The fused Adam + operand repack of part ``k`` (:func:`prepare_update_parts`).
    ``zero_g``: clear the part's gradients as they are consumed (the parts
    together cover every parameter; padding between parameters is never
    written, so it stays zero)."""
    ent = _FUSED.get((id(flat), "part", k))
    if ent is None or ent["rev"] != _REV[0] or ent["flat"] is not flat:
        raise RuntimeError("update-part tables missing or stale (prepare_update_parts before the capture)")
    _adam_fused_launch(flat, m, v, ema, hp, ent, zero_g)
    if ent.get("attn"):
        _attn_refresh()                     # this part updates attention output maps: re-derive the merged operands


def _adam_fused_launch(flat, m, v, ema, hp, ent, zero_g=False) -> None:
    (tt, tb, tblk), (rt, rb, rblk), (rd, rm, rest_blk) = ent["tiles"], ent["ranges"], ent["rest"]
    if tblk or rblk:
        _chk(_lib.d3d_adam_fused(flat.data.data_ptr(), flat.grad.data_ptr(), m.data_ptr(), v.data_ptr(), _ptr(ema),
                                 hp.data_ptr(), _ptr(rt), _ptr(rb), int(rblk), _ptr(tt), _ptr(tb), int(tblk),
                                 int(bool(zero_g)), _st()),
             "adam_fused")
    if rest_blk:
        _chk(_lib.d3d_pack_all(rd.data_ptr(), rm.data_ptr(), rest_blk, _st()), "pack_all")


def adam_update_all(flat, m, v, ema, hp, zero_g=False) -> None:
    """One optimizer step over the whole flat buffer with the cached bf16
    operands repacked from the updated weights (replaces adam_flat_dev +
    refresh_weights).  Inside a graph capture the tables must already exist
    (:func:`prepare_fused_update`).  ``zero_g``: the gradient buffer is left
    zeroed (the range table covers every element the tile table does not)."""
    capturing = torch.cuda.is_current_stream_capturing()
    ent = _FUSED.get(id(flat))
    if ent is None or ent["rev"] != _REV[0] or ent["flat"] is not flat:
        if capturing:
            raise RuntimeError("fused update tables are stale inside a graph capture")
        ent = _fused_tables(flat)
    (tt, tb, tblk), (rt, rb, rblk), (rd, rm, rest_blk) = ent["tiles"], ent["ranges"], ent["rest"]
    _chk(_lib.d3d_adam_fused(flat.data.data_ptr(), flat.grad.data_ptr(), m.data_ptr(), v.data_ptr(), _ptr(ema),
                             hp.data_ptr(), _ptr(rt), _ptr(rb), int(rblk), _ptr(tt), _ptr(tb), int(tblk),
                             int(bool(zero_g)), _st()),
         "adam_fused")
    if rest_blk:
        _chk(_lib.d3d_pack_all(rd.data_ptr(), rm.data_ptr(), rest_blk, _st()), "pack_all")
    _EPOCH[0] += 1
    for e in _WCACHE.values():
        e[0] = (e[2][0]._version, _EPOCH[0])
    _attn_refresh()                         # the merged attention operands of the updated weights


def set_words(dst: torch.Tensor, vals) -> torch.Tensor:
    """dst[:len(vals)] = vals (fp32, <= 8) by a kernel whose arguments carry
    the values: unlike a host-to-device copy from pageable memory this never
    makes the host wait for the stream (graph-capture safe as well)."""
    vals = [float(v) for v in vals]
    assert dst.dtype == F32 and dst.is_cuda and dst.is_contiguous() and len(vals) <= min(8, dst.numel())
    _chk(_lib.d3d_set_words(dst.data_ptr(), len(vals), *(vals + [0.0] * (8 - len(vals))), _st()), "set_words")
    return dst


def set_words64(dst: torch.Tensor, vals) -> torch.Tensor:
    """dst[:len(vals)] = vals (int64, <= 3) by one kernel whose arguments
    carry the values (the graph step's per-step seed block)."""
    vals = [int(v) for v in vals]
    assert dst.dtype == torch.int64 and dst.is_cuda and dst.is_contiguous() and len(vals) <= min(3, dst.numel())
    vals = [v - (1 << 64) if v >= (1 << 63) else v for v in vals]       # (two's complement for the ABI)
    _chk(_lib.d3d_set_words64(dst.data_ptr(), len(vals), *(vals + [0] * (3 - len(vals))), _st()), "set_words64")
    return dst


def adam_flat_dev(p, g, m, v, ema, hp, refresh=True):
    """Adam with its per-step hyper-parameters read from the device block
    ``hp`` (graph-replay form; see d3d_adam_dev).  Works on any contiguous
    span of the flat buffers (refresh=False: the caller repacks the bf16
    operand caches once after the last span)."""
    _chk(_lib.d3d_adam_dev(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), _ptr(ema), p.numel(),
                           hp.data_ptr(), _st()), "adam_dev")
    if refresh:
        refresh_weights()


# ------------------------------------------- training input and loss ---
def diffusion_inputs(img, seed, e0=0, cond_prob=0.1, logsnr_min=-20.0, logsnr_max=20.0, dtype=BF16):
    """One launch (diffusion_fwd2_k): t, lambda, eps, z_t, CFG drop -> the
    stem's NHWC bf16 input, eps, logsnr [B,2], keep mask.  Same numbers as
    ``torch_impl.diffusion_inputs``; in a graph replay the per-step part of the
    seed is the device word of :func:`set_device_seed`."""
    assert dtype == BF16
    img = img.float().contiguous()
    B, _, C, H, W = img.shape
    assert C == 3, img.shape
    dev = img.device
    xz = torch.empty(2 * B, H, W, 8, dtype=BF16, device=dev)
    eps = torch.empty(B, 3, H, W, dtype=F32, device=dev)
    lam = torch.empty(B, 2, dtype=F32, device=dev)
    keep = torch.empty(B, dtype=torch.uint8, device=dev)
    a, b = _t.schedule_ab(logsnr_min, logsnr_max)
    _chk(_lib.d3d_diffusion_fwd2(img.data_ptr(), B, H * W, int(seed) & 0xFFFFFFFFFFFFFFFF, _ptr(_SEED_DEV[0]), int(e0),
                                 float(cond_prob), float(a), float(b), eps.data_ptr(), lam.data_ptr(),
                                 keep.data_ptr(), xz.data_ptr(), _st()), "diffusion_fwd2")
    return xz, eps, lam, keep.view(torch.bool)


_LOSS_MODES = {"l2": 0, "l1": 1, "huber": 2}


class _DiffLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, eps, mode):
        B, H, W, CP = y.shape
        part = torch.empty(256, dtype=F32, device=y.device)
        out = torch.empty((), dtype=F32, device=y.device)
        _chk(_lib.d3d_diff_loss(y.data_ptr(), eps.data_ptr(), B, H * W, CP, mode, part.data_ptr(), out.data_ptr(),
                                _st()), "diff_loss")
        ctx.save_for_backward(y, eps)
        ctx.mode = mode
        return out

    @staticmethod
    def backward(ctx, dl):
        y, eps = ctx.saved_tensors
        B, H, W, CP = y.shape
        dl = dl.float().contiguous()
        dy = torch.empty_like(y)
        _chk(_lib.d3d_diff_loss_bwd(y.data_ptr(), eps.data_ptr(), dl.data_ptr(), B, H * W, CP, ctx.mode,
                                    dy.data_ptr(), _st()), "diff_loss_bwd")
        return dy, None, None


def diff_loss_nhwc(y, eps, loss_type="l2"):
    """Epsilon loss read straight from the channel-padded NHWC head output
    (two launches forward, one backward; deterministic partial sums)."""
    if loss_type not in _LOSS_MODES:
        raise ValueError(f"loss_type {loss_type!r}: expected one of {sorted(_LOSS_MODES)}")
    if y.shape[-1] != 8 or y.dtype != BF16:
        _fallback("diff_loss", f"head layout {tuple(y.shape)} {y.dtype}")
        return _t.diff_loss_nhwc(y, eps, loss_type)
    return _DiffLoss.apply(y.contiguous(), eps.float().contiguous(), _LOSS_MODES[loss_type])


# ------------------------------------------------------------- sampler ---
def sampler_inputs(xc, z, prm, sd, seed, c0, xz, logsnr):
    b = z.shape[0]
    HW = z.shape[-1] * z.shape[-2]
    _chk(_lib.d3d_sampler_inputs(xc.data_ptr(), z.data_ptr(), b, HW, prm.data_ptr(), _ptr(sd),
                                 int(seed) & 0xFFFFFFFFFFFFFFFF, int(c0), xz.data_ptr(), logsnr.data_ptr(), _st()),
         "sampler_inputs")


def sampler_step2(z, y, w, prm, sd, seed, c0):
    b = z.shape[0]
    HW = z.shape[-1] * z.shape[-2]
    assert y.shape[-1] == 8 and y.shape[0] == 2 * b and z.is_contiguous()
    _chk(_lib.d3d_sampler_step2(z.data_ptr(), y.data_ptr(), w.data_ptr(), b, HW, prm.data_ptr(), _ptr(sd),
                                int(seed) & 0xFFFFFFFFFFFFFFFF, int(c0), _st()), "sampler_step2")


def randn_hash(shape, seed, off, device):
    out = torch.empty(shape, dtype=F32, device=device)
    _chk(_lib.d3d_randn_hash(out.data_ptr(), out.numel(), int(seed) & 0xFFFFFFFFFFFFFFFF, int(off), _st()),
         "randn_hash")
    return out


def sampler_step(z, eps_c, eps_u, w, alpha, sigma, alpha_n, c, var_sqrt, add_noise, seed):
    b = z.shape[0]
    D = z[0].numel()
    out = torch.empty_like(z)
    _chk(_lib.d3d_sampler_step(z.data_ptr(), eps_c.contiguous().data_ptr(), eps_u.contiguous().data_ptr(),
                               w.float().contiguous().data_ptr(), out.data_ptr(), b, D, alpha, sigma, alpha_n, c,
                               var_sqrt, int(add_noise), int(seed), _st()), "sampler_step")
    return out
