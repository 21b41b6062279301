"""NHWC op set of the X-UNet, dispatched to hand-written HIP kernels (gfx950)
or to the PyTorch reference composition.

Every function here has identical semantics in both backends; the torch
versions (``torch_impl``) are the numerics oracle used by the tests.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import torch_impl as _t
from ._backend import use_hip, set_backend, load_library, library_error, lib_path

_hip = None


def _h():
    global _hip
    if _hip is None:
        from . import hip_impl
        _hip = hip_impl
    return _hip


def group_norm(x, weight, bias, groups: int = 32, eps: float = 1e-5, silu: bool = False, res_slot=None):
    if use_hip(x):
        return _h().group_norm(x, weight, bias, groups, eps, silu, res_slot)
    return _t.group_norm(x, weight, bias, groups, eps, silu)


def gn_film(x, weight, bias, ss, groups: int = 32, eps: float = 1e-5, dropout_p: float = 0.0,
            training: bool = False, seed: int = 0, ss_map: Optional[torch.Tensor] = None):
    """ss_map (int32 [N], inference): image n is modulated by ss[ss_map[n]]
    (shared conditioning, XUNet.forward(shared_cond=))."""
    if use_hip(x):
        return _h().gn_film(x, weight, bias, ss, groups, eps, dropout_p, training, seed, ss_map)
    return _t.gn_film(x, weight, bias, ss, groups, eps, dropout_p, training, seed, ss_map)


def conv3x3(x, weight, bias, stride: int = 1, residual: Optional[torch.Tensor] = None,
            out_scale: float = 1.0, row_bias: Optional[torch.Tensor] = None, res_period: int = 0,
            gn_groups: int = 0, res_slot=None, keep_pad: bool = False):
    """gn_groups: the output feeds a GroupNorm with that many groups (the HIP
    path then fuses that GroupNorm's statistics into the conv epilogue).
    res_slot / in_slot (HIP path; :class:`ResGradSlot`): hand the residual's /
    the input's gradient to the GroupNorm that reads the same tensor.
    keep_pad: (IC or OC not a multiple of 8, i.e. stem / head) the HIP path
    returns the channel-padded output (the fused loss reads it in place).
    Inputs may carry zero channels beyond the weight's IC (pre-padded stem
    input)."""
    if use_hip(x):
        return _h().conv3x3(x, weight, bias, stride, residual, out_scale, row_bias, res_period, gn_groups, res_slot,
                            keep_pad)
    if x.shape[-1] > weight.shape[1]:
        x = x[..., :weight.shape[1]]
    return _t.conv3x3(x, weight, bias, stride, residual, out_scale, row_bias, res_period)


def linear(x, weight, bias, residual: Optional[torch.Tensor] = None, out_scale: float = 1.0, res_slot=None,
           in_slot=None, gn_groups: int = 0):
    """gn_groups: the output feeds a GroupNorm with that many groups (the HIP
    epilogue then also emits its partial statistics)."""
    if use_hip(x):
        return _h().linear(x, weight, bias, residual, out_scale, res_slot, in_slot, gn_groups)
    return _t.linear(x, weight, bias, residual, out_scale)


def attn_out(a, W_out, b_out, W_lin, b_lin, residual: Optional[torch.Tensor] = None, out_scale: float = 1.0,
             res_slot=None, gn_groups: int = 0):
    """The attention block's output map ``linear(out_proj(a))`` + residual,
    x out_scale (`xunet.py:175,217-220`).  HIP: one merged GEMM forward and
    backward (hip_impl.attn_out); torch: the two layers as written."""
    if use_hip(a):
        return _h().attn_out(a, W_out, b_out, W_lin, b_lin, residual, out_scale, res_slot, gn_groups)
    return _t.linear(_t.linear(a, W_out, b_out), W_lin, b_lin, residual, out_scale)


def carry_gn_stats(src: torch.Tensor, dst: torch.Tensor) -> torch.Tensor:
    """A reshaped view keeps the fused GroupNorm statistics of its source."""
    part = getattr(src, "_d3d_gnpart", None)
    if part is not None:
        dst._d3d_gnpart = part
    return dst


def cond_conv(rays_dir, orig_pe, weight, bias, stride: int, row_bias=None, residual=None, res_period: int = 0,
              silu_out: bool = False):
    """``silu_out``: (HIP) the output also carries silu(output) for the FiLM
    projections (film_batch then skips its SiLU pass); ignored by the torch
    composition, which film_batch handles itself."""
    if use_hip(rays_dir):
        return _h().cond_conv(rays_dir, orig_pe, weight, bias, stride, row_bias, residual, res_period,
                              silu_out=silu_out)
    return _t.cond_conv(rays_dir, orig_pe, weight, bias, stride, row_bias, residual, res_period)


def ray_posenc_dir(R, t, K, H: int, W: int, cond_mask, rescale_from: int = 0, out_dtype=None):
    if out_dtype == torch.bfloat16 and R.is_cuda and use_hip(R, any_dtype=True):
        return _h().ray_posenc_dir(R, t, K, H, W, cond_mask, rescale_from)
    y = _t.ray_posenc_dir(R, t, K, H, W, cond_mask, rescale_from)
    return y.to(out_dtype) if out_dtype is not None else y


def ray_conditioning(R, t, K, H: int, W: int, cond_mask, rescale_from: int = 0, out_dtype=None):
    """(masked ray-direction image [2B,H,W,>=51], masked origin posenc [2B,93]
    fp32) -- :func:`ray_posenc_dir` and :func:`ray_origin_pe` together; two
    HIP launches for bf16 GPU runs."""
    if out_dtype == torch.bfloat16 and R.is_cuda and use_hip(R, any_dtype=True):
        return _h().ray_conditioning(R, t, K, H, W, cond_mask, rescale_from)
    return ray_posenc_dir(R, t, K, H, W, cond_mask, rescale_from, out_dtype), ray_origin_pe(t, cond_mask)


def ray_origin_pe(t, cond_mask):
    return _t.ray_origin_pe(t, cond_mask)


def cat_gn_silu_dense(a, b, gw, gb, dw, db, groups: int = 32, eps: float = 1e-5):
    if use_hip(a):
        return _h().cat_gn_silu_dense(a, b, gw, gb, dw, db, groups, eps)
    return _t.cat_gn_silu_dense(a, b, gw, gb, dw, db, groups, eps)


def film_batch(emb, weights, biases, block_events: bool = False, split: int = 0):
    """``dense_i(silu(emb))`` for every FiLM projection of one level
    (``block_events``, HIP path: one GEMM and ready event per block;
    ``split``: blocks ``[split:]`` get their own, earlier weight-gradient job)."""
    if use_hip(emb):
        return _h().film_batch(emb, weights, biases, block_events, split)
    return _t.film_batch(emb, weights, biases)


def attention(qkv, heads: int, cross: bool):
    if use_hip(qkv):
        return _h().attention(qkv, heads, cross)
    return _t.attention(qkv, heads, cross)


def diffusion_inputs(img, seed: int, e0: int = 0, cond_prob: float = 0.1, logsnr_min: float = -20.0,
                     logsnr_max: float = 20.0, dtype=torch.float32):
    """Counter-based training-input draw (see torch_impl.diffusion_inputs);
    one HIP launch for bf16 GPU runs."""
    if dtype == torch.bfloat16 and img.is_cuda and use_hip(img, any_dtype=True):
        return _h().diffusion_inputs(img, seed, e0, cond_prob, logsnr_min, logsnr_max, dtype)
    return _t.diffusion_inputs(img, seed, e0, cond_prob, logsnr_min, logsnr_max, dtype)


def diff_loss_nhwc(y, eps, loss_type: str = "l2"):
    if use_hip(y):
        return _h().diff_loss_nhwc(y, eps, loss_type)
    return _t.diff_loss_nhwc(y, eps, loss_type)


def avgpool2(x):
    if use_hip(x):
        return _h().avgpool2(x)
    return _t.avgpool2(x)


def upsample2(x):
    if use_hip(x):
        return _h().upsample2(x)
    return _t.upsample2(x)


def logsnr_mlp(logsnr, w1, b1, w2, b2, max_time: float = 1.0, dtype=None):
    """posenc_ddpm(clamp(logsnr)) -> Linear -> SiLU -> Linear, [B, 2] -> [2B, E]
    fp32.  HIP (``csrc/mlp.hip``) for bf16 GPU runs (``dtype``: the model's
    activation dtype)."""
    if dtype == torch.bfloat16 and logsnr.is_cuda and use_hip(logsnr, any_dtype=True):
        return _h().logsnr_mlp(logsnr, w1, b1, w2, b2, max_time)
    return _t.logsnr_mlp(logsnr, w1, b1, w2, b2, max_time)


def silu(x):
    if use_hip(x):
        return _h().silu(x)
    return _t.silu(x)


def ray_posenc(R, t, K, H: int, W: int, cond_mask, pos_emb, first_emb, other_emb,
               rescale_from: int = 0, out_dtype: torch.dtype = torch.float32):
    if out_dtype == torch.bfloat16 and use_hip(R, any_dtype=True):
        return _h().ray_posenc(R, t, K, H, W, cond_mask, pos_emb, first_emb, other_emb,
                               rescale_from, out_dtype)
    return _t.ray_posenc(R, t, K, H, W, cond_mask, pos_emb, first_emb, other_emb,
                         rescale_from).to(out_dtype)


posenc_ddpm = _t.posenc_ddpm
camera_rays = _t.camera_rays
posenc_nerf = _t.posenc_nerf

__all__ = ["diffusion_inputs", "diff_loss_nhwc", "group_norm", "gn_film", "conv3x3", "linear", "film_batch", "cat_gn_silu_dense", "cond_conv", "ray_posenc_dir",
           "ray_origin_pe", "ray_conditioning", "attention", "avgpool2", "upsample2",
           "silu", "logsnr_mlp", "ray_posenc", "posenc_ddpm", "camera_rays", "posenc_nerf", "set_backend",
           "use_hip", "load_library", "library_error", "lib_path"]


def gn_silu_conv3x3(x, gw, gb, cw, cb, groups: int = 32, eps: float = 1e-5, gn1_groups: int = 0, res_slot=None):
    """``conv3x3(silu(group_norm(x)))``: HIP path with the GroupNorm + SiLU in
    the conv's input staging when the shape allows it (``None`` otherwise:
    the caller runs the two ops)."""
    if use_hip(x) and _h().gn_silu_conv_ok(x, cw.shape[0], groups):
        return _h().gn_silu_conv3x3(x, gw, gb, cw, cb, groups, eps, gn1_groups, res_slot)
    return None


def res_slot(x: torch.Tensor):
    """A residual-gradient hand-off slot for x (HIP path), else None."""
    if use_hip(x):
        return _h().ResGradSlot()
    return None
