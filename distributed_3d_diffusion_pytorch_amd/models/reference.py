"""Independent fp32 NCHW oracle of the reference X-UNet semantics.

The upstream model cannot be executed here (it needs ``visu3d`` and CUDA,
D11), so parity is pinned against this functional re-statement of
`xunet.py:17-536`, written in the reference's own ``[B, F, C, H, W]`` layout
with plain ``torch.nn.functional`` calls and reading weights straight from a
``state_dict``.  It is deliberately layout- and code-path-independent from
:mod:`.xunet` (which runs NHWC through :mod:`..ops`), so agreement between the
two is a real check of the re-designed execution path.
"""
from __future__ import annotations

import math
from typing import Dict

import torch
import torch.nn.functional as F

from ..ops import torch_impl as T


def _gn(sd, prefix, h, eps=1e-5):
    B, Fr, C, H, W = h.shape
    y = F.group_norm(h.reshape(B * Fr, C, H, W), 32, sd[prefix + ".gn.weight"], sd[prefix + ".gn.bias"], eps)
    return y.reshape(B, Fr, C, H, W)


def _conv(sd, prefix, h, stride=1, padding=1):
    B, Fr, C, H, W = h.shape
    y = F.conv2d(h.reshape(B * Fr, C, H, W), sd[prefix + ".weight"], sd[prefix + ".bias"],
                 stride=stride, padding=padding)
    return y.reshape(B, Fr, *y.shape[1:])


def _resblock(sd, p, h_in, emb, resample=None):
    B, Fr, C, H, W = h_in.shape
    h = F.silu(_gn(sd, p + ".groupnorm0", h_in))
    h = _conv(sd, p + ".conv1", h)
    h = _gn(sd, p + ".groupnorm1", h)
    Cout = h.shape[2]
    # FiLM: Linear over the channel axis of silu(emb)
    e = F.silu(emb).permute(0, 1, 3, 4, 2)
    e = F.linear(e, sd[p + ".film.dense.weight"], sd[p + ".film.dense.bias"]).permute(0, 1, 4, 2, 3)
    scale, shift = e[:, :, :Cout], e[:, :, Cout:]
    h = h * (1.0 + scale) + shift
    h = _conv(sd, p + ".conv2", h)
    if (p + ".dense.weight") in sd:
        h_in = _conv(sd, p + ".dense", h_in, padding=0)
    h = (h + h_in) / math.sqrt(2.0)
    if resample == "down":
        h = F.avg_pool2d(h.reshape(B * Fr, Cout, H, W), 2, 2).reshape(B, Fr, Cout, H // 2, W // 2)
    elif resample == "up":
        h = F.interpolate(h.reshape(B * Fr, Cout, H, W), scale_factor=2, mode="nearest")
        h = h.reshape(B, Fr, Cout, 2 * H, 2 * W)
    return h


def _mha(sd, p, q_in, kv_in, heads):
    # q_in, kv_in: [B, L, C]
    W_in, b_in = sd[p + ".in_proj_weight"], sd[p + ".in_proj_bias"]
    C = q_in.shape[-1]
    q = F.linear(q_in, W_in[:C], b_in[:C])
    k = F.linear(kv_in, W_in[C:2 * C], b_in[C:2 * C])
    v = F.linear(kv_in, W_in[2 * C:], b_in[2 * C:])
    B, L, _ = q.shape
    d = C // heads
    q, k, v = (t.reshape(B, L, heads, d).transpose(1, 2) for t in (q, k, v))
    a = torch.softmax(q @ k.transpose(-1, -2) / math.sqrt(d), dim=-1) @ v
    a = a.transpose(1, 2).reshape(B, L, C)
    return F.linear(a, sd[p + ".out_proj.weight"], sd[p + ".out_proj.bias"])


def _attnblock(sd, p, h_in, kind, heads):
    B, Fr, C, H, W = h_in.shape
    h = _gn(sd, p + ".groupnorm", h_in)
    h0 = h[:, 0].reshape(B, C, H * W).transpose(1, 2)
    h1 = h[:, 1].reshape(B, C, H * W).transpose(1, 2)
    mp = p + ".attn_layer.attn"
    if kind == "self":
        o0, o1 = _mha(sd, mp, h0, h0, heads), _mha(sd, mp, h1, h1, heads)
    else:
        o0, o1 = _mha(sd, mp, h0, h1, heads), _mha(sd, mp, h1, h0, heads)
    h = torch.stack([o0.transpose(1, 2), o1.transpose(1, 2)], 1).reshape(B, Fr, C, H, W)
    h = _conv(sd, p + ".linear", h, padding=0)
    return (h + h_in) / math.sqrt(2.0)


def _xblock(sd, p, h, emb, use_attn, heads):
    h = _resblock(sd, p + ".resnetblock", h, emb)
    if use_attn:
        h = _attnblock(sd, p + ".attnblock_self", h, "self", heads)
        h = _attnblock(sd, p + ".attnblock_cross", h, "cross", heads)
    return h


def reference_forward_grad(sd: Dict[str, torch.Tensor], batch: Dict[str, torch.Tensor], cond_mask: torch.Tensor,
                      ch_mult=(1, 2, 2, 4), num_res_blocks=3, attn_resolutions=(2, 3, 4), attn_heads=4,
                      emb_ch=1024, rescale_from: int = 0) -> torch.Tensor:
    """Eval-mode (no dropout) fp32 forward of the reference X-UNet."""
    sd = {k[7:] if k.startswith("module.") else k: v if v.dtype == torch.float32 else v.float()
          for k, v in sd.items()}
    x, z = batch["x"].float(), batch["z"].float()
    B, _, H, W = x.shape
    L = len(ch_mult)
    cp = "conditioningprocessor"
    logsnr = torch.clip(batch["logsnr"].float(), -20, 20)
    le = T.posenc_ddpm(logsnr, emb_ch, 1.0)
    le = F.linear(F.silu(F.linear(le, sd[cp + ".logsnr_emb_emb.0.weight"], sd[cp + ".logsnr_emb_emb.0.bias"])),
                  sd[cp + ".logsnr_emb_emb.2.weight"], sd[cp + ".logsnr_emb_emb.2.bias"])      # [B,2,E]
    pos, dirs = T.camera_rays(batch["R"], batch["t"], batch["K"], H, W, rescale_from)
    pe = torch.cat([T.posenc_nerf(pos, 0, 15), T.posenc_nerf(dirs, 0, 8)], -1)                 # [B,2,H,W,144]
    pe = torch.where(cond_mask.bool().view(B, 1, 1, 1, 1), pe, torch.zeros_like(pe))
    pe = pe.permute(0, 1, 4, 2, 3)
    if cp + ".pos_emb" in sd:
        pe = pe + sd[cp + ".pos_emb"][None, None]
    if cp + ".first_emb" in sd:
        pe = torch.cat([sd[cp + ".first_emb"], sd[cp + ".other_emb"]], 1) + pe
    pose_embs = [_conv(sd, f"{cp}.convs.{i}", pe, stride=2 ** i) for i in range(L)]
    embs = [le[..., None, None] + pose_embs[i] for i in range(L)]

    h = _conv(sd, "conv", torch.stack([x, z], 1))
    hs = [h]
    for i in range(L):
        for j in range(num_res_blocks):
            h = _xblock(sd, f"xunetblocks.{i}.{j}", h, embs[i], i in attn_resolutions, attn_heads)
            hs.append(h)
        if i != L - 1:
            h = _resblock(sd, f"xunetblocks.{i}.{num_res_blocks}", h, embs[i], "down")
            hs.append(h)
    h = _xblock(sd, "middle", h, embs[-1], L in attn_resolutions, attn_heads)
    for i in reversed(range(L)):
        for j in range(num_res_blocks + 1):
            h = torch.cat([h, hs.pop()], 2)
            h = _xblock(sd, f"upsample.{i}.{j}", h, embs[i], i in attn_resolutions, attn_heads)
        if i != 0:
            h = _resblock(sd, f"upsample.{i}.{num_res_blocks + 1}", h, embs[i], "up")
    h = F.silu(_gn(sd, "lastgn", h))
    return _conv(sd, "lastconv", h)[:, 1]


@torch.no_grad()
def reference_forward(sd, batch, cond_mask, **kw) -> torch.Tensor:
    """Eval-mode (no dropout) fp32 forward of the reference X-UNet (no grad)."""
    return reference_forward_grad(sd, batch, cond_mask, **kw)
