"""Pure-PyTorch implementations of the NHWC op set.

These are the numerics oracle for the HIP kernels (fp32 composition of the
same op) and the CPU execution path.  Layout convention everywhere in the
framework: activations are ``[N, H, W, C]`` with ``N = 2*B`` and the two views
of an example adjacent (``n = 2*b + frame``), i.e. the reference's
``[B, F=2, C, H, W]`` (`xunet.py:61-71`) folded frame-into-batch, channels-last.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn.functional as F

INV_SQRT2 = 1.0 / math.sqrt(2.0)


def _cast(t: Optional[torch.Tensor], dtype: torch.dtype) -> Optional[torch.Tensor]:
    if t is None:
        return None
    return t if t.dtype == dtype else t.to(dtype)


def group_norm(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, groups: int = 32,
               eps: float = 1e-5, silu: bool = False) -> torch.Tensor:
    """GroupNorm over each (example, frame) image; optional fused SiLU.
    Matches ``nn.GroupNorm(32, C)`` on the frame-folded batch (`xunet.py:61-71`)."""
    N, H, W, C = x.shape
    xf = x.float().reshape(N, H * W, groups, C // groups)
    mean = xf.mean(dim=(1, 3), keepdim=True)
    var = xf.var(dim=(1, 3), unbiased=False, keepdim=True)
    y = (xf - mean) * torch.rsqrt(var + eps)
    y = y.reshape(N, H, W, C) * weight.float() + bias.float()
    if silu:
        y = F.silu(y)
    return y.to(x.dtype)


def dropout_mask(shape, p: float, seed: int, device) -> torch.Tensor:
    g = torch.Generator(device="cpu")
    g.manual_seed(int(seed) & 0x7FFFFFFFFFFFFFFF)
    keep = (torch.rand(shape, generator=g) >= p).to(device)
    return keep


def gn_film(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, ss: torch.Tensor,
            groups: int = 32, eps: float = 1e-5, dropout_p: float = 0.0,
            training: bool = False, seed: int = 0, ss_map: Optional[torch.Tensor] = None) -> torch.Tensor:
    """dropout(GN(x) * (1 + scale) + shift); ``ss = [scale | shift]`` on the
    channel axis (FiLM, `xunet.py:74-87`; ResBlock ordering `xunet.py:140-146`).
    ``ss_map``: image n takes the modulation ss[ss_map[n]]."""
    C = x.shape[-1]
    h = group_norm(x, weight, bias, groups, eps).float()
    if ss_map is not None:
        ss = ss.index_select(0, ss_map.long())
    ssf = ss.float()
    y = h * (1.0 + ssf[..., :C]) + ssf[..., C:]
    if training and dropout_p > 0.0:
        y = F.dropout(y, dropout_p, training=True)
    return y.to(x.dtype)


def conv3x3(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor], stride: int = 1,
            residual: Optional[torch.Tensor] = None, out_scale: float = 1.0,
            row_bias: Optional[torch.Tensor] = None, res_period: int = 0) -> torch.Tensor:
    """3x3 conv, padding 1, on NHWC.  Epilogue: + row_bias[n] (per image),
    + residual (broadcast as residual[n % res_period] when res_period > 0),
    * out_scale."""
    dt = x.dtype
    y = F.conv2d(x.permute(0, 3, 1, 2), _cast(weight, dt), _cast(bias, dt), stride=stride, padding=1)
    y = y.permute(0, 2, 3, 1)
    if row_bias is not None:
        y = y + row_bias.to(dt)[:, None, None, :]
    if residual is not None:
        if res_period:
            residual = residual.repeat(y.shape[0] // res_period, 1, 1, 1)
        y = y + residual
    if out_scale != 1.0:
        y = y * out_scale
    return y.contiguous()


def linear(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor],
           residual: Optional[torch.Tensor] = None, out_scale: float = 1.0) -> torch.Tensor:
    """Per-pixel dense layer (1x1 conv / nn.Linear) with fused residual epilogue."""
    dt = x.dtype
    w = weight.reshape(weight.shape[0], -1)
    y = F.linear(x, _cast(w, dt), _cast(bias, dt))
    if residual is not None:
        y = y + residual
    if out_scale != 1.0:
        y = y * out_scale
    return y


def attention(qkv: torch.Tensor, heads: int, cross: bool) -> torch.Tensor:
    """Multi-head attention within an example: queries of frame f attend to
    keys/values of frame f (self) or frame 1-f (cross) (`xunet.py:202-211`).
    ``qkv``: [N, L, 3C] (packed in_proj output).  Returns [N, L, C]."""
    N, L, C3 = qkv.shape
    C = C3 // 3
    d = C // heads
    q, k, v = qkv.split(C, dim=-1)
    if cross:
        perm = torch.arange(N, device=qkv.device) ^ 1
        k = k[perm]
        v = v[perm]
    q = q.reshape(N, L, heads, d).transpose(1, 2)
    k = k.reshape(N, L, heads, d).transpose(1, 2)
    v = v.reshape(N, L, heads, d).transpose(1, 2)
    s = torch.matmul(q.float(), k.float().transpose(-1, -2)) * (1.0 / math.sqrt(d))
    p = torch.softmax(s, dim=-1)
    o = torch.matmul(p, v.float()).to(qkv.dtype)
    return o.transpose(1, 2).reshape(N, L, C)


def avgpool2(x: torch.Tensor) -> torch.Tensor:
    N, H, W, C = x.shape
    return x.reshape(N, H // 2, 2, W // 2, 2, C).float().mean(dim=(2, 4)).to(x.dtype)


def upsample2(x: torch.Tensor) -> torch.Tensor:
    N, H, W, C = x.shape
    return x[:, :, None, :, None, :].expand(N, H, 2, W, 2, C).reshape(N, 2 * H, 2 * W, C)


def silu(x: torch.Tensor) -> torch.Tensor:
    return F.silu(x)


def camera_rays(R: torch.Tensor, t: torch.Tensor, K: torch.Tensor, H: int, W: int,
                rescale_from: int = 0):
    """Per-pixel world rays of a pinhole camera (OpenCV convention, pixel
    centres at +0.5), following visu3d's ``Camera.rays()`` as used in
    `xunet.py:311-314`: ``pos = t``, ``dir = R @ normalize(K^-1 [u+.5, v+.5, 1])``.

    R: [B,F,3,3] cam-to-world rotation, t: [B,F,3], K: [B,3,3].
    Returns pos, dir: [B,F,H,W,3] in fp32 (computed in fp64).
    """
    dt = torch.float64
    Rd, td, Kd = R.to(dt), t.to(dt), K.to(dt)
    if rescale_from:
        s = torch.tensor([W / rescale_from, H / rescale_from, 1.0], dtype=dt, device=K.device)
        Kd = Kd * s[None, :, None]
    dev = R.device
    u = torch.arange(W, dtype=dt, device=dev) + 0.5
    v = torch.arange(H, dtype=dt, device=dev) + 0.5
    vv, uu = torch.meshgrid(v, u, indexing="ij")
    pix = torch.stack([uu, vv, torch.ones_like(uu)], dim=-1)          # [H,W,3]
    Kinv = torch.linalg.inv(Kd)                                        # [B,3,3]
    d_cam = torch.einsum("bij,hwj->bhwi", Kinv, pix)                   # [B,H,W,3]
    d_cam = d_cam / d_cam.norm(dim=-1, keepdim=True)
    d_world = torch.einsum("bfij,bhwj->bfhwi", Rd, d_cam)              # [B,F,H,W,3]
    B, Fr = R.shape[:2]
    pos = td[:, :, None, None, :].expand(B, Fr, H, W, 3)
    return pos.float(), d_world.float()


def posenc_nerf(x: torch.Tensor, min_deg: int, max_deg: int) -> torch.Tensor:
    """[x, sin(x*2^k), sin(x*2^k + pi/2)] with scale-major / xyz-minor packing
    (`xunet.py:49-59`)."""
    if min_deg == max_deg:
        return x
    # exact powers of two built on the device (no host->device copy: graph-capturable)
    scales = torch.pow(2.0, torch.arange(min_deg, max_deg, device=x.device, dtype=torch.float32)).to(x.dtype)
    xb = (x[..., None, :] * scales[:, None]).flatten(-2)
    emb = torch.sin(torch.cat([xb, xb + math.pi / 2.0], dim=-1))
    return torch.cat([x, emb], dim=-1)


def posenc_ddpm(t: torch.Tensor, emb_ch: int, max_time: float = 1.0) -> torch.Tensor:
    """DDPM sinusoidal embedding of (clipped) logSNR, t*1000/max_time
    (`xunet.py:32-46`)."""
    t = t.float() * (1000.0 / max_time)
    half = emb_ch // 2
    k = torch.arange(half, dtype=torch.float32, device=t.device)
    freqs = torch.exp(k * (-math.log(10000.0) / (half - 1)))
    arg = t[..., None] * freqs
    return torch.cat([torch.sin(arg), torch.cos(arg)], dim=-1)


def logsnr_mlp(logsnr: torch.Tensor, w1, b1, w2, b2, max_time: float = 1.0) -> torch.Tensor:
    """[B, 2] logSNR -> [2B, E] fp32: clip +-20, DDPM posenc, Linear-SiLU-Linear
    (`xunet.py:273-277,305-308`)."""
    E = w1.shape[0]
    l = torch.clamp(logsnr.float(), -20.0, 20.0)
    e = posenc_ddpm(l, E, max_time=max_time).reshape(-1, E)
    return torch.nn.functional.linear(torch.nn.functional.silu(torch.nn.functional.linear(e, w1, b1)), w2, b2)


def ray_posenc(R: torch.Tensor, t: torch.Tensor, K: torch.Tensor, H: int, W: int,
               cond_mask: torch.Tensor, pos_emb: Optional[torch.Tensor],
               first_emb: Optional[torch.Tensor], other_emb: Optional[torch.Tensor],
               rescale_from: int = 0) -> torch.Tensor:
    """144-channel camera conditioning input, NHWC frame-interleaved
    [2B, H, W, 144] in fp32 (`xunet.py:311-336`): rays -> NeRF posenc (origins
    deg 0..15, directions deg 0..8) -> zeroed for unconditional examples ->
    + learned pos_emb[144,H,W] -> + per-frame embedding."""
    pos, dirs = camera_rays(R, t, K, H, W, rescale_from)
    emb = torch.cat([posenc_nerf(pos, 0, 15), posenc_nerf(dirs, 0, 8)], dim=-1)  # [B,2,H,W,144]
    emb = torch.where(cond_mask.view(-1, 1, 1, 1, 1), emb, torch.zeros_like(emb))
    if pos_emb is not None:
        emb = emb + pos_emb.permute(1, 2, 0)[None, None]
    if first_emb is not None:
        fe = torch.cat([first_emb, other_emb], dim=1).reshape(1, 2, 1, 1, -1)
        emb = emb + fe
    B = emb.shape[0]
    return emb.reshape(B * 2, H, W, emb.shape[-1])


def film_batch(emb, weights, biases):
    """Level-batched FiLM projections (oracle): ``silu(emb)`` through one linear
    over the concatenated weights, split into per-block ``[.., 2C_i]``
    modulations (`xunet.py:84-87`)."""
    semb = F.silu(emb)
    y = F.linear(semb, torch.cat([w.to(semb.dtype) for w in weights], 0),
                 torch.cat([b.to(semb.dtype) for b in biases], 0))
    return tuple(torch.split(y, [w.shape[0] for w in weights], dim=-1))


def ray_posenc_dir(R, t, K, H, W, cond_mask, rescale_from: int = 0, ld: int = 64):
    """Direction half of the ray conditioning (channels 93..143 of
    :func:`ray_posenc`, masked, no learned embeddings), zero-padded to ``ld``
    channels: [2B, H, W, ld] fp32."""
    _, dirs = camera_rays(R, t, K, H, W, rescale_from)
    emb = posenc_nerf(dirs, 0, 8)
    emb = torch.where(cond_mask.view(-1, 1, 1, 1, 1), emb, torch.zeros_like(emb))
    B = emb.shape[0]
    emb = emb.reshape(B * 2, H, W, emb.shape[-1])
    return F.pad(emb, (0, ld - emb.shape[-1]))


def ray_origin_pe(t, cond_mask):
    """Origin half (channels 0..92): NeRF posenc of the camera position, which
    is the same for every pixel of an image: [2B, 93] fp32."""
    B = t.shape[0]
    pe = posenc_nerf(t.float().reshape(B * 2, 3), 0, 15)
    m = cond_mask.to(pe.dtype).repeat_interleave(2)
    return pe * m[:, None]


def cond_conv(rays_dir, orig_pe, weight, bias, stride, row_bias=None, residual=None, res_period=0):
    """Conditioning conv on the split ray input (oracle): rebuild the 144
    channels (origin broadcast over pixels + direction) and convolve."""
    N, H, W, _ = rays_dir.shape
    nd = weight.shape[1] - orig_pe.shape[1]
    full = torch.cat([orig_pe[:, None, None, :].to(rays_dir.dtype).expand(N, H, W, orig_pe.shape[1]),
                      rays_dir[..., :nd]], dim=-1)
    return conv3x3(full, weight, bias, stride, residual, 1.0, row_bias, res_period)


def cat_gn_silu_dense(a, b, gw, gb, dw, db, groups: int = 32, eps: float = 1e-5):
    """silu(GN(cat[a, b])) and dense(cat[a, b]) (decoder block entry, oracle)."""
    x = torch.cat([a, b], -1)
    return group_norm(x, gw, gb, groups, eps, True), linear(x, dw, db)


# ------------------------------------------------ training-input draw ----
# Counter-based RNG shared bit-for-bit with the HIP kernels (common.h
# hash_u32 / normal01; elementwise.hip diffusion_fwd2_k): splitmix64 of
# (seed, index) in wrapping int64 arithmetic with logical shifts.
_M64 = (1 << 64) - 1
GOLDEN = 0x9E3779B97F4A7C15
K_EPS = 0x5851F42D4C957F2D
K_XN = 0x14057B7EF767814F
K_XU = 0xA0761D6478BD642F       # sampler: unconditional-pass input noise
K_NZ = 0xE7037ED1A0B428DB       # sampler: ancestral-step noise
K_Z0 = 0x8EBC6AF09C88C6E3       # sampler: initial z


def _s64(v: int) -> int:
    v &= _M64
    return v - (1 << 64) if v >= (1 << 63) else v


def _lsr(z: torch.Tensor, k: int) -> torch.Tensor:
    return (z >> k) & ((1 << (64 - k)) - 1)


def hash_u32(seed: int, idx: torch.Tensor) -> torch.Tensor:
    """common.h ``hash_u32`` on an int64 index tensor -> values in [0, 2^32)."""
    z = idx.to(torch.int64) + _s64(seed * GOLDEN + 0x632BE59BD9B4E019)
    z = (z ^ _lsr(z, 30)) * _s64(0xBF58476D1CE4E5B9)
    z = (z ^ _lsr(z, 27)) * _s64(0x94D049BB133111EB)
    z = z ^ _lsr(z, 31)
    return _lsr(z, 32)


def u01(seed: int, idx: torch.Tensor) -> torch.Tensor:
    return (hash_u32(seed, idx) >> 8).to(torch.float32) * (1.0 / 16777216.0)


def normal01(seed: int, idx: torch.Tensor) -> torch.Tensor:
    idx = idx.to(torch.int64)
    u1 = ((hash_u32(seed, 2 * idx) >> 8) + 1).to(torch.float32) * torch.tensor(1.0 / 16777217.0)
    u2 = (hash_u32(seed, 2 * idx + 1) >> 8).to(torch.float32) * (1.0 / 16777216.0)
    return torch.sqrt(-2.0 * torch.log(u1)) * torch.cos(6.283185307179586 * u2)


def schedule_ab(logsnr_min: float, logsnr_max: float):
    b = math.atan(math.exp(-0.5 * logsnr_max))
    a = math.atan(math.exp(-0.5 * logsnr_min)) - b
    return a, b


def diffusion_inputs(img: torch.Tensor, seed: int, e0: int = 0, cond_prob: float = 0.1,
                     logsnr_min: float = -20.0, logsnr_max: float = 20.0, dtype=torch.float32):
    """The training-input draw of `train.py:80-100` for examples
    ``e0 .. e0+B-1`` of a step whose RNG seed is ``seed`` (same numbers as
    ``diffusion_fwd2_k``).  img [B,2,3,H,W] -> (xz [2B,H,W,8] NHWC stem input
    (frame 0 = CFG-dropped x, frame 1 = z_t; channels 3..7 zero), eps
    [B,3,H,W] fp32, logsnr [B,2], keep [B] bool)."""
    B, _, C, H, W = img.shape
    HW = H * W
    dev = img.device
    s = seed & _M64
    g = torch.arange(B, device=dev, dtype=torch.int64) + e0
    a, b = schedule_ab(logsnr_min, logsnr_max)
    af, bf = torch.tensor(a, dtype=torch.float32), torch.tensor(b, dtype=torch.float32)
    t = u01(s, 4 * g)
    lam = -2.0 * torch.log(torch.tan(af.to(dev) * t + bf.to(dev)))
    keep = u01(s, 4 * g + 1) > cond_prob
    lam0 = (-2.0 * torch.log(torch.tan(bf))).to(dev).expand(B)
    idx = g[:, None, None] * (3 * HW) + torch.arange(3, device=dev)[None, :, None] * HW + \
        torch.arange(HW, device=dev)[None, None, :]
    eps = normal01(s ^ K_EPS, idx).reshape(B, 3, H, W)
    xn = normal01(s ^ K_XN, idx).reshape(B, 3, H, W)
    alpha = torch.sqrt(torch.sigmoid(lam)).view(B, 1, 1, 1)
    sigma = torch.sqrt(torch.sigmoid(-lam)).view(B, 1, 1, 1)
    x, z = img[:, 0].float(), img[:, 1].float()
    xc = torch.where(keep.view(B, 1, 1, 1), x, xn)
    zt = alpha * z + sigma * eps
    xz = torch.zeros(B, 2, H, W, 8, dtype=dtype, device=dev)
    xz[:, 0, ..., :3] = xc.permute(0, 2, 3, 1).to(dtype)
    xz[:, 1, ..., :3] = zt.permute(0, 2, 3, 1).to(dtype)
    return xz.reshape(2 * B, H, W, 8), eps, torch.stack([lam0, lam], 1), keep


def diff_loss_nhwc(y: torch.Tensor, eps: torch.Tensor, loss_type: str = "l2") -> torch.Tensor:
    """Epsilon loss (`train.py:102-112`) on the NHWC head output y [B,H,W,>=3]
    (only the first 3 channels are the prediction) against eps [B,3,H,W]."""
    yh = y[..., :3].permute(0, 3, 1, 2).float()
    if loss_type == "l2":
        return torch.mean((eps.float() - yh) ** 2)
    if loss_type == "l1":
        return torch.mean((eps.float() - yh).abs())
    if loss_type == "huber":
        return F.smooth_l1_loss(yh, eps.float())
    raise NotImplementedError(loss_type)
