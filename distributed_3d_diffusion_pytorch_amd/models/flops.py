"""Analytic forward FLOP count of an X-UNet (multiply-add = 2 FLOPs).

Walks the module tree with the resolution routing of ``XUNet.forward``
(reference `xunet.py:477-536`): every 3x3 conv, 1x1 NIN skip, FiLM
projection, attention projection / core / 1x1, the conditioning convs and the
logSNR MLP.  Normalisation and elementwise work is not counted (< 0.1 %).

Two parts are reported separately because the sampler's shared-conditioning
path runs them on fewer images than the trunk:
  * ``trunk``: per (example, frame) image -- stem, ResBlock convs / skips,
    attention, head;
  * ``cond``: per CONDITIONING image -- FiLM projections, conditioning convs,
    logSNR MLP (``XUNet.forward(shared_cond=)`` runs them on the distinct
    conditioning examples only).

At 64x64 / ch 128 one training example (2 images, both frames through the
head as in the reference) is 235.9 GFLOP, SURVEY Appendix C's measured figure
(tests/test_model.py pins the match).
"""
from __future__ import annotations

from typing import Dict, Optional


def _resblock(blk, hw: int):
    i, o = blk.in_features, blk.features
    t = 2 * 9 * i * o * hw + 2 * 9 * o * o * hw
    if i != o:
        t += 2 * i * o * hw                          # 1x1 NIN skip (xunet.py:129)
    c = 2 * blk.film.dense.in_features * 2 * o * hw  # FiLM projection (xunet.py:84)
    return t, c


def _attn(blk, hw: int) -> int:
    C = blk.in_channels
    # q/k/v projections, QK^T + PV over all heads, out_proj, the 1x1 linear
    return 2 * hw * C * 3 * C + 4 * hw * hw * C + 2 * hw * C * C + 2 * hw * C * C


def image_flops(model) -> Dict[str, float]:
    """Forward FLOPs of ONE image (one frame of one example): ``trunk`` and
    ``cond`` (the conditioning-dependent part), plus ``head`` (the output conv,
    which the framework runs on frame 1 only)."""
    from .xunet import ResnetBlock, XUNetBlock
    H, W = model.H, model.W
    L = model.num_resolutions
    hw = [(H >> i) * (W >> i) for i in range(L)]
    trunk = cond = 0

    def block(b, r):
        nonlocal trunk, cond
        rb = b.resnetblock if isinstance(b, XUNetBlock) else b
        assert isinstance(rb, ResnetBlock)
        t, c = _resblock(rb, r)
        trunk += t
        cond += c
        if isinstance(b, XUNetBlock) and b.use_attn:
            trunk += _attn(b.attnblock_self, r) + _attn(b.attnblock_cross, r)

    trunk += 2 * 9 * model.conv.in_channels * model.conv.out_channels * hw[0]        # stem
    for i in range(L):
        for b in model.xunetblocks[i]:
            block(b, hw[i])
    block(model.middle, hw[L - 1])
    for i in reversed(range(L)):
        for b in model.upsample[str(i)]:
            block(b, hw[i])
    head = 2 * 9 * model.lastconv.in_channels * model.lastconv.out_channels * hw[0]
    cp = model.conditioningprocessor
    for i, conv in enumerate(cp.convs):
        cond += 2 * 9 * conv.in_channels * conv.out_channels * hw[i]
    l0, _, l1 = cp.logsnr_emb_emb
    cond += 2 * l0.in_features * l0.out_features + 2 * l1.in_features * l1.out_features
    return {"trunk": float(trunk), "cond": float(cond), "head": float(head)}


def forward_flops(model, batch: int, cond_examples: Optional[int] = None, head_frames: int = 1) -> float:
    """Executed forward FLOPs of ``batch`` examples (2 images each) with the
    conditioning part on ``cond_examples`` examples (default: all of them;
    the shared-conditioning sampler passes its distinct classes) and the head
    on ``head_frames`` frames per example (1 here; the reference runs 2)."""
    f = image_flops(model)
    ce = batch if cond_examples is None else cond_examples
    return 2 * batch * f["trunk"] + 2 * ce * f["cond"] + head_frames * batch * f["head"]


def reference_example_flops(model) -> float:
    """Forward FLOPs of one training example as the reference executes it
    (both frames through the head): 235.9 GFLOP at 64x64 / ch 128."""
    return forward_flops(model, 1, head_frames=2)
