"""Numerics of every HIP kernel against the fp32 PyTorch composition of the
same op (ops.torch_impl) on identical bf16-rounded inputs.  GPU only."""
import ctypes
import math
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from distributed_3d_diffusion_pytorch_amd.ops import torch_impl as T  # noqa: E402

DEV = "cuda"
BF = torch.bfloat16


@pytest.fixture(scope="module")
def H():
    from distributed_3d_diffusion_pytorch_amd.ops import hip_impl
    return hip_impl


@pytest.fixture
def no_gn_img(H):
    """Whole-image GroupNorm kernels off for the test (it pins the epilogue
    statistics path, which small images no longer take by default)."""
    prev = H._lib.d3d_gn_img_cfg(-1)
    H._lib.d3d_gn_img_cfg(0)
    yield
    H._lib.d3d_gn_img_cfg(prev)


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


def leaf(t, dtype=None):
    t = t.detach().clone()
    if dtype is not None:
        t = t.to(dtype)
    return t.requires_grad_(True)


def run_both(fn_hip, fn_ref, inputs, grad_out):
    """Run fwd+bwd of HIP op (bf16 inputs) and reference (fp32 copies)."""
    xh = [leaf(x) for x in inputs]
    xr = [leaf(x, torch.float32) if x.dtype == BF else leaf(x) for x in inputs]
    yh = fn_hip(*xh)
    yr = fn_ref(*xr)
    yh.backward(grad_out.to(yh.dtype))
    yr.backward(grad_out.float())
    return yh, yr, [a.grad for a in xh], [b.grad for b in xr]


@pytest.mark.parametrize("N,Hh,W,C,silu", [(4, 16, 16, 128, True), (2, 8, 8, 256, False), (3, 8, 8, 384, True),
                                           (2, 4, 4, 1024, False), (2, 32, 32, 768, True)])
def test_group_norm(H, N, Hh, W, C, silu):
    torch.manual_seed(0)
    x = (torch.randn(N, Hh, W, C, device=DEV) * 2 + 0.5).to(BF)
    w = torch.randn(C, device=DEV) * 0.5 + 1
    b = torch.randn(C, device=DEV) * 0.1
    go = torch.randn(N, Hh, W, C, device=DEV)
    yh, yr, gh, gr = run_both(lambda x, w, b: H.group_norm(x, w, b, 32, 1e-5, silu),
                              lambda x, w, b: T.group_norm(x, w, b, 32, 1e-5, silu), [x, w, b], go)
    assert rel(yh, yr) < 2e-2
    assert rel(gh[0], gr[0]) < 3e-2
    assert rel(gh[1], gr[1]) < 1e-2
    assert rel(gh[2], gr[2]) < 1e-2


@pytest.mark.parametrize("G,C", [(1, 128), (4, 128), (8, 256), (16, 384), (64, 256)])
def test_group_norm_group_counts(H, G, C):
    """Group counts other than 32: the backward's per-block group reduction
    splits each group over a power-of-two lane team (64 lanes at G <= 4, one
    lane at G >= 256) -- every team width of the rule is exercised."""
    torch.manual_seed(5)
    x = (torch.randn(2, 16, 16, C, device=DEV) * 2 + 0.5).to(BF)
    w = torch.randn(C, device=DEV) * 0.5 + 1
    b = torch.randn(C, device=DEV) * 0.1
    go = torch.randn(2, 16, 16, C, device=DEV)
    yh, yr, gh, gr = run_both(lambda x, w, b: H.group_norm(x, w, b, G, 1e-5, True),
                              lambda x, w, b: T.group_norm(x, w, b, G, 1e-5, True), [x, w, b], go)
    assert rel(yh, yr) < 2e-2
    assert rel(gh[0], gr[0]) < 3e-2
    assert rel(gh[1], gr[1]) < 1e-2
    assert rel(gh[2], gr[2]) < 1e-2


@pytest.mark.parametrize("N,Hh,W,C", [(4, 16, 16, 128), (2, 8, 8, 512)])
def test_gn_film(H, N, Hh, W, C):
    torch.manual_seed(1)
    x = torch.randn(N, Hh, W, C, device=DEV).to(BF)
    w = torch.randn(C, device=DEV) * 0.5 + 1
    b = torch.randn(C, device=DEV) * 0.1
    ss = (torch.randn(N, Hh, W, 2 * C, device=DEV) * 0.5).to(BF)
    go = torch.randn(N, Hh, W, C, device=DEV)
    yh, yr, gh, gr = run_both(lambda x, w, b, ss: H.gn_film(x, w, b, ss, 32, 1e-5, 0.0, False, 0),
                              lambda x, w, b, ss: T.gn_film(x, w, b, ss, 32, 1e-5, 0.0, False, 0), [x, w, b, ss], go)
    assert rel(yh, yr) < 2e-2
    for a, c in zip(gh, gr):
        assert rel(a, c) < 3e-2


def test_gn_film_ss_map(H):
    """Shared-conditioning GN-FiLM: image n modulated by class ss_map[n] of a
    strided level-batched modulation == the torch op on the gathered ss."""
    torch.manual_seed(4)
    N, Hh, C = 6, 8, 256
    x = torch.randn(N, Hh, Hh, C, device=DEV).to(BF)
    w = torch.randn(C, device=DEV) * 0.5 + 1
    b = torch.randn(C, device=DEV) * 0.1
    parent = (torch.randn(4, Hh, Hh, 3 * 2 * C, device=DEV) * 0.5).to(BF)
    ss = parent[..., 2 * C:4 * C]                    # channel slice, ld = 6C
    smap = torch.tensor([0, 1, 2, 3, 0, 3], dtype=torch.int32, device=DEV)
    with torch.no_grad():
        y = H.gn_film(x, w, b, ss, 32, 1e-5, 0.0, False, 0, smap)
        yr = T.gn_film(x.float(), w, b, ss.float()[smap.long()], 32, 1e-5, 0.0, False, 0)
    assert rel(y, yr) < 1e-2
    with pytest.raises(RuntimeError):
        H.gn_film(x, w.clone().requires_grad_(True), b, ss, 32, 1e-5, 0.0, False, 0, smap)


def test_gn_film_dropout(H):
    torch.manual_seed(2)
    N, Hh, W, C, p = 2, 16, 16, 128, 0.1
    x = torch.randn(N, Hh, W, C, device=DEV).to(BF)
    w = torch.ones(C, device=DEV)
    b = torch.zeros(C, device=DEV)
    ss = torch.zeros(N, Hh, W, 2 * C, device=DEV).to(BF)
    xh = leaf(x)
    ssh = leaf(ss)
    y = H.gn_film(xh, w, b, ssh, 32, 1e-5, p, True, 1234)
    y0 = H.gn_film(x, w, b, ss, 32, 1e-5, 0.0, False, 0)
    dropped = (y == 0) & (y0 != 0)
    frac = dropped.float().mean().item()
    assert abs(frac - p) < 0.01
    kept = ~dropped
    assert rel(y[kept], (y0 * (1 / (1 - p)))[kept]) < 1e-2
    # same seed -> same mask; backward uses the regenerated mask
    y2 = H.gn_film(x, w, b, ss, 32, 1e-5, p, True, 1234)
    assert torch.equal(y, y2)
    y.backward(torch.ones_like(y))
    # d shift = dz = keep/(1-p)
    dshift = ssh.grad[..., C:]
    assert torch.equal(dshift == 0, dropped)


def test_gn_whole_image_batch_rule(H):
    """The 32x32 level takes the whole-image kernels only for batches of
    64..128 images (norm.hip img_plan; measured per batch size), and every
    caller sees the same answer for one shape."""
    assert H._lib.d3d_gn_img_cfg(-1) == 256
    assert H.gn_img_ok(256, 256, 32, 32) and H.gn_img_ok(256, 256, 32)
    for n, want in ((32, False), (64, True), (128, True), (256, False), (0, False)):
        assert H.gn_img_ok(1024, 256, 32, n) == want, n
    lo = H._lib.d3d_gn_img_wide_cfg(-1, 0)
    try:
        H._lib.d3d_gn_img_wide_cfg(1 << 30, 0)
        assert not H.gn_img_ok(1024, 256, 32, 64)
    finally:
        H._lib.d3d_gn_img_wide_cfg(lo, 128)
    assert H.gn_img_ok(1024, 256, 32, 64)


@pytest.mark.parametrize("N,Hh,C,C1,mode,maxp", [
    (32, 8, 512, 0, 1, 256), (32, 16, 256, 0, 2, 256), (32, 8, 512, 0, 0, 256), (5, 16, 768, 512, 1, 256),
    (4, 8, 1024, 512, 1, 256), (3, 8, 768, 256, 1, 256), (6, 4, 256, 0, 2, 256), (4, 32, 256, 0, 1, 1024),
    (3, 32, 256, 0, 2, 1024)])
def test_gn_whole_image(H, N, Hh, C, C1, mode, maxp):
    """Whole-image GroupNorm kernels (norm.hip gn_img_*: statistics and the
    backward reductions inside one block per (image, channel slab), one
    launch per pass): forward and every gradient against the fp32 torch
    composition and against the chunked kernels on the same inputs; with a
    virtual concat [a | b] (C1 > 0, 24-channel groups at C = 768), dropout
    (mode 2), and the 512-thread form (32x32, maxp 1024)."""
    torch.manual_seed(31)
    x = (torch.randn(N, Hh, Hh, C, device=DEV) * 1.7 + 0.4).to(BF)
    w = torch.randn(C, device=DEV) * 0.5 + 1
    b = torch.randn(C, device=DEV) * 0.1
    ss = (torch.randn(N, Hh, Hh, 2 * C, device=DEV) * 0.5).to(BF)
    go = torch.randn(N, Hh, Hh, C, device=DEV)
    p = 0.1 if mode == 2 else 0.0

    def hip(*ins):
        if C1:
            return H.cat_gn_silu_dense(ins[0][..., :C1].contiguous(), ins[0][..., C1:].contiguous(), ins[1], ins[2],
                                       wd, None)[0]
        if mode == 2:
            return H.gn_film(ins[0], ins[1], ins[2], ins[3], 32, 1e-5, p, True, 77)
        return H.group_norm(ins[0], ins[1], ins[2], 32, 1e-5, mode == 1)

    wd = torch.randn(64, C, device=DEV) / 30
    ins = [x, w, b] + ([ss] if mode == 2 else [])
    prev = H._lib.d3d_gn_img_cfg(-1)
    try:
        H._lib.d3d_gn_img_cfg(maxp)
        assert H.gn_img_ok(Hh * Hh, C, 32)
        xi = [leaf(t) for t in ins]
        yi = hip(*xi)
        yi.backward(go.to(yi.dtype))
        H._lib.d3d_gn_img_cfg(0)                       # the chunked kernels, same inputs
        assert not H.gn_img_ok(Hh * Hh, C, 32)
        xc = [leaf(t) for t in ins]
        yc = hip(*xc)
        yc.backward(go.to(yc.dtype))
    finally:
        H._lib.d3d_gn_img_cfg(prev)
    torch.cuda.synchronize()
    assert rel(yi, yc) < 1e-2, rel(yi, yc)
    for a, c in zip(xi, xc):
        assert rel(a.grad, c.grad) < 2e-2, rel(a.grad, c.grad)
    if not C1:
        xr = [leaf(t, torch.float32) if t.dtype == BF else leaf(t) for t in ins]
        if mode == 2:
            # the fp32 composition with the kernel's own dropout mask (identity when p = 0)
            keep = (H.gn_film(x, torch.ones_like(w), torch.zeros_like(b), torch.zeros_like(ss) , 32, 1e-5, p, True, 77)
                    != 0).float()
            yr = T.gn_film(*xr, 32, 1e-5, 0.0, False, 0) * keep / (1 - p)
        else:
            yr = T.group_norm(*xr, 32, 1e-5, mode == 1)
        yr.backward(go)
        assert rel(yi, yr) < 2e-2, rel(yi, yr)
        for a, c in zip(xi, xr):
            assert rel(a.grad, c.grad) < 3e-2, rel(a.grad, c.grad)


@pytest.mark.parametrize("split", [False, True])
@pytest.mark.parametrize("N,L,C", [(8, 256, 256), (16, 64, 512), (3, 100, 256)])
def test_attn_out_merged(H, N, L, C, split, monkeypatch):
    """AttnBlock output map out_proj -> 1x1 linear as ONE merged GEMM
    (hip_impl.attn_out: W = W_lin W_out, b = W_lin b_out + b_lin; input
    gradient against W^T; weight gradients from the recomputed intermediates
    or -- split -- from one dy^T a reduction split by C x C products) against
    the fp32 two-layer composition: output and the gradients of a, the
    residual and all four parameters; the merged operands follow an in-place
    parameter update (version bump)."""
    monkeypatch.setattr(H, "_ATTN_SPLIT", 0 if split else 1 << 30)
    monkeypatch.setattr(H, "_ATTN_SMALL", True)
    torch.manual_seed(23)
    a = torch.randn(N, L, C, device=DEV).to(BF)
    x = torch.randn(N, L, C, device=DEV).to(BF)
    Wo = torch.randn(C, C, device=DEV) / math.sqrt(C)
    bo = torch.randn(C, device=DEV) * 0.1
    Wl = torch.randn(C, C, 1, 1, device=DEV) / math.sqrt(C)
    bl = torch.randn(C, device=DEV) * 0.1
    go = torch.randn(N, L, C, device=DEV)
    s = 1 / math.sqrt(2)

    def ref(a, x, Wo, bo, Wl, bl):
        return T.linear(T.linear(a, Wo, bo), Wl, bl, x, s)

    for rep in range(2):
        yh, yr, gh, gr = run_both(lambda a, x, Wo, bo, Wl, bl: H.attn_out(a, Wo, bo, Wl, bl, residual=x, out_scale=s),
                                  ref, [a, x, Wo, bo, Wl, bl], go)
        assert rel(yh, yr) < 2e-2, (rep, rel(yh, yr))
        for i, (u, v) in enumerate(zip(gh, gr)):
            assert rel(u, v) < 3e-2, (rep, i, rel(u, v))
        with torch.no_grad():              # a parameter update: the next forward re-derives W and b
            Wl.mul_(-0.5)
            bo.add_(0.3)


CONV_SHAPES = [
    # N, H, W, Cin, Cout, stride, residual, row_bias, scale
    (4, 16, 16, 128, 128, 1, True, False, 1 / math.sqrt(2)),
    (12, 64, 64, 128, 128, 1, True, False, 1 / math.sqrt(2)),   # >= 384 tiles: no split-K
    (2, 8, 8, 256, 512, 1, False, False, 1.0),
    (2, 8, 8, 512, 256, 1, True, False, 1 / math.sqrt(2)),
    (2, 16, 16, 144, 256, 1, False, True, 1.0),
    (2, 16, 16, 144, 256, 2, False, True, 1.0),
    (2, 16, 16, 144, 128, 4, False, True, 1.0),
    (2, 16, 16, 144, 128, 8, False, True, 1.0),
    (2, 12, 20, 384, 128, 1, False, False, 1.0),
    (2, 16, 16, 3, 128, 1, False, False, 1.0),     # stem
    (2, 16, 16, 128, 3, 1, False, False, 1.0),     # head
]


@pytest.mark.parametrize("N,Hh,W,Ci,Co,s,res,rb,scale", CONV_SHAPES)
def test_conv3x3(H, N, Hh, W, Ci, Co, s, res, rb, scale):
    torch.manual_seed(3)
    x = torch.randn(N, Hh, W, Ci, device=DEV).to(BF)
    w = torch.randn(Co, Ci, 3, 3, device=DEV) / math.sqrt(9 * Ci)
    b = torch.randn(Co, device=DEV) * 0.1
    OH, OW = (Hh - 1) // s + 1, (W - 1) // s + 1
    r = torch.randn(N, OH, OW, Co, device=DEV).to(BF) if res else None
    rbias = torch.randn(N, Co, device=DEV) if rb else None
    go = torch.randn(N, OH, OW, Co, device=DEV)
    ins = [x, w, b] + ([r] if res else []) + ([rbias] if rb else [])

    def mk(fn):
        def f(*a):
            x, w, b = a[:3]
            k = 3
            rr = a[k] if res else None
            k += int(res)
            rbb = a[k] if rb else None
            return fn(x, w, b, s, rr, scale, rbb)
        return f

    yh, yr, gh, gr = run_both(mk(H.conv3x3), mk(T.conv3x3), ins, go)
    assert yh.shape == yr.shape
    assert rel(yh, yr) < 2e-2
    names = ["dx", "dw", "db", "dres", "drow"]
    for i, (a, c) in enumerate(zip(gh, gr)):
        assert a is not None and c is not None
        assert rel(a, c) < 3e-2, (names[i], rel(a, c))


HSM_SHAPES = [
    # the 8x8 / 16x16 levels at 16 examples per GPU: small-image halo conv (conv_hsm_k)
    (32, 8, 8, 512, 512, 1, True, True, 1 / math.sqrt(2)),
    (32, 16, 16, 256, 256, 1, True, False, 1 / math.sqrt(2)),
    (32, 8, 8, 1024, 512, 1, False, True, 1.0),                 # decoder concat input
    (32, 16, 16, 512, 256, 1, False, False, 1.0),
    (32, 16, 16, 96, 128, 1, True, False, 0.5),                 # IC < ICp (padded K), 128 blocks
    (64, 8, 8, 512, 512, 1, True, False, 1.0),                  # bs32 share: 512 blocks
]


@pytest.mark.parametrize("N,Hh,W,Ci,Co,s,res,rb,scale", HSM_SHAPES)
def test_conv3x3_small_halo(H, N, Hh, W, Ci, Co, s, res, rb, scale):
    """conv_hsm_k (fwd and input gradient) against fp32, and every wave-group
    form against the 64 x 64 im2col kernel it replaces (D3D_CONV_HSM=0)."""
    test_conv3x3(H, N, Hh, W, Ci, Co, s, res, rb, scale)
    torch.manual_seed(5)
    x = torch.randn(N, Hh, W, Ci, device=DEV).to(BF)
    w = torch.randn(Co, Ci, 3, 3, device=DEV) / math.sqrt(9 * Ci)
    b = torch.randn(Co, device=DEV) * 0.1
    ys = {}
    with torch.no_grad():
        try:
            for cfg in (0, 1, 2, 3, 4):          # off, auto, 1 / 2 / 3-4 wave groups
                H._lib.d3d_conv_hsm_cfg(cfg)
                ys[cfg] = H.conv3x3(x, w, b)
        finally:
            H._lib.d3d_conv_hsm_cfg(1)
    for cfg in (1, 2, 3, 4):
        assert rel(ys[cfg], ys[0]) < 1e-2, (cfg, rel(ys[cfg], ys[0]))
    assert torch.equal(ys[1], ys[3] if N * (Hh // 8) * (Co // 64) > 320 else ys[4])   # auto form, deterministic


W8_SHAPES = [
    # large grids (>= 256 blocks of 256 pixels): the 8-wave conv_w8_k path
    (32, 64, 64, 128, 128, 1, True, False, 1 / math.sqrt(2)),     # BM=128 (w8w: 128x512 tiles)
    (64, 32, 32, 256, 256, 1, False, True, 1.0),                  # BM=256
    (300, 12, 20, 128, 384, 1, False, False, 1.0),                # partial pixel tile, OC 384 -> 3 x BM=128
    (16, 64, 64, 64, 640, 1, True, False, 0.5),                   # OC 640: BM=256 tile overhangs the weights
    (32, 32, 32, 256, 256, 1, True, False, 1.0),                  # w8n: 256 x 128 tiles (128 of 256x256 < 256 CUs)
    (16, 32, 32, 512, 512, 1, False, True, 0.5),                  # w8n: 2 x 128 tiles of 256 x 128
    (32, 64, 64, 384, 128, 1, True, True, 1 / math.sqrt(2)),      # halo: 8-row tiles, 12 channel chunks
    (8, 128, 128, 128, 256, 1, False, False, 1.0),                # halo: 4-row tiles of 128-wide images
    (64, 32, 32, 128, 256, 1, False, False, 1.0),                 # 32-wide: halo (16-row tiles), else conv_w8_k
    (128, 16, 16, 256, 256, 1, True, False, 1 / math.sqrt(2)),    # 16-wide: halo 1-image tiles when enabled
    (32, 32, 32, 256, 256, 1, False, False, 1.0),                 # 32-wide at bs16: halo 8-row tiles when enabled
]


@pytest.mark.parametrize("impl", ["w8", "w8w", "w8n", "halo"])
@pytest.mark.parametrize("N,Hh,W,Ci,Co,s,res,rb,scale", W8_SHAPES)
def test_conv3x3_w8(H, impl, N, Hh, W, Ci, Co, s, res, rb, scale):
    H.set_conv_impl(impl)
    try:
        test_conv3x3(H, N, Hh, W, Ci, Co, s, res, rb, scale)
    finally:
        H.set_conv_impl("halo")


S64_SHAPES = [
    # small grids that the 128x128 kernels would split over K: the 64x64
    # no-split tiles of conv_small.hip (16-32 examples per GPU, levels 2-3)
    (32, 8, 8, 512, 512, 1, True, False, 1 / math.sqrt(2)),
    (32, 16, 16, 256, 256, 1, False, False, 1.0),
    (32, 8, 8, 1024, 512, 1, True, False, 1 / math.sqrt(2)),
    (32, 16, 16, 768, 256, 1, False, False, 1.0),
    (32, 16, 16, 144, 1024, 2, False, True, 1.0),       # strided conditioning conv
    (20, 8, 8, 256, 512, 1, False, True, 0.5),          # partial pixel tiles (1280 px)
]


@pytest.mark.parametrize("N,Hh,W,Ci,Co,s,res,rb,scale", S64_SHAPES)
def test_conv3x3_small_tiles(H, N, Hh, W, Ci, Co, s, res, rb, scale):
    test_conv3x3(H, N, Hh, W, Ci, Co, s, res, rb, scale)


@pytest.mark.parametrize("cfg", [1, 2, 3, 4])
@pytest.mark.parametrize("N,Hh,W,Ci,Co,s,res,rb,scale", [S64_SHAPES[0], S64_SHAPES[1], S64_SHAPES[4],
                                                         S64_SHAPES[5]])
def test_conv3x3_small_tiles_wave_groups(H, cfg, N, Hh, W, Ci, Co, s, res, rb, scale):
    """Every wave-group split of the small-grid conv (one 4-wave group; 2 / 4
    groups with 2-stage rings; 2 groups with 4-stage rings) against fp32,
    forward and input gradient (the fused GN statistics are covered by
    test_conv_fused_gn_stats at the automatic choice)."""
    H._lib.d3d_conv_s64_cfg(cfg)
    try:
        test_conv3x3(H, N, Hh, W, Ci, Co, s, res, rb, scale)
    finally:
        H._lib.d3d_conv_s64_cfg(0)


WGRAD_W8_SHAPES = [
    # 3x3 stride-1 weight gradients on the 8-wave kernel (impl "w8")
    (8, 32, 32, 256, 256, 1, False, False, 1.0),                  # 256 x 256 tiles
    (3, 16, 16, 128, 256, 1, True, False, 1.0),                   # 256 x 128, partial last split
    (4, 16, 16, 384, 128, 1, False, False, 1.0),                  # 128 x 256, IC tile overhang
    (2, 8, 8, 512, 512, 1, True, False, 1 / math.sqrt(2)),
]


@pytest.mark.parametrize("N,Hh,W,Ci,Co,s,res,rb,scale", WGRAD_W8_SHAPES)
def test_conv3x3_wgrad_w8(H, N, Hh, W, Ci, Co, s, res, rb, scale):
    H.set_wgrad_impl("w8")
    try:
        test_conv3x3(H, N, Hh, W, Ci, Co, s, res, rb, scale)
    finally:
        H.set_wgrad_impl("w8")


@pytest.mark.parametrize("cfg", [8, 4, 2])
@pytest.mark.parametrize("M,N,K,lda,ldb,ldo,bias,res,alpha,scale", [
    (256, 256, 128, 128, 128, 256, False, False, 1.0, 1.0),
    (768, 8192, 256, 256, 256, 768, True, False, 1.0, 1.0),
    (200, 1000, 192, 200, 256, 208, True, True, 0.5, 0.7),        # M / N tails, padded rows
    (1024, 4096, 4608, 4608, 4608, 1024, False, False, 1.0, 1.0),  # long reduction
    (128, 70000, 256, 256, 256, 128, True, True, 1.0, 0.25),       # M < tile, many tiles per block
    (4608, 2048, 1024, 1024, 1024, 4608, True, False, 1.0, 1.0),
])
def test_gemm_nt(H, cfg, M, N, K, lda, ldb, ldo, bias, res, alpha, scale):
    """gfx950 GEMM (every tile configuration) against the fp32 product: bias /
    residual / alpha / scale epilogue, tails in M and N, row strides wider
    than K, output rows wider than M left untouched."""
    H._lib.d3d_gemm_tune(cfg, 0, 0)
    try:
        torch.manual_seed(11)
        a = torch.randn(M, lda, device=DEV).to(BF)
        b = torch.randn(N, ldb, device=DEV).to(BF)
        bb = torch.randn(M, device=DEV) if bias else None
        r = torch.randn(N, ldo, device=DEV).to(BF) if res else None
        out = torch.full((N, ldo), 7.0, device=DEV).to(BF)
        H.gemm_nt(a, b, out, M, N, K, lda, ldb, ldo, bias=bb, res=r, alpha=alpha, scale=scale)
        ref = a[:, :K].float() @ b[:, :K].float().t() * alpha
        ref = ref.t()
        if bias:
            ref = ref + bb
        if res:
            ref = ref + r[:, :M].float()
        ref = ref * scale
        assert rel(out[:, :M], ref) < 1e-2
        if ldo > M:
            assert (out[:, M:] == 7.0).all()          # columns past M untouched
    finally:
        H._lib.d3d_gemm_tune(1, 0, 0)


@pytest.mark.parametrize("cfg", [8, 4, 2])
@pytest.mark.parametrize("grid", [0, 7])
@pytest.mark.parametrize("K", [128, 192, 512, 1536])
def test_gemm_deep_ring(H, cfg, grid, K):
    """4-stage LDS ring of the small-problem GEMM (gemm.hip NST): equals the
    2-stage ring bit for bit and the fp32 product -- one tile per block, and a
    forced 7-block grid where each block walks many tiles with the loader up to
    two tiles ahead (bias slots, K = 128: two stages per tile).  cfg 8 (2-stage
    only) pins the K = 128 multi-tile bias: the prologue crossed into a block's
    second tile without loading its bias (the bs128 128->256 skip projection)."""
    torch.manual_seed(17)
    M, N = 200, 1000
    a = torch.randn(M, K, device=DEV).to(BF)
    b = torch.randn(N, K, device=DEV).to(BF)
    bb = torch.randn(M, device=DEV)
    r = torch.randn(N, M, device=DEV).to(BF)
    outs = []
    try:
        for deep in (-1, -2):      # 4-, 2-stage rings
            H._lib.d3d_gemm_tune(deep, 0, 0)
            H._lib.d3d_gemm_tune(cfg, 0, grid if grid else 0)
            out = torch.empty(N, M, device=DEV, dtype=BF)
            H.gemm_nt(a, b, out, M, N, K, K, K, M, bias=bb, res=r, alpha=0.5, scale=0.75)
            outs.append(out)
    finally:
        H._lib.d3d_gemm_tune(-1, 0, 0)
        H._lib.d3d_gemm_tune(1, 0, 0)
        H._lib.d3d_gemm_tune(0, 0, -1)
    ref = ((b.float() @ a.float().t()) * 0.5 + bb + r.float()) * 0.75
    assert rel(outs[0], ref) < 1e-2
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("cfg", [8, 4, 2])
def test_gemm_bf16_bias_and_dsilu_epilogue(H, cfg):
    """bf16 bias, the in-place residual (out == res) of the virtual-concat
    skip, and the dsilu epilogue (FiLM input gradient) against fp32."""
    H._lib.d3d_gemm_tune(cfg, 0, 0)
    try:
        torch.manual_seed(3)
        M, N, K = 1024, 3000, 2048
        a = torch.randn(M, K, device=DEV).to(BF)
        b = torch.randn(N, K, device=DEV).to(BF)
        bb = torch.randn(M, device=DEV).to(BF)
        out = torch.empty(N, M, device=DEV, dtype=BF)
        H.gemm_nt(a, b, out, M, N, K, K, K, M, bias=bb)
        ref = (b.float() @ a.float().t()) + bb.float()
        assert rel(out, ref) < 1e-2
        keep = out.clone()
        H.gemm_nt(a, b, out, M, N, K, K, K, M, res=out)            # accumulate in place
        assert rel(out, keep.float() + b.float() @ a.float().t()) < 1e-2
        e = torch.randn(N, M, device=DEV).to(BF) * 3
        H.gemm_nt(a, b, out, M, N, K, K, K, M, dsilu_of=e, ldr=M, alpha=0.5)
        s = torch.sigmoid(e.float())
        ref = 0.5 * (b.float() @ a.float().t()) * s * (1 + e.float() * (1 - s))
        assert rel(out, ref) < 1e-2
    finally:
        H._lib.d3d_gemm_tune(1, 0, 0)


@pytest.mark.parametrize("N,L,C", [(4, 256, 256), (8, 64, 512), (32, 64, 512)])
def test_gemm_gn_partials(H, N, L, C):
    """GroupNorm partial statistics from the GEMM epilogue (every tile config
    that carries them) equal the statistics pass over the written output."""
    torch.manual_seed(5)
    for cfg in (8, 4):
        H._lib.d3d_gemm_tune(cfg, 0, 0)
        try:
            P = N * L
            a = torch.randn(C, C, device=DEV).to(BF)
            b = torch.randn(P, C, device=DEV).to(BF)
            out = torch.empty(P, C, device=DEV, dtype=BF)
            gnp = torch.empty(N * 32 * (L // 64) * 2, device=DEV)
            H.gemm_nt(a, b, out, C, P, C, C, C, C, gnp=gnp, gn_groups=32, gn_hw=L)
            y = out.float().view(N, L // 64, 64, 32, C // 32)
            s = y.sum((2, 4)).permute(0, 2, 1)
            q = (y * y).sum((2, 4)).permute(0, 2, 1)
            got = gnp.view(N, 32, L // 64, 2)
            assert rel(got[..., 0], s) < 1e-4 and rel(got[..., 1], q) < 1e-4
        finally:
            H._lib.d3d_gemm_tune(1, 0, 0)


@pytest.mark.parametrize("P,IC,OC", [(128, 256, 768), (8192, 256, 768), (2048, 512, 512), (2048, 512, 1536),
                                     (4096, 384, 128), (32768, 1024, 512)])
def test_linear(H, P, IC, OC):
    """Per-pixel dense layer (GEMM with the fused bias / residual / scale
    epilogue, input gradient on the same kernel, split-K weight gradient)
    against the torch composition."""
    torch.manual_seed(4)
    x = torch.randn(2, P // 2, IC, device=DEV).to(BF)
    w = torch.randn(OC, IC, device=DEV) / math.sqrt(IC)
    b = torch.randn(OC, device=DEV) * 0.1
    r = torch.randn(2, P // 2, OC, device=DEV).to(BF)
    go = torch.randn(2, P // 2, OC, device=DEV)
    nfb = len(H.FALLBACKS)
    yh, yr, gh, gr = run_both(lambda x, w, b, r: H.linear(x, w, b, r, 0.7),
                              lambda x, w, b, r: T.linear(x, w, b, r, 0.7), [x, w, b, r], go)
    assert len(H.FALLBACKS) == nfb, H.FALLBACKS          # the native GEMM ran
    assert rel(yh, yr) < 2e-2
    for a, c in zip(gh, gr):
        assert rel(a, c) < 3e-2


@pytest.mark.parametrize("N,L,C,cross", [(4, 256, 256, False), (4, 256, 256, True), (4, 64, 512, False),
                                         (4, 64, 512, True), (2, 1024, 256, True),
                                         # ragged sequences (masked last block): the 4x4 level of the 32x32
                                         # chairs config, 7x7 / 14x14 levels of 56x56 images, 10x10
                                         (4, 16, 512, True), (4, 49, 512, False), (2, 196, 256, True),
                                         (2, 100, 256, False)])
def test_attention(H, N, L, C, cross):
    torch.manual_seed(5)
    qkv = torch.randn(N, L, 3 * C, device=DEV).to(BF)
    go = torch.randn(N, L, C, device=DEV)
    yh, yr, gh, gr = run_both(lambda q: H.attention(q, 4, cross), lambda q: T.attention(q, 4, cross), [qkv], go)
    assert rel(yh, yr) < 2e-2
    assert rel(gh[0], gr[0]) < 4e-2


@pytest.mark.parametrize("N,L,cross", [(4, 256, False), (4, 256, True), (2, 196, True), (2, 100, False),
                                         (128, 256, True)])
def test_attention_backward_one_workgroup_per_head(H, N, L, cross):
    """Head dim 64, 64 < L <= 256: one 8-wave workgroup owns all keys of an
    (image, head) and writes dQ directly (no fp32 slabs / conversion launch;
    the default; d3d_attn_bwd_cfg(1 << 30) restores the 64-key path).
    Gradients against fp32 and against the 64-key-workgroup + slab path."""
    torch.manual_seed(8)
    C = 256
    qkv = torch.randn(N, L, 3 * C, device=DEV).to(BF)
    go = torch.randn(N, L, C, device=DEV)
    H._ensure_impl()
    outs = []
    try:
        for wide_min in (0, 1 << 30):
            H._lib.d3d_attn_bwd_cfg(wide_min)
            assert (H._lib.d3d_attn_bwd_slabs(N, L, C, 4) == 0) == (wide_min == 0)
            yh, yr, gh, gr = run_both(lambda q: H.attention(q, 4, cross), lambda q: T.attention(q, 4, cross), [qkv],
                                      go)
            assert rel(yh, yr) < 2e-2
            assert rel(gh[0], gr[0]) < 4e-2, (wide_min, rel(gh[0], gr[0]))
            outs.append(gh[0].float())
    finally:
        H._lib.d3d_attn_bwd_cfg(0)
    assert rel(outs[0], outs[1]) < 1e-2


@pytest.mark.parametrize("N,L,cross", [(4, 256, False), (4, 256, True), (2, 196, True), (2, 100, False),
                                         (2, 65, True)])
def test_attention_forward_one_workgroup_per_head(H, N, L, cross):
    """Head dim 64, 64 < L <= 256: one 16-wave workgroup per (image, head)
    stages all K / V in LDS once (the default from 512 (image, head) pairs;
    d3d_attn_fwd_cfg(0) forces it, d3d_attn_fwd_cfg(1 << 30) the 64-query
    workgroups).  Output and saved log-sum-exp against fp32 and
    against the 64-query path."""
    torch.manual_seed(9)
    C = 256
    qkv = torch.randn(N, L, 3 * C, device=DEV).to(BF)
    H._ensure_impl()
    outs = []
    try:
        for all_ in (0, 1 << 30):
            H._lib.d3d_attn_fwd_cfg(all_)
            yh = H.attention(qkv, 4, cross)
            yr = T.attention(qkv.float(), 4, cross)
            assert rel(yh, yr) < 2e-2, (all_, rel(yh, yr))
            out = torch.empty(N, L, C, device=DEV, dtype=BF)
            lse = torch.empty(N, 4, L, device=DEV)
            assert H._lib.d3d_attn_fwd(qkv.data_ptr(), out.data_ptr(), lse.data_ptr(), N, L, C, 4, int(cross),
                                       64 ** -0.5, H._st()) == 0
            q, k = qkv[..., :C].float(), qkv[..., C:2 * C].float()
            if cross:
                k = k.view(N // 2, 2, L, C).flip(1).reshape(N, L, C)
            s = torch.einsum("nqhd,nkhd->nhqk", q.view(N, L, 4, 64), k.view(N, L, 4, 64)) * 64 ** -0.5
            assert rel(lse, torch.logsumexp(s, -1)) < 1e-3
            outs.append((out.float(), lse))
    finally:
        H._lib.d3d_attn_fwd_cfg(512)
    assert rel(outs[0][0], outs[1][0]) < 1e-2
    assert rel(outs[0][1], outs[1][1]) < 1e-4


@pytest.mark.parametrize("N,C,OC", [(32, 128, 256), (32, 256, 256)])
def test_gn_silu_conv_fused(H, N, C, OC, monkeypatch):
    """ResnetBlock GN0 + SiLU folded into conv1's halo staging (conv_halo_k
    GNA, 32x32 images on 256-pixel tiles): output, the output's GroupNorm
    partials and every gradient against the separate GroupNorm + conv ops
    and against fp32; h is never written in the forward, and the weight
    gradient runs on h rematerialised from x."""
    torch.manual_seed(11)
    Hh = 32
    x = (torch.randn(N, Hh, Hh, C, device=DEV) * 1.5 + 0.3).to(BF)
    gw = torch.rand(C, device=DEV) + 0.5
    gb = torch.randn(C, device=DEV) * 0.2
    cw = torch.randn(OC, C, 3, 3, device=DEV) / (3 * C ** 0.5)
    cb = torch.randn(OC, device=DEV) * 0.1
    go = torch.randn(N, Hh, Hh, OC, device=DEV)
    monkeypatch.setattr(H, "_GN_CONV", True)          # (off by default: measured slower)
    assert H.gn_silu_conv_ok(x, OC, 32)
    # 512-pixel tiles (64 images) keep the separate GroupNorm pass
    assert not H.gn_silu_conv_ok(torch.cat([x, x]), OC, 32)

    def run(mode):
        xs = leaf(x) if mode != "ref" else leaf(x, torch.float32)
        ps = [leaf(t) for t in (gw, gb, cw, cb)]
        if mode == "fused":
            y = H.gn_silu_conv3x3(xs, *ps, 32, 1e-5, gn1_groups=32)
        elif mode == "sep":
            h = H.group_norm(xs, ps[0], ps[1], 32, 1e-5, silu=True)
            y = H.conv3x3(h, ps[2], ps[3], gn_groups=32)
        else:
            h = T.group_norm(xs, ps[0], ps[1], 32, 1e-5, silu=True)
            y = T.conv3x3(h, ps[2], ps[3])
        (y.float() * go).sum().backward()
        return y, [xs.grad] + [p_.grad for p_ in ps]

    yf, gf = run("fused")
    ys, gs = run("sep")
    yr, gr = run("ref")
    assert rel(yf, ys) < 1e-3, rel(yf, ys)
    assert rel(yf, yr) < 2e-2
    pf, ps_ = getattr(yf, "_d3d_gnpart", None), getattr(ys, "_d3d_gnpart", None)
    assert pf is not None and ps_ is not None and pf[1:] == ps_[1:]
    assert rel(pf[0], ps_[0]) < 1e-3
    for a, b, c in zip(gf, gs, gr):
        assert rel(a, b) < 1e-2, rel(a, b)
        assert rel(a, c) < 4e-2, rel(a, c)


def test_attention_spiky(H):
    """A key that dominates one query's softmax in a late key block forces the
    online-softmax rescale branch."""
    torch.manual_seed(6)
    N, L, C = 2, 256, 256
    qkv = torch.randn(N, L, 3 * C, device=DEV) * 0.3
    qkv[:, 7, :C] = 2.0           # query 7
    qkv[:, 200, C:2 * C] = 2.0    # key 200 (block 3)
    qkv = qkv.to(BF)
    yh = H.attention(qkv, 4, False)
    yr = T.attention(qkv.float(), 4, False)
    assert rel(yh, yr) < 2e-2


def test_pool_upsample_silu(H):
    torch.manual_seed(7)
    x = torch.randn(2, 16, 16, 128, device=DEV).to(BF)
    for fh, fr, oshape in [(H.avgpool2, T.avgpool2, (2, 8, 8, 128)), (H.upsample2, T.upsample2, (2, 32, 32, 128)),
                           (H.silu, T.silu, (2, 16, 16, 128))]:
        go = torch.randn(*oshape, device=DEV)
        yh, yr, gh, gr = run_both(fh, fr, [x], go)
        assert rel(yh, yr) < 1e-2
        assert rel(gh[0], gr[0]) < 1e-2


def test_ray_posenc(H):
    from distributed_3d_diffusion_pytorch_amd.data.synthetic import random_orbit_poses
    g = torch.Generator(device=DEV)
    g.manual_seed(0)
    B, Hh, W = 3, 16, 16
    R, t = random_orbit_poses(2 * B, g, DEV)
    R, t = R.reshape(B, 2, 3, 3), t.reshape(B, 2, 3)
    K = torch.tensor([[131.25, 0, 64.0], [0, 131.25, 64.0], [0, 0, 1]], dtype=torch.float64, device=DEV)
    K = K.expand(B, 3, 3)
    mask = torch.tensor([True, False, True], device=DEV)
    pe = torch.randn(144, Hh, W, device=DEV) * 0.1
    fe = torch.randn(1, 1, 144, 1, 1, device=DEV) * 0.1
    oe = torch.randn(1, 1, 144, 1, 1, device=DEV) * 0.1
    yh = H.ray_posenc(R, t, K, Hh, W, mask, pe, fe, oe)
    yr = T.ray_posenc(R, t, K, Hh, W, mask, pe, fe, oe)
    assert (yh.float() - yr).abs().max().item() < 2e-2
    # gradients of the learned embeddings
    pe_, fe_, oe_ = leaf(pe), leaf(fe), leaf(oe)
    pr_, fr_, or_ = leaf(pe), leaf(fe), leaf(oe)
    go = torch.randn(2 * B, Hh, W, 144, device=DEV)
    H.ray_posenc(R, t, K, Hh, W, mask, pe_, fe_, oe_).backward(go.to(BF))
    T.ray_posenc(R, t, K, Hh, W, mask, pr_, fr_, or_).backward(go)
    assert rel(pe_.grad, pr_.grad) < 1e-2
    assert rel(fe_.grad, fr_.grad) < 1e-2
    assert rel(oe_.grad, or_.grad) < 1e-2


def test_adam_matches_torch(H):
    from distributed_3d_diffusion_pytorch_amd.parallel.flat import FlatParams
    from distributed_3d_diffusion_pytorch_amd.engine.optim import FusedAdam
    torch.manual_seed(8)
    ps = [torch.nn.Parameter(torch.randn(s, device=DEV)) for s in [(33, 7), (128,), (5, 5, 3)]]
    ref = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    flat = FlatParams(ps)
    opt = FusedAdam(flat, lr=1e-2, betas=(0.9, 0.99))
    topt = torch.optim.Adam(ref, lr=1e-2, betas=(0.9, 0.99))
    for step in range(5):
        grads = [torch.randn_like(p) for p in ps]
        for p, g in zip(ps, grads):
            p.grad.copy_(g)
        for p, g in zip(ref, grads):
            p.grad = g.clone()
        opt.step()
        topt.step()
    for p, r in zip(ps, ref):
        assert torch.allclose(p, r, atol=1e-6, rtol=1e-5)


def test_model_hip_vs_torch_backend():
    """Whole X-UNet forward+backward: HIP backend vs torch backend (bf16)."""
    from distributed_3d_diffusion_pytorch_amd import ops
    from distributed_3d_diffusion_pytorch_amd.models import XUNet
    from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches
    torch.manual_seed(9)
    m = XUNet(H=32, W=32, ch=128).to(DEV)
    with torch.no_grad():
        for p in m.parameters():
            if p.abs().sum() == 0:
                p.normal_(0, 0.02)
    m.compute_dtype = BF
    m.eval()
    img, R, t, K = next(SyntheticBatches(2, 32, DEV, seed=0))
    batch = {"x": img[:, 0], "z": img[:, 1], "logsnr": torch.tensor([[20.0, 1.5], [20.0, -3.0]], device=DEV),
             "R": R, "t": t, "K": K}
    mask = torch.tensor([True, False], device=DEV)
    outs, grads = [], []
    for be in ("hip", "torch"):
        ops.set_backend(be)
        m.zero_grad(set_to_none=True)
        y = m(batch, cond_mask=mask)
        y.float().square().mean().backward()
        outs.append(y.float())
        grads.append(torch.cat([p.grad.flatten() for p in m.parameters()]))
    ops.set_backend(None)
    assert rel(outs[0], outs[1]) < 5e-2
    cos = torch.nn.functional.cosine_similarity(grads[0], grads[1], dim=0).item()
    assert cos > 0.98, cos


def test_grad_sink_and_reducer_two_ranks_one_gpu(tmp_path):
    import sys, os
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import dist_workers as W
    from distributed_3d_diffusion_pytorch_amd.parallel import spawn
    spawn(W.gpu_sink_reducer, 2, (str(tmp_path),))
    for r in range(2):
        cos, rel = map(float, open(tmp_path / f"g{r}.txt").read().split())
        assert cos > 0.9999 and rel < 1e-2, (r, cos, rel)


def test_graph_step_two_ranks_one_gpu(tmp_path):
    """world=2 HIP-graph step (flat all-reduce between the graphs) == eager
    step (bucketed hooks); replicas identical after every step."""
    import sys, os
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import dist_workers as W
    from distributed_3d_diffusion_pytorch_amd.parallel import spawn
    spawn(W.gpu_graph_vs_eager, 2, (str(tmp_path),))
    for r in range(2):
        d, de, dg, dl = map(float, open(tmp_path / f"gr{r}.txt").read().split())
        assert de == 0.0 and dg == 0.0, (r, de, dg)
        assert d < 5e-4 and dl < 2e-3, (r, d, dl)


def test_sampler_step_matches_posterior(H):
    from distributed_3d_diffusion_pytorch_amd.diffusion import cfg_posterior
    torch.manual_seed(11)
    z = torch.randn(4, 3, 16, 16, device=DEV)
    ec, eu = torch.randn_like(z), torch.randn_like(z)
    w = torch.tensor([0.0, 1.0, 3.0, 7.0], device=DEV)
    lam, lamn = 0.7, 1.9
    c = -math.expm1(lam - lamn)
    sig = lambda x: 1 / (1 + math.exp(-x))  # noqa: E731
    out = H.sampler_step(z, ec, eu, w, math.sqrt(sig(lam)), math.sqrt(sig(-lam)), math.sqrt(sig(lamn)), c,
                         math.sqrt(sig(-lamn) * c), False, 0)
    mean, var = cfg_posterior(z, ec, eu, w, torch.tensor(lam), torch.tensor(lamn))
    assert torch.allclose(out, mean, atol=1e-5, rtol=1e-5)
    noisy = H.sampler_step(z, ec, eu, w, math.sqrt(sig(lam)), math.sqrt(sig(-lam)), math.sqrt(sig(lamn)), c,
                           math.sqrt(sig(-lamn) * c), True, 123)
    nz = (noisy - mean) / var.sqrt()
    assert abs(nz.mean().item()) < 0.05 and abs(nz.std().item() - 1) < 0.05


@pytest.mark.parametrize("mode", ["tn", "blas", "seg"])
@pytest.mark.parametrize("chans,N,Hh", [([128, 128, 256], 4, 8), ([512, 512], 4, 8),
                                        ([128, 256, 384], 32, 32),    # 32768 rows: 8-wave 1x1 wgrad
                                        ([256, 512], 8, 32)])         # 8192 rows: 4 blas slabs
def test_film_batch_with_gn_film(H, chans, N, Hh, mode):
    """Level-batched FiLM projection ``dense_i(silu(emb))`` feeding strided
    GN-FiLM: forward, the shared d(scale|shift) buffer, the input gradient
    through the SiLU (GEMM epilogue) and the segmented weight-gradient scatter
    against per-block fp32 linears."""
    torch.manual_seed(0)
    K = 1024
    semb = (torch.randn(N, Hh, Hh, K, device=DEV) * 2).to(BF)
    Ws = [torch.randn(2 * c, K, device=DEV) / 32 for c in chans]
    Bs = [torch.randn(2 * c, device=DEV) * 0.1 for c in chans]
    xs = [torch.randn(N, Hh, Hh, c, device=DEV).to(BF) for c in chans]
    gam = [torch.rand(c, device=DEV) + 0.5 for c in chans]
    bet = [torch.randn(c, device=DEV) * 0.1 for c in chans]
    gos = [torch.randn(N, Hh, Hh, c, device=DEV) for c in chans]

    def run(hip):
        s = leaf(semb) if hip else leaf(semb, torch.float32)
        ws = [leaf(w) for w in Ws]
        bs = [leaf(b) for b in Bs]
        if hip:
            sss = H.film_batch(s, ws, bs)
        else:
            sss = [T.linear(torch.nn.functional.silu(s), w, b) for w, b in zip(ws, bs)]
        loss = 0
        for x, g, b, ss, go in zip(xs, gam, bet, sss, gos):
            xx = x if hip else x.float()
            y = (H if hip else T).gn_film(xx, g, b, ss, 32, 1e-5, 0.0, False, 0)
            loss = loss + (y.float() * go).sum()
        loss.backward()
        return [s.grad] + [w.grad for w in ws] + [b.grad for b in bs]

    prev = H._FILM_WGRAD
    H._FILM_WGRAD = mode       # transposed-read TN GEMM, hipBLASLt product + scatter, or the 1x1 conv wgrad
    try:
        gh, gr = run(True), run(False)
    finally:
        H._FILM_WGRAD = prev
    for a, b in zip(gh, gr):
        assert rel(a, b) < 3e-2, rel(a, b)


def test_film_early_weight_gradients(H, monkeypatch):
    """Training step with sink-managed parameters: each level's FiLM weight
    gradients run as two jobs -- the decoder blocks' submitted by the GN-FiLM
    backward that completes them (overlapping the rest of the backward), the
    encoder blocks' after -- instead of one level-wide job after the level's
    last block; the flat gradient matches the level-wide path."""
    from distributed_3d_diffusion_pytorch_amd.config import make_config
    from distributed_3d_diffusion_pytorch_amd.engine import Trainer
    from distributed_3d_diffusion_pytorch_amd.parallel import DistContext
    from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches
    ctx = DistContext(device=torch.device("cuda", 0))
    batch = next(SyntheticBatches(8, 64, "cuda", seed=5))
    calls = []
    orig = H._film_group_wgrad

    def counting(*a):
        r = orig(*a)
        calls.append(r)
        return r

    monkeypatch.setattr(H, "_film_group_wgrad", counting)
    grads, nblocks = [], 0
    for early in (True, False):
        monkeypatch.setattr(H, "_FILM_EARLY", 2 if early else 0)
        torch.manual_seed(0)
        cfg = make_config(None, {"model.H": 64, "model.W": 64, "data.imgsize": 64, "global_batch": 8,
                                 "micro_batch": 0, "data.synthetic": True, "log_every": 0, "ckpt_every": 0,
                                 "graph": False, "optim.warmup_examples": 0})
        tr = Trainer(cfg, ctx)
        tr.optim.zero_in_step = False          # keep the step's gradient for the comparison
        tr.train_step(*batch)
        torch.cuda.synchronize()
        grads.append(tr.flat.grad.clone())
        if early:
            nblocks = 2 * len(tr.model._film_groups())        # two jobs per level
            assert len(calls) == nblocks and all(calls), (len(calls), nblocks)
        del tr
    assert len(calls) == nblocks                # the level-wide run submitted no per-block job
    assert torch.isfinite(grads[0]).all()
    assert rel(grads[0], grads[1]) < 1e-4, rel(grads[0], grads[1])


@pytest.mark.parametrize("P,M,N,ldy,splits", [(16384, 2048, 1024, 2048, 0), (8192, 4608, 1024, 4608, 0),
                                               (256, 200, 136, 200, 1), (1024, 264, 520, 384, 2),
                                               (4096, 512, 256, 512, 3), (128, 256, 256, 256, 1)])
def test_wgrad_tn_matches_fp32(H, P, M, N, ldy, splits):
    """Transposed-read split-K weight-gradient GEMM (wgrad_gemm.hip): the
    slabs sum to dy^T x and the bias partials to the column sums of dy, for
    full 256 x 256 tiles, ragged M / N (past-the-end columns), a column
    slice of a wider dy (ldy > M) and uneven splits."""
    torch.manual_seed(3)
    dyw = torch.randn(P, ldy, device=DEV).to(BF)
    dy = dyw[:, :M]
    x = torch.randn(P, N, device=DEV).to(BF)
    ws, bws, used = H.wgrad_tn(dy, x, splits)
    assert used >= 1 and ws.shape == (used, M, N)
    ref = dy.float().t() @ x.float()
    got = ws.sum(0)
    assert rel(got, ref) < 1e-4, rel(got, ref)
    rb = dy.float().sum(0)
    assert (bws.sum(0) - rb).abs().max().item() <= 1e-3 * rb.abs().max().item() + 1e-3


# grouped weight-gradient jobs: (N, H, W, IC, OC, taps, C1 of a virtual concat or 0, bias)
WG_JOBS = [
    (32, 64, 64, 128, 128, 9, 0, True),      # 64x64 level at 16 examples / GPU: split-K
    (32, 8, 8, 512, 512, 9, 0, True),        # 8x8 level: unsplit, direct OIHW epilogue
    (128, 16, 16, 384, 256, 9, 0, False),    # halo tile at W = 16 (>= 32768 pixels): two image rows per 32-pixel step
    (2, 8, 8, 128, 128, 9, 0, True),         # W = 8: per-tap tile, unsplit
    (6, 8, 16, 72, 200, 9, 0, True),         # channel tails (partial tiles), non-square image
    (2048, 1, 1, 512, 1536, 1, 0, True),     # 1x1 projection
    (8192, 1, 1, 768, 256, 1, 256, True),    # 1x1 over the virtual concat [x | x2]
    (32, 32, 32, 256, 256, 9, 0, True),
    (4, 16, 64, 192, 128, 9, 128, False),    # halo tiles over the virtual concat, non-square, 3 channel tiles
    (1, 32, 32, 64, 256, 9, 0, True),        # halo tile, small: unsplit OIHW epilogue
    (1, 128, 128, 128, 128, 9, 0, True),     # 128-wide image: four 32-pixel steps per row
]


def _wg_ref(g, x, taps):
    N, Hh, W, OC = g.shape
    IC = x.shape[-1]
    if taps == 1:
        return (g.reshape(-1, OC).float().t() @ x.reshape(-1, IC).float()).reshape(OC, IC, 1)
    dw = torch.nn.grad.conv2d_weight(x.permute(0, 3, 1, 2).float(), (OC, IC, 3, 3), g.permute(0, 3, 1, 2).float(),
                                     padding=1)
    return dw.reshape(OC, IC, 9)


@pytest.mark.parametrize("pk,blocks,minpix,halo,ns", [
    (32, 512, 512, 1, 2), (32, 512, 512, 0, 2), (64, 512, 512, 1, 2), (32, 4096, 64, 1, 2),
    (32, 4096, 64, 0, 2), (64, 512, 512, 0, 2), (32, 512, 512, 1, 3), (32, 64, 512, 1, 2),
    (32, 512, 512, 3, 2), (32, 4096, 64, 3, 2), (32, 256, 512, 4, 2)])
def test_wgrad_group_matches_fp32(H, pk, blocks, minpix, halo, ns):
    """Grouped weight gradients (wgrad_group.hip): the per-tap 128 x 128 tile
    launch and the all-taps halo tile launch (3x3 jobs on W % 32 == 0 images)
    over a mixed batch of 3x3 / 1x1 / virtual-concat jobs (+ the grouped slab
    reduce for the split ones) == the fp32 torch weight gradients, accumulated
    onto the existing gradient with the scale, bias sums included; bitwise
    equal on a re-run.  blocks=4096 plans many more splits (small blocks),
    blocks=64 leaves the big halo jobs nearly unsplit."""
    torch.manual_seed(5)
    H._lib.d3d_wgrad_group_cfg(blocks, pk, minpix)
    # halo 3: the 64-pixel K-step halo kernel for the W >= 64 jobs (the rest as halo 1);
    # halo 4: halo 1 with the big-flush block target forced (2^10 work threshold, 64 blocks)
    H._lib.d3d_wgrad_group_halo(1 if halo in (3, 4) else halo, blocks, ns)
    if halo == 4:
        H._lib.d3d_wgrad_group_halo_big(64, 10)
    H._lib.d3d_wgrad_group_halo_pk(64 if halo == 3 else 32)       # (restored to the default 64 below)
    try:
        jobs, refs, outs = [], [], []
        for (N, Hh, W, IC, OC, taps, C1, bias) in WG_JOBS:
            g = torch.randn(N, Hh, W, OC, device=DEV).to(BF)
            x = torch.randn(N, Hh, W, IC, device=DEV).to(BF)
            dw0 = torch.randn(OC, IC, taps, device=DEV)
            db0 = torch.randn(OC, device=DEV) if bias else None
            ref_w = dw0 + 0.7 * _wg_ref(g, x, taps)
            ref_b = db0 + 0.7 * g.reshape(-1, OC).float().sum(0) if bias else None
            dw, db = dw0.clone(), db0.clone() if bias else None
            if C1:
                xa, xb = x[..., :C1].contiguous(), x[..., C1:].contiguous()
                j = H.wgrad_job(g, xa, OC, IC, N, Hh, W, taps, dw, db, 0.7, x2=xb, C1=C1)
                keep = (g, xa, xb)
            else:
                j = H.wgrad_job(g, x, OC, IC, N, Hh, W, taps, dw, db, 0.7)
                keep = (g, x)
            assert j is not None, (N, Hh, W, IC, OC, taps)
            jobs.append(j)
            refs.append((ref_w, ref_b, dw0, db0))
            outs.append((dw, db, keep))
        sp = (ctypes.c_int * len(jobs))()
        pp = (ctypes.c_int * len(jobs))()
        H._lib.d3d_wgrad_group_plan((H._WgJob * len(jobs))(*jobs), len(jobs), sp, pp, None)
        eng = [H._lib.d3d_wgrad_group_engine(ctypes.byref(j)) for j in jobs]
        want = [int(bool(halo) and t == 9 and Hh >= 32 // min(W, 32) and OC % 128 == 0 and IC % 64 == 0
                    and (W >= 32 or (W == 16 and N * Hh * W >= 32768)))
                for (N, Hh, W, IC, OC, t, C1, b) in WG_JOBS]
        assert eng == want, (eng, want)
        H.wgrad_group_run(jobs)
        torch.cuda.synchronize()
        first = []
        for (ref_w, ref_b, _, _), (dw, db, _), s in zip(refs, outs, sp):
            assert rel(dw, ref_w) < 1e-4, (s, rel(dw, ref_w))
            if ref_b is not None:
                assert rel(db, ref_b) < 1e-4, (s, rel(db, ref_b))
            first.append((dw.clone(), db.clone() if db is not None else None))
        assert max(sp) > 1, list(sp)                          # split-K slabs + grouped reduce exercised
        if blocks <= 1024:
            assert min(sp) == 1, list(sp)                     # ... and the direct OIHW epilogue
        if halo:
            hs = [s_ for s_, e in zip(sp, eng) if e]
            # (halo 3 plans the W >= 64 jobs in a launch of their own: the small job may split)
            assert (blocks > 1024 or halo == 3 or min(hs) == 1) and (blocks < 512 or max(hs) > 1), hs
        for (_, _, dw0, db0), (dw, db, _) in zip(refs, outs):  # re-run: bitwise
            dw.copy_(dw0)
            if db is not None:
                db.copy_(db0)
        H.wgrad_group_run(jobs)
        torch.cuda.synchronize()
        for (dw, db, _), (w1, b1) in zip(outs, first):
            assert torch.equal(dw, w1)
            if db is not None:
                assert torch.equal(db, b1)
    finally:
        H._lib.d3d_wgrad_group_cfg(512, 32, 512)
        H._lib.d3d_wgrad_group_halo(1, 256, 2)             # (the library defaults)
        H._lib.d3d_wgrad_group_halo_big(128, 21)
        H._lib.d3d_wgrad_group_halo_pk(64)


@pytest.mark.parametrize("micro", [2, 0])
def test_graph_train_step_matches_eager(micro):
    """HIP-graph replayed training step == eager step (dropout ON: the graph
    adds the same per-step device words the eager step uses as host seeds;
    counter-based input draw): losses and parameters after 3 steps.  With one
    micro-batch (micro=0) the graph step defers each update into the next
    replay, overlapped with its forward (engine/graphs.py): Trainer.sync()
    applies the last one before the comparison."""
    from distributed_3d_diffusion_pytorch_amd.config import make_config
    from distributed_3d_diffusion_pytorch_amd.engine import Trainer
    from distributed_3d_diffusion_pytorch_amd.parallel import DistContext
    from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches
    ctx = DistContext(device=torch.device("cuda", 0))

    def make(graph):
        cfg = make_config(None, {"model.H": 32, "model.W": 32, "model.dropout": 0.1, "data.imgsize": 32,
                                 "global_batch": 4, "micro_batch": micro, "data.synthetic": True, "log_every": 0,
                                 "ckpt_every": 0, "graph": graph, "optim.warmup_examples": 8})
        return Trainer(cfg, ctx)

    data = SyntheticBatches(4, 32, "cuda", seed=5)
    batches = [next(data) for _ in range(3)]
    te, tg = make(False), make(True)
    assert torch.equal(te.flat.data, tg.flat.data)
    le = [te.train_step(*b).item() for b in batches]
    lg = [tg.train_step(*b).item() for b in batches]
    assert tg._graphed is not None and tg._graphed.defer == (micro == 0)
    tg.sync()
    for a, b in zip(le, lg):
        assert abs(a - b) <= 2e-3 * abs(a) + 1e-4, (le, lg)
    d = (te.flat.data - tg.flat.data).abs().max().item()
    assert d < 5e-4, d
    dm = (te.optim.exp_avg_sq - tg.optim.exp_avg_sq).abs().max().item()
    assert dm <= 1e-3 * te.optim.exp_avg_sq.abs().max().item() + 1e-12, dm
    assert tg.flat.grad.abs().max().item() == 0.0        # the flush zeroed the gradients like the eager step
    from distributed_3d_diffusion_pytorch_amd.ops import hip_impl
    hip_impl.set_device_seed(None)


def test_eager_grouped_wgrad_keeps_attention_split_order(monkeypatch):
    """D3D_WGRAD_EAGER_GROUP=1 (eager weight-gradient jobs queued and flushed
    as grouped launches) with the attention block's SPLIT backward: the C x C
    split job reads M = dy^T a, which the queued grouped job produces, so it
    must be queued behind it (GradSink.submit), never run ahead on a stale or
    uninitialised M.  Parameters after 2 eager steps match the default mode
    (one-job grouped launches, run at once)."""
    from distributed_3d_diffusion_pytorch_amd.config import make_config
    from distributed_3d_diffusion_pytorch_amd.engine import Trainer
    from distributed_3d_diffusion_pytorch_amd.parallel import DistContext
    from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches
    from distributed_3d_diffusion_pytorch_amd.ops.gradsink import SINK
    from distributed_3d_diffusion_pytorch_amd.ops import hip_impl
    monkeypatch.setattr(hip_impl, "_ATTN_SPLIT", 0)          # split backward at every attention block
    ctx = DistContext(device=torch.device("cuda", 0))
    data = SyntheticBatches(4, 32, "cuda", seed=7)
    batches = [next(data) for _ in range(2)]
    prev = (SINK.eager_group, SINK.eager_single)
    res = []
    try:
        for grp, single in ((False, True), (True, False)):
            SINK.eager_group, SINK.eager_single = grp, single
            torch.manual_seed(0)
            cfg = make_config(None, {"model.H": 32, "model.W": 32, "data.imgsize": 32, "global_batch": 4,
                                     "data.synthetic": True, "log_every": 0, "ckpt_every": 0,
                                     "optim.warmup_examples": 8})
            tr = Trainer(cfg, ctx)
            losses = [tr.train_step(*b).item() for b in batches]
            torch.cuda.synchronize()
            res.append((losses, tr.flat.data.clone()))
            del tr
    finally:
        SINK.eager_group, SINK.eager_single = prev
    (la, pa), (lb, pb) = res
    assert all(math.isfinite(v) for v in la + lb), (la, lb)
    assert max(abs(a - b) for a, b in zip(la, lb)) < 2e-3, (la, lb)
    assert (pa - pb).abs().max().item() < 5e-4


@pytest.mark.parametrize("N,Hh,C1,C2,OC", [(32, 64, 128, 0, 128), (12, 64, 256, 128, 128), (8, 128, 128, 0, 128)])
def test_gn_silu_conv_composition(H, N, Hh, C1, C2, OC):
    """GN0 + SiLU -> conv1 (`xunet.py:139-140`; C2 > 0: the decoder's virtual
    concat) forward and backward against the fp32 composition."""
    torch.manual_seed(9)
    C = C1 + C2
    xa = (torch.randn(N, Hh, Hh, C1, device=DEV) * 1.5 + 0.3).to(BF)
    xb = (torch.randn(N, Hh, Hh, C2, device=DEV) - 0.2).to(BF) if C2 else None
    gw = torch.randn(C, device=DEV) * 0.3 + 1
    gb = torch.randn(C, device=DEV) * 0.2
    w = torch.randn(OC, C, 3, 3, device=DEV) / math.sqrt(9 * C)
    dw_ = torch.randn(OC, C, device=DEV) / math.sqrt(C)
    go = torch.randn(N, Hh, Hh, OC, device=DEV)

    def hip(xa, xb, gw, gb, w):
        if xb is None:
            h = H.group_norm(xa, gw, gb, 32, 1e-5, True)
        else:
            h, _ = H.cat_gn_silu_dense(xa, xb, gw, gb, dw_, None)
        return H.conv3x3(h, w, None)

    def ref(xa, xb, gw, gb, w):
        x = xa if xb is None else torch.cat([xa, xb], -1)
        return T.conv3x3(T.group_norm(x, gw, gb, 32, 1e-5, True), w, None)

    ins = [xa, xb, gw, gb, w] if C2 else [xa, gw, gb, w]
    fh = hip if C2 else (lambda xa, gw, gb, w: hip(xa, None, gw, gb, w))
    fr = ref if C2 else (lambda xa, gw, gb, w: ref(xa, None, gw, gb, w))
    yh, yr, gh, gr = run_both(fh, fr, ins, go)
    assert rel(yh, yr) < 2e-2
    for a, b in zip(gh, gr):
        assert rel(a, b) < 3e-2, rel(a, b)


@pytest.mark.parametrize("s", [1, 2, 4, 8])
def test_cond_conv_split_matches_full_conv(H, s):
    """Origin/direction split conditioning conv == 144-channel conv on the
    rebuilt ray image (forward, weight / bias / per-image bias / residual
    gradients)."""
    torch.manual_seed(7)
    N, Hh, OC, no = 4, 16, 256, 93
    rays_dir = torch.zeros(N, Hh, Hh, 64, device=DEV)
    rays_dir[..., :51] = torch.randn(N, Hh, Hh, 51, device=DEV)
    rays_dir = rays_dir.to(BF)
    orig = torch.randn(N, no, device=DEV)
    w = torch.randn(OC, 144, 3, 3, device=DEV) / 36
    b = torch.randn(OC, device=DEV) * 0.1
    rb = torch.randn(N, OC, device=DEV)
    OHs = (Hh - 1) // s + 1
    res = torch.randn(2, OHs, OHs, OC, device=DEV).to(BF)
    go = torch.randn(N, OHs, OHs, OC, device=DEV)
    yh, yr, gh, gr = run_both(lambda w, b, rb, r: H.cond_conv(rays_dir, orig, w, b, s, rb, r, 2),
                              lambda w, b, rb, r: T.cond_conv(rays_dir.float(), orig, w, b, s, rb, r.float(), 2),
                              [w, b, rb, res], go)
    assert rel(yh, yr) < 2e-2
    for name, a, c in zip(["dw", "db", "drb", "dres"], gh, gr):
        assert rel(a, c) < 3e-2, (name, rel(a, c))


@pytest.mark.parametrize("N,Hh,s", [(4, 16, 1), (4, 16, 2), (4, 16, 4), (8, 64, 1), (8, 64, 2), (4, 64, 8),
                                    (32, 64, 4), (32, 64, 8), (64, 64, 8)])
def test_cond_conv_silu_companion(H, N, Hh, s):
    """cond_conv(silu_out=True): the conv epilogue (halo / w8 / bufl / split-K
    / small-tile forms, by shape) + the border correction write silu(output)
    next to the output -- bitwise what the SiLU pass makes of the stored
    output -- and film_batch consumes it (same projections as from the
    output alone)."""
    torch.manual_seed(8)
    OC, no = 1024, 93
    rays_dir = torch.zeros(N, Hh, Hh, 64, device=DEV)
    rays_dir[..., :51] = torch.randn(N, Hh, Hh, 51, device=DEV)
    rays_dir = rays_dir.to(BF)
    orig = torch.randn(N, no, device=DEV)
    w = torch.randn(OC, 144, 3, 3, device=DEV) / 36
    b = torch.randn(OC, device=DEV) * 0.1
    rb = torch.randn(N, OC, device=DEV)
    OHs = (Hh - 1) // s + 1
    res = torch.randn(2, OHs, OHs, OC, device=DEV).to(BF)
    with torch.no_grad():
        y = H.cond_conv(rays_dir, orig, w, b, s, rb, res, 2, silu_out=True)
        se = y._d3d_silu
        ref = torch.empty_like(y)
        H._chk(H._lib.d3d_silu(y.data_ptr(), ref.data_ptr(), y.numel(), H._st()), "silu")
        torch.cuda.synchronize()
        assert torch.equal(se, ref)
        ws = [torch.randn(256, OC, device=DEV) / 32, torch.randn(512, OC, device=DEV) / 32]
        bs = [torch.randn(256, device=DEV), torch.randn(512, device=DEV)]
        a = H.film_batch(y, ws, bs)
        y2 = y.clone()                         # no companion: film_batch runs its own SiLU pass
        c = H.film_batch(y2, ws, bs)
        for u, v in zip(a, c):
            assert torch.equal(u, v)


def test_sgemm_strided_matches_einsum(H):
    """Strided batched fp32 GEMM (small_gemm.hip) on the conditioning conv's
    three permuted products == the fp32 einsums, incl. beta accumulation."""
    torch.manual_seed(5)
    N, OC, IC, no = 6, 200, 144, 93
    pe = torch.randn(N, no, device=DEV)
    w = torch.randn(OC, IC, 3, 3, device=DEV)
    U = torch.empty(N, 9, OC, device=DEV)
    H._sgemm(pe, w, U, N, OC, no, 9, (0, no, 1), (1, 9, IC * 9), (OC, 9 * OC, 1))
    ref = torch.einsum("nk,okt->nto", pe, w[:, :no].reshape(OC, no, 9))
    assert rel(U, ref) < 1e-5
    M9 = torch.randn(9, 9, device=DEV)
    st = torch.randn(N, 9, OC, device=DEV)
    dU = torch.empty(N, 9, OC, device=DEV)
    H._sgemm(M9, st, dU, 9, OC, 9, N, (0, 9, 1), (9 * OC, OC, 1), (9 * OC, OC, 1))
    assert rel(dU, torch.einsum("tk,nko->nto", M9, st)) < 1e-5
    tgt = torch.randn(OC, IC, 3, 3, device=DEV)
    want = tgt.clone()
    want.view(OC, IC, 9)[:, :no] += torch.einsum("nto,nk->okt", dU, pe)
    H._sgemm(dU, pe, tgt.view(OC, IC, 9), OC, no, N, 9, (OC, 1, 9 * OC), (0, no, 1), (1, IC * 9, 9), beta=1.0)
    assert rel(tgt, want) < 1e-5


def test_ray_dir_matches_torch(H):
    torch.manual_seed(2)
    B, Hh = 3, 16
    R = torch.linalg.qr(torch.randn(B, 2, 3, 3, device=DEV))[0]
    t = torch.randn(B, 2, 3, device=DEV)
    K = torch.tensor([[20.0, 0, 8], [0, 20.0, 8], [0, 0, 1]], device=DEV).expand(B, 3, 3).contiguous()
    mask = torch.tensor([True, False, True], device=DEV)
    a = H.ray_posenc_dir(R, t, K, Hh, Hh, mask).float()
    b = T.ray_posenc_dir(R, t, K, Hh, Hh, mask)
    assert (a - b).abs().max().item() < 2e-2
    full = T.ray_posenc(R, t, K, Hh, Hh, mask, None, None, None)
    assert torch.allclose(T.ray_origin_pe(t, mask)[:, None, None, :].expand(-1, Hh, Hh, -1), full[..., :93])


@pytest.mark.parametrize("C1,C2,OC", [(256, 128, 128), (128, 128, 128), (512, 512, 512), (512, 256, 256)])
@pytest.mark.parametrize("Hh", [8, 32])
def test_cat_gn_silu_dense(H, C1, C2, OC, Hh):
    """Decoder block entry on the virtual concat == GN+SiLU and dense on the
    materialised concat (forward and every gradient); the skip runs as two
    GEMMs, the second accumulating through its residual epilogue."""
    torch.manual_seed(11)
    N = 4
    a = (torch.randn(N, Hh, Hh, C1, device=DEV) + 0.3).to(BF)
    b = (torch.randn(N, Hh, Hh, C2, device=DEV) * 2).to(BF)
    gw = torch.rand(C1 + C2, device=DEV) + 0.5
    gb = torch.randn(C1 + C2, device=DEV) * 0.1
    dw = torch.randn(OC, C1 + C2, 1, 1, device=DEV) / 20
    db = torch.randn(OC, device=DEV) * 0.1
    gy = torch.randn(N, Hh, Hh, C1 + C2, device=DEV)
    gs = torch.randn(N, Hh, Hh, OC, device=DEV)

    def run(hip):
        ins = [leaf(a) if hip else leaf(a, torch.float32), leaf(b) if hip else leaf(b, torch.float32),
               leaf(gw), leaf(gb), leaf(dw), leaf(db)]
        y, s = (H if hip else T).cat_gn_silu_dense(*ins, 32, 1e-5)
        ((y.float() * gy).sum() + (s.float() * gs).sum()).backward()
        return [y, s] + [t.grad for t in ins]

    hr, rr = run(True), run(False)
    names = ["y", "skip", "da", "db", "dgw", "dgb", "ddw", "ddb"]
    for n, x, r in zip(names, hr, rr):
        assert rel(x, r) < 3e-2, (n, rel(x, r))


@pytest.mark.parametrize("C,OC,N,Hh", [(128, 128, 3, 10), (256, 256, 2, 16), (512, 512, 5, 8), (128, 256, 1, 64),
                                       (256, 512, 3, 7)])
@pytest.mark.parametrize("with_bias", [True, False])
def test_cat_gemm_one_launch(H, C, OC, N, Hh, with_bias):
    """Decoder NIN skip over [h | skip] with equal halves as ONE GEMM
    (gemm.hip F_CAT: the B operand switches tensors at K = C) == the fp32
    dense of the materialised concat and == the two-GEMM form; pixel counts
    that leave partial 256 / 128 / 64-row tiles (rows past the end read
    zeros through each half's own descriptor range); the decoder op takes
    the one-GEMM path for equal halves."""
    from distributed_3d_diffusion_pytorch_amd.ops import hip_impl as HI
    torch.manual_seed(5)
    P = N * Hh * Hh
    a = torch.randn(P, C, device=DEV).to(BF)
    b = (torch.randn(P, C, device=DEV) * 2).to(BF)
    w = (torch.randn(OC, 2 * C, device=DEV) / 20).to(BF)
    db = torch.randn(OC, device=DEV) * 0.1 if with_bias else None
    ref = torch.cat([a, b], -1).float() @ w.float().t()
    if with_bias:
        ref = ref + db
    one = torch.full((P, OC), float("nan"), device=DEV, dtype=BF)
    rc = HI._lib.d3d_gemm_cat(w.data_ptr(), a.data_ptr(), b.data_ptr(), C, one.data_ptr(), HI._ptr(db), OC, P,
                              2 * C, 2 * C, OC, 1.0, 1.0, HI._st())
    assert rc == 0, rc
    two = torch.empty(P, OC, device=DEV, dtype=BF)
    HI.gemm_nt(w, a, two, OC, P, C, 2 * C, C, OC, bias=db)
    HI.gemm_nt(w[:, C:], b, two, OC, P, C, 2 * C, C, OC, res=two)
    torch.cuda.synchronize()
    assert rel(one.float(), ref) < 1e-2, rel(one.float(), ref)
    assert rel(two.float(), ref) < 1e-2, rel(two.float(), ref)
    assert rel(one.float(), two.float()) < 1e-2
    # unequal halves are refused (the op falls back to two GEMMs)
    assert HI._lib.d3d_gemm_cat(w.data_ptr(), a.data_ptr(), b.data_ptr(), C // 2, one.data_ptr(), HI._ptr(db), OC,
                                P, 2 * C, 2 * C, OC, 1.0, 1.0, HI._st()) < 0 or C // 2 < 64


@pytest.mark.parametrize("OC,IC,taps", [(128, 128, 9), (256, 384, 9), (1024, 144, 9), (3, 128, 9),
                                        (2048, 1024, 1), (768, 256, 1), (128, 3, 9)])
def test_batched_weight_refresh_matches_pack(H, OC, IC, taps):
    """pack_all_k (one launch re-derives every cached operand after the
    optimizer step) == the per-weight pack kernel, for forward and transposed
    packs and the plain bf16 cast."""
    torch.manual_seed(11)
    shape = (OC, IC, 3, 3) if taps == 9 else (OC, IC)
    w = torch.nn.Parameter(torch.randn(*shape, device=DEV))
    fwd = H.packed_weight(w, False, taps)
    trn = H.packed_weight(w, True, taps)
    cast = H.bf16_weight(w) if taps == 1 else None
    with torch.no_grad():
        w.mul_(-0.5).add_(0.25)           # an "optimizer step" on the fp32 master
    H.refresh_weights()
    ref_f = H.packed_weight(torch.nn.Parameter(w.detach().clone()), False, taps)
    ref_t = H.packed_weight(torch.nn.Parameter(w.detach().clone()), True, taps)
    assert torch.equal(fwd, ref_f)
    assert torch.equal(trn, ref_t)
    if cast is not None:
        assert torch.equal(cast.reshape(-1), w.detach().to(BF).reshape(-1))


@pytest.mark.parametrize("N,Hh,Ci,Co,fused,res", [
    (16, 64, 128, 128, True, False),      # w8 128x512 tiles, 4-channel groups
    (32, 32, 256, 256, True, False),      # 8-channel groups
    (128, 16, 256, 256, True, True),      # 4-wave 128x128 kernel
    (32, 32, 512, 512, True, False),      # w8 256x256, 16-channel groups
    (16, 32, 1024, 1024, True, False),    # 32-channel groups span two MFMA row tiles
    (64, 8, 512, 512, True, True),        # split-K grid: statistics from the split-K epilogue
    (2, 16, 128, 256, True, False),       # split-K, 8-channel groups
    (2, 16, 64, 96, False, False),        # OC % 64 != 0 under split-K: separate statistics pass
    (32, 8, 512, 512, True, True),        # 64x64 small tiles (conv_small.hip), 16-channel groups
    (32, 8, 1024, 1024, True, False),     # small tiles, 32-channel groups
    (32, 16, 256, 256, True, True)])      # small tiles, 8-channel groups
def test_conv_fused_gn_stats(H, no_gn_img, N, Hh, Ci, Co, fused, res):
    """GroupNorm statistics emitted by the conv epilogue (w8 / bufl / split-K
    epilogue paths) == the separate statistics pass: GN+SiLU and GN-FiLM."""
    torch.manual_seed(12)
    x = torch.randn(N, Hh, Hh, Ci, device=DEV).to(BF)
    w = torch.randn(Co, Ci, 3, 3, device=DEV) / math.sqrt(9 * Ci)
    b = torch.randn(Co, device=DEV) * 0.3 + 0.2
    gam = torch.rand(Co, device=DEV) + 0.5
    bet = torch.randn(Co, device=DEV) * 0.1
    r = torch.randn(N, Hh, Hh, Co, device=DEV).to(BF) if res else None
    y = H.conv3x3(x, w, b, residual=r, out_scale=1 / math.sqrt(2) if res else 1.0, gn_groups=32)
    if res:
        ref = F.conv2d(x.float().permute(0, 3, 1, 2), w, b, 1, 1).permute(0, 2, 3, 1)
        ref = (ref + r.float()) / math.sqrt(2)
        assert rel(y, ref) < 2e-2, rel(y, ref)
    assert hasattr(y, "_d3d_gnpart") == fused, "fused GroupNorm partials not produced as planned"
    plain = y.detach().clone()            # no partials attached: statistics pass
    a = H.group_norm(y, gam, bet, 32, 1e-5, True)
    r = H.group_norm(plain, gam, bet, 32, 1e-5, True)
    assert rel(a, r) < 1e-2, rel(a, r)
    ss = (torch.randn(N, Hh, Hh, 2 * Co, device=DEV) * 0.5).to(BF)
    a2 = H.gn_film(y, gam, bet, ss, 32, 1e-5, 0.0, False, 0)
    r2 = H.gn_film(plain, gam, bet, ss, 32, 1e-5, 0.0, False, 0)
    assert rel(a2, r2) < 1e-2, rel(a2, r2)


def test_training_step_bitwise_deterministic():
    """Race screen: two identical 2-step training runs through
    every HIP kernel (split-K slabs, fused GroupNorm partials, attention,
    dropout masks) produce bitwise-identical parameters and losses, with the
    weight gradients on the side stream (ops/gradsink.py) or not."""
    from distributed_3d_diffusion_pytorch_amd.config import make_config
    from distributed_3d_diffusion_pytorch_amd.engine import Trainer
    from distributed_3d_diffusion_pytorch_amd.parallel import DistContext
    from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches
    ctx = DistContext(device=torch.device("cuda", 0))
    data = SyntheticBatches(8, 64, "cuda", seed=21)
    batches = [next(data) for _ in range(2)]
    from distributed_3d_diffusion_pytorch_amd.ops.gradsink import SINK
    runs = []
    prev = SINK.stream_enabled
    # the third run puts the weight gradients back on the compute stream: the
    # side stream must not change a single bit either
    for side in (True, True, False):
        SINK.stream_enabled = side
        torch.manual_seed(0)
        cfg = make_config(None, {"model.H": 64, "model.W": 64, "data.imgsize": 64, "global_batch": 8,
                                 "micro_batch": 4, "data.synthetic": True, "log_every": 0, "ckpt_every": 0,
                                 "optim.warmup_examples": 0})
        tr = Trainer(cfg, ctx)
        losses = [tr.train_step(*b).item() for b in batches]
        runs.append((losses, tr.flat.data.clone()))
        del tr
    SINK.stream_enabled = prev
    for r in runs[1:]:
        assert runs[0][0] == r[0], runs
        assert torch.equal(runs[0][1], r[1]), (runs[0][1] - r[1]).abs().max().item()


def test_graph_step_bitwise_deterministic():
    """Race screen of the REPLAYED step (the 8-GPU per-GPU share):
    64x64, batch 16, one micro-batch, graph=True -- so the captured step runs
    the deferred overlapped update (update stream + parameter fence), the
    conditioning stream and the in-graph weight-gradient side stream (jobs
    flushed 8 per fork).  Two identical 4-step runs must agree bit for bit in
    losses, parameters, Adam moments and the EMA-free flat gradient; a third
    run with the weight-gradient side stream off must too (every reduction has
    a fixed order, so stream placement may not change a bit)."""
    from distributed_3d_diffusion_pytorch_amd.config import make_config
    from distributed_3d_diffusion_pytorch_amd.engine import Trainer
    from distributed_3d_diffusion_pytorch_amd.parallel import DistContext
    from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches
    from distributed_3d_diffusion_pytorch_amd.ops.gradsink import SINK
    from distributed_3d_diffusion_pytorch_amd.ops import hip_impl
    ctx = DistContext(device=torch.device("cuda", 0))
    data = SyntheticBatches(16, 64, "cuda", seed=33)
    batches = [next(data) for _ in range(4)]
    runs = []
    prev = SINK.stream_enabled
    try:
        for side in (True, True, False):
            SINK.stream_enabled = side
            torch.manual_seed(0)
            cfg = make_config(None, {"model.H": 64, "model.W": 64, "data.imgsize": 64, "global_batch": 16,
                                     "micro_batch": 0, "data.synthetic": True, "log_every": 0, "ckpt_every": 0,
                                     "graph": True, "optim.warmup_examples": 32})
            tr = Trainer(cfg, ctx)
            losses = [tr.train_step(*b).item() for b in batches]
            g = tr._graphed
            assert g is not None and g.defer, "graph step with the deferred update expected"
            tr.sync()
            torch.cuda.synchronize()
            runs.append((losses, tr.flat.data.clone(), tr.optim.exp_avg.clone(), tr.optim.exp_avg_sq.clone()))
            del tr, g
    finally:
        SINK.stream_enabled = prev
        hip_impl.set_device_seed(None)
    ref = runs[0]
    assert hip_impl.FALLBACKS == {}, hip_impl.FALLBACKS     # every op of the replayed step ran natively
    assert all(math.isfinite(v) for v in ref[0]), ref[0]
    for r in runs[1:]:
        assert ref[0] == r[0], (ref[0], r[0])
        for a, b in zip(ref[1:], r[1:]):
            assert torch.equal(a, b), (a - b).abs().max().item()


@pytest.mark.parametrize("kind", ["conv_res", "linear_res", "nin_input", "skip_concat"])
def test_residual_grad_slot(H, kind):
    """ResGradSlot: the residual branch's gradient of x handed to the
    GroupNorm backward kernel == autograd summing the two branches.
    skip_concat: x also feeds a decoder-style virtual concat [y | x]
    (cat_gn_silu_dense), whose gradient of x is the slot's second deposit."""
    torch.manual_seed(5)
    C, Co = 128, (256 if kind == "nin_input" else 128)
    x = torch.randn(4, 16, 16, C, device=DEV).to(BF).requires_grad_(True)
    gam = torch.rand(C, device=DEV) + 0.5
    bet = torch.randn(C, device=DEV) * 0.1
    w = torch.randn(Co, C, 3, 3, device=DEV) / math.sqrt(9 * C)
    wl = torch.randn(Co, C, device=DEV) / math.sqrt(C)
    bl = torch.randn(Co, device=DEV) * 0.1
    go = torch.randn(4, 16, 16, Co, device=DEV).to(BF)
    gam2 = torch.rand(2 * C, device=DEV) + 0.5
    bet2 = torch.randn(2 * C, device=DEV) * 0.1
    wd = torch.randn(C, 2 * C, device=DEV) / math.sqrt(2 * C)
    bd = torch.randn(C, device=DEV) * 0.1
    go2 = torch.randn(4, 16, 16, 2 * C, device=DEV)
    go3 = torch.randn(4, 16, 16, C, device=DEV)

    def run(use):
        x.grad = None
        x.__dict__.pop("_d3d_res_slot", None)
        slot = H.ResGradSlot() if use else None
        if kind == "conv_res":
            h = H.group_norm(x, gam, bet, 32, 1e-5, True, slot)
            y = H.conv3x3(h, w, None, residual=x, out_scale=1 / math.sqrt(2), res_slot=slot)
        elif kind == "linear_res":
            h = H.group_norm(x, gam, bet, 32, 1e-5, False, slot)
            y = H.linear(h, wl, bl, residual=x, out_scale=1 / math.sqrt(2), res_slot=slot)
        elif kind == "nin_input":
            h = H.group_norm(x, gam, bet, 32, 1e-5, True, slot)
            s = H.linear(x, wl, bl, in_slot=slot)
            y = H.conv3x3(h, w, None, residual=s, out_scale=1 / math.sqrt(2))
        else:
            h = H.group_norm(x, gam, bet, 32, 1e-5, True, slot)
            y1 = H.conv3x3(h, w, None, residual=x, out_scale=1 / math.sqrt(2), res_slot=slot)
            if use:
                x._d3d_res_slot = slot
            hc, sk = H.cat_gn_silu_dense(y1, x, gam2, bet2, wd, bd, 32)
            ((hc.float() * go2).sum() + (sk.float() * go3).sum()).backward()
            if use:
                assert slot.consumed and slot.g is None and slot.g2 is None
            return x.grad.float().clone()
        y.backward(go)
        if use:
            assert slot.consumed and slot.g is None
        return x.grad.float().clone()

    a, b = run(True), run(False)
    assert rel(a, b) < 1e-2, rel(a, b)


@pytest.mark.parametrize("N,period", [(256, 2), (6, 2), (5, 1)])
def test_period_sum_matches_fp32(H, N, period):
    """period_sum_k (gradient of a batch-broadcast residual) == fp32 torch sum
    over the repeats, cast to bf16."""
    torch.manual_seed(2)
    g = torch.randn(N, 8, 8, 40, device=DEV).to(BF)
    out = H._period_sum(g, period)
    ref = g.float().reshape(N // period, period, 8, 8, 40).sum(0)
    assert out.shape == (period, 8, 8, 40) and out.dtype == BF
    assert (out.float() - ref).abs().max().item() <= 0.01 * ref.abs().max().item() + 1e-2


def test_diffusion_inputs_kernel_matches_torch(H):
    """diffusion_fwd2_k (one launch: t, lambda, eps, q_sample, CFG drop, NHWC
    stem input) == the torch composition of the same counter-based draw."""
    torch.manual_seed(3)
    img = (torch.rand(24, 2, 3, 32, 32, device=DEV) * 2 - 1)
    xz, eps, lam, keep = H.diffusion_inputs(img, 0xDEADBEEF12345678, e0=5, cond_prob=0.3)
    xr, er, lr, kr = T.diffusion_inputs(img, 0xDEADBEEF12345678, e0=5, cond_prob=0.3, dtype=torch.float32)
    assert torch.equal(keep, kr) and 0 < int((~keep).sum()) < 24
    assert (lam - lr).abs().max().item() < 2e-4 * 20
    assert (eps - er).abs().max().item() < 1e-3
    assert (xz.float() - xr).abs().max().item() < 2e-2
    # graph form: baked seed + device words [dropout, draw word, offset]
    word, off = 7, 3
    seed_blk = torch.tensor([0, word, off], dtype=torch.int64, device=DEV)
    base = 0x1111
    H.set_device_seed(seed_blk)
    try:
        xg, eg, lg, kg = H.diffusion_inputs(img, base, e0=0)
    finally:
        H.set_device_seed(None)
    xe, ee, le, ke = H.diffusion_inputs(img, (base + word * 0x9E3779B97F4A7C15) & (2 ** 64 - 1), e0=off)
    assert torch.equal(eg, ee) and torch.equal(xg, xe) and torch.equal(lg, le) and torch.equal(kg, ke)


@pytest.mark.parametrize("loss_type", ["l2", "l1", "huber"])
def test_diff_loss_kernel(H, loss_type):
    torch.manual_seed(4)
    y = torch.randn(6, 32, 32, 8, device=DEV).to(BF)
    y[..., 3:] = 0
    eps = torch.randn(6, 3, 32, 32, device=DEV)
    yh = leaf(y)
    yr = leaf(y, torch.float32)
    lh = H.diff_loss_nhwc(yh, eps, loss_type)
    lr_ = T.diff_loss_nhwc(yr, eps, loss_type)
    assert abs(lh.item() - lr_.item()) < 1e-5 * abs(lr_.item())
    (lh * 0.37).backward()
    (lr_ * 0.37).backward()
    assert rel(yh.grad, yr.grad) < 1e-2
    assert float(yh.grad[..., 3:].abs().max()) == 0.0


def _probe_worker(out_dir):
    import datetime
    import torch.distributed as dist
    from distributed_3d_diffusion_pytorch_amd.parallel import cleanup
    from distributed_3d_diffusion_pytorch_amd.parallel.dist import rccl_env_defaults
    from distributed_3d_diffusion_pytorch_amd.engine.graphs import probe_graph_collective
    # a 1-rank RCCL group (init_distributed skips the group at world 1; RCCL
    # refuses two ranks on one device, so 1 rank is all a 1-GPU box can run)
    rccl_env_defaults()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev, timeout=datetime.timedelta(seconds=120))
    ok = probe_graph_collective(dev)
    with open(os.path.join(out_dir, "probe.txt"), "w") as f:
        f.write(f"{int(ok)} {dist.get_backend()}")
    cleanup()


def test_rccl_allreduce_graph_capture_probe(tmp_path):
    """The RCCL ("nccl") process group on this stack can capture an
    all-reduce into a HIP graph and replay it correctly (the mechanism the
    multi-GPU graph step overlaps its gradient reduction with)."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from distributed_3d_diffusion_pytorch_amd.parallel import spawn
    import test_ops_gpu as me
    spawn(me._probe_worker, 1, (str(tmp_path),))
    ok, be = open(tmp_path / "probe.txt").read().split()
    assert be == "nccl" and ok == "1"


def _graph_comm_worker(out_dir, graph_comm="1"):
    """world=2 RCCL: the graph step with the all-reduce captured inside graph
    A (graph_comm "1"), or captured as segments with eager bucket all-reduces
    between the replays (graph_comm "0": comm_mode "seg"), must equal the
    eager bucketed step, with identical parameters on both ranks."""
    os.environ["D3D_GRAPH_COMM"] = graph_comm
    import torch.distributed as dist
    from distributed_3d_diffusion_pytorch_amd.config import make_config
    from distributed_3d_diffusion_pytorch_amd.engine import Trainer
    from distributed_3d_diffusion_pytorch_amd.parallel import init_distributed, cleanup
    from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches
    ctx = init_distributed("nccl", 180)

    def make(graph):
        cfg = make_config(None, {"model.H": 32, "model.W": 32, "data.imgsize": 32, "global_batch": 8,
                                 "data.synthetic": True, "log_every": 0, "ckpt_every": 0, "graph": graph,
                                 "optim.warmup_examples": 16, "dist.bucket_mb": 16.0})
        return Trainer(cfg, ctx)

    data = SyntheticBatches(4, 32, "cuda", seed=11 + ctx.rank)
    batches = [next(data) for _ in range(3)]
    res = []
    for graph in (False, True):
        tr = make(graph)
        losses = [float(tr.train_step(*b)) for b in batches]
        mode = tr._graphed.comm_mode if tr._graphed is not None else "eager"
        tr.sync()
        p = tr.flat.data.clone()
        other = p.clone()
        dist.broadcast(other, 0)
        res.append((losses, p, (p - other).abs().max().item(), mode))
        del tr
    (le, pe, de, _), (lg, pg, dg, mode) = res
    with open(os.path.join(out_dir, f"gc{ctx.rank}.txt"), "w") as f:
        f.write(f"{(pe - pg).abs().max().item()} {de} {dg} {max(abs(a - b) for a, b in zip(le, lg))} {mode}")
    cleanup()


def _graph_comm_1rank_worker(out_dir, bucket_flush=False):
    """The multi-GPU step topology on ONE GPU: a 1-rank RCCL group with the
    bucketed reducer forced on (dist.force_comm), so graph A is captured with
    the real bucket all-reduces, the sink's collective flushes, the
    conditioning stream and the deferred update -- against the eager bucketed
    step, for fp32 and bf16 gradient payloads."""
    import datetime
    import torch.distributed as dist
    from distributed_3d_diffusion_pytorch_amd.config import make_config
    from distributed_3d_diffusion_pytorch_amd.engine import Trainer
    from distributed_3d_diffusion_pytorch_amd.parallel import DistContext, cleanup
    from distributed_3d_diffusion_pytorch_amd.parallel.dist import rccl_env_defaults
    from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches
    rccl_env_defaults()
    if bucket_flush:
        # bucket-aware sink flushing (the round-5 NaN variant; experimental)
        os.environ["D3D_WGRAD_BUCKET_FLUSH"] = "1"
        os.environ["D3D_WGRAD_DEFER_BATCH"] = "16"
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev, timeout=datetime.timedelta(seconds=120))
    ctx = DistContext(device=dev)
    data = SyntheticBatches(4, 32, "cuda", seed=21)
    batches = [next(data) for _ in range(3)]
    lines = []
    # (payload, micro-batch): one micro-batch (deferred update) for both
    # payloads, and two micro-batches, where the leading one's graph gA0 is
    # captured next to the comm graph (thread_local, no watchdog wait)
    # gc "0": no RCCL capture -> the segmented capture (comm_mode "seg"); "p":
    # no segmented capture either (D3D_GRAPH_SEG=0) -> the post-graph reduction
    for gd, mb, gc in (("fp32", 0, "1"), ("bf16", 0, "1"), ("fp32", 2, "1"), ("fp32", 0, "0"), ("bf16", 0, "0"),
                       ("fp32", 2, "0"), ("fp32", 0, "p"), ("bf16", 0, "p")):
        os.environ["D3D_GRAPH_COMM"] = "1" if gc == "1" else "0"
        os.environ["D3D_GRAPH_SEG"] = "0" if gc == "p" else "64"
        res = []
        for graph in (False, True):
            cfg = make_config(None, {"model.H": 32, "model.W": 32, "data.imgsize": 32, "global_batch": 4,
                                     "micro_batch": mb, "data.synthetic": True, "log_every": 0, "ckpt_every": 0,
                                     "graph": graph, "optim.warmup_examples": 8, "dist.bucket_mb": 16.0,
                                     "dist.grad_dtype": gd, "dist.force_comm": True})
            tr = Trainer(cfg, ctx)
            assert tr.reducer is not None and tr.reducer.active
            assert (tr.sink.bucket_flush is not None) == (bucket_flush and gd == "fp32")   # (bf16: kept off)
            # race probe: each collective reduces a snapshot of its bucket taken
            # at issue time (result discarded: 1-rank identity); after every step
            # the snapshots must equal the complete gradient bit for bit
            tr.reducer.enable_race_probe()
            losses, race = [], 0.0
            for b in batches:
                losses.append(float(tr.train_step(*b)))
                snap, final = tr.reducer.race_probe
                race = max(race, (snap - final).abs().max().item())
                probed = final.abs().max().item() > 0
            g = tr._graphed
            mode = f"{g.comm_mode}/{int(g.defer)}/{int(g.gA0 is not None)}" if g is not None else "eager"
            if g is not None and g.segs is not None:
                mode += f"/{len(g.segs)}/{sum(len(b) for b in g.seg_bk)}/{len(tr.reducer.buckets)}"
            tr.sync()
            res.append((losses, tr.flat.data.clone(), mode, race, probed))
            exposed = g.measure_comm(2) if g is not None else 0.0      # (changes the training state)
            del tr
        (le, pe, _, re_, pre), (lg, pg, mode, rg, prg) = res
        lines.append(f"{gd}/{mb}/{gc} {(pe - pg).abs().max().item()} {max(abs(a - b) for a, b in zip(le, lg))} "
                     f"{mode} {exposed} {re_} {rg} {int(pre)}{int(prg)}")
    os.environ.pop("D3D_GRAPH_COMM", None)
    os.environ.pop("D3D_GRAPH_SEG", None)
    with open(os.path.join(out_dir, "gc1.txt"), "w") as f:
        f.write("\n".join(lines))
    cleanup()


def test_graph_step_captured_collectives_one_rank(tmp_path, bucket_flush=False):
    """Graph A captured with the real bucketed RCCL all-reduces (1-rank
    group), deferred update on, fp32 and bf16 payloads, and a two-micro-batch
    step (leading graph gA0 captured too): comm_mode "graph", parameters equal
    to the eager bucketed step within 5e-4.  No sleep before any capture.
    The same three with D3D_GRAPH_COMM=0: comm_mode "seg" (graph A captured
    as a chain of segments cut every 64 MiB of complete buckets, each
    segment's buckets all-reduced eagerly between the replays, deferred update
    kept): more than one segment, every bucket issued exactly once, the same
    parameters.  With D3D_GRAPH_SEG=0 as well: comm_mode "post" (chunked bf16
    reduction after the replay, each chunk's Adam behind its collective).
    measure_comm works in every mode.  Every row runs the reducer's race probe
    (GradReducer.enable_race_probe): a collective that read its bucket before
    the last deposit landed -- invisible to a 1-rank in-place all-reduce --
    fails the test.  (``bucket_flush``: the same with the opt-in bucket-aware
    weight-gradient flushing, D3D_WGRAD_BUCKET_FLUSH=1 -- not run by the
    suite: that experimental mode showed NaN / a crash in this step at some
    flush batches, profiles/r6/bucket_flush.txt; tools/diag_bucket_flush_race.py
    runs it.)"""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from distributed_3d_diffusion_pytorch_amd.parallel import spawn
    import test_ops_gpu as me
    spawn(me._graph_comm_1rank_worker, 1, (str(tmp_path), bucket_flush))
    rows = open(tmp_path / "gc1.txt").read().split("\n")
    assert [r.split()[0] for r in rows] == ["fp32/0/1", "bf16/0/1", "fp32/2/1", "fp32/0/0", "bf16/0/0", "fp32/2/0",
                                            "fp32/0/p", "bf16/0/p"]
    for r in rows:
        gd, d, dl, mode, exp, race_e, race_g, probed = r.split()
        # no collective read a bucket before its last deposit (eager step, and
        # the captured / segmented steps; the post mode reduces after the replay)
        assert float(race_e) == 0.0 and float(race_g) == 0.0, r
        assert probed == ("10" if gd.endswith("/p") else "11"), r
        if gd.endswith("/1"):
            assert mode == ("graph/0/1" if gd == "fp32/2/1" else "graph/1/0"), r
        elif gd.endswith("/0"):
            # no RCCL capture: segmented capture, deferred update with one micro-batch
            m = mode.split("/")
            assert m[:3] == (["seg", "0", "1"] if gd == "fp32/2/0" else ["seg", "1", "0"]), r
            assert int(m[3]) > 1 and m[4] == m[5], r       # several segments; every bucket once
            assert float(exp) >= 0.0, r
        else:
            # no segmented capture either: the chunked post-graph reduction (bf16 payload), no deferred update
            assert mode == "post/0/0" and float(exp) >= 0.0, r
        assert float(d) < 5e-4 and float(dl) < 2e-3, r


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs 2 GPUs (RCCL: one rank per device)")
@pytest.mark.parametrize("graph_comm,want", [("1", "graph"), ("0", "seg")])
def test_graph_step_rccl_captured_allreduce_two_gpus(tmp_path, graph_comm, want):
    """2 ranks on 2 GPUs: the captured-collective step and the segmented
    fallback (the path taken whenever the RCCL capture probe fails: bucket
    all-reduces issued eagerly between segment replays, agreed segment
    layout) against the eager bucketed step; replicas identical."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from distributed_3d_diffusion_pytorch_amd.parallel import spawn
    import test_ops_gpu as me
    spawn(me._graph_comm_worker, 2, (str(tmp_path), graph_comm))
    for r in range(2):
        d, de, dg, dl, mode = open(tmp_path / f"gc{r}.txt").read().split()
        assert mode == want
        assert float(de) == 0.0 and float(dg) == 0.0
        assert float(d) < 5e-4 and float(dl) < 2e-3


def test_sampler_step2_matches_posterior(H):
    """Graph-form CFG step (eps read from the padded NHWC head output, scalars
    from the device block) == cfg_posterior + the counter-based noise."""
    from distributed_3d_diffusion_pytorch_amd.diffusion import cfg_posterior
    from distributed_3d_diffusion_pytorch_amd.engine import DiffusionSampler
    torch.manual_seed(12)
    b, S = 3, 16
    y = torch.randn(2 * b, S, S, 8, device=DEV).to(BF)
    z = torch.randn(b, 3, S, S, device=DEV)
    w = torch.tensor([0.0, 2.0, 5.0], device=DEV)
    smp = DiffusionSampler(torch.nn.Linear(1, 1).to(DEV), timesteps=8, seed=3, chain_offset=4)
    for k in (2, 7):
        prm = torch.tensor(smp.params(k), device=DEV)
        zz = z.clone()
        H.sampler_step2(zz, y, w, prm, None, smp.step_seed(k), 4)
        ec = y[:b, ..., :3].float().permute(0, 3, 1, 2)
        eu = y[b:, ..., :3].float().permute(0, 3, 1, 2)
        mean, var = cfg_posterior(z, ec, eu, w, torch.tensor(smp.lam[k]), torch.tensor(smp.lam_next[k]))
        if smp.add_noise(k):
            mean = mean + var.sqrt() * smp._noise(T.K_NZ, k, (b, 3, S, S), torch.device(DEV))
        assert (zz - mean).abs().max().item() < 1e-4


def test_sampler_graph_replay_matches_eager():
    """256-step sampler: the HIP-graph replayed step == the eager step with the
    same kernels and seeds (a few steps, 2 record entries)."""
    from distributed_3d_diffusion_pytorch_amd.models import XUNet
    from distributed_3d_diffusion_pytorch_amd.engine import DiffusionSampler, RecordEntry
    from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches
    torch.manual_seed(13)
    m = XUNet(H=32, W=32, ch=128).to(DEV)
    with torch.no_grad():
        for p in m.parameters():
            if p.abs().sum() == 0:
                p.normal_(0, 0.02)
    m.compute_dtype = BF
    m.eval()
    img, R, t, K = next(SyntheticBatches(4, 32, DEV, seed=1))
    rec = [RecordEntry(img[:, 0].contiguous(), R[0, 0].float(), t[0, 0].float()),
           RecordEntry(img[:, 1].contiguous(), R[1, 0].float(), t[1, 0].float())]
    w = torch.tensor([0.0, 1.0, 2.0, 3.0])
    outs = []
    for graph in (False, True):
        smp = DiffusionSampler(m, timesteps=5, seed=9, device=torch.device(DEV), graph=graph)
        outs.append(smp.sample(rec, R[2, 1].float(), t[2, 1].float(), K[0].float(), w))
    assert torch.isfinite(outs[0]).all()
    assert (outs[0] - outs[1]).abs().max().item() < 1e-3


def test_sampler_shared_cond_matches_per_chain():
    """HIP sampler step with the conditioning computed per class (4
    conditioning images, GN-FiLM through the row -> class map) == the
    per-chain step, to bf16 accuracy.  Compared on single mid-schedule steps:
    a whole short-schedule run is ill-conditioned (x0 = (z - sigma eps) /
    alpha with alpha ~ 5e-5 at logsnr -20 amplifies bf16 rounding to the
    x0 clamp), so bitwise agreement is only expected between identical
    kernel sequences (test_sampler_graph_replay_matches_eager)."""
    from distributed_3d_diffusion_pytorch_amd.models import XUNet
    from distributed_3d_diffusion_pytorch_amd.engine import DiffusionSampler
    from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches
    torch.manual_seed(14)
    m = XUNet(H=32, W=32, ch=128).to(DEV)
    with torch.no_grad():
        for p in m.parameters():
            if p.abs().sum() == 0:
                p.normal_(0, 0.02)
    m.compute_dtype = BF
    m.eval()
    b = 4
    img, R, t, K = next(SyntheticBatches(b, 32, DEV, seed=2))
    Rb = torch.stack([R[0, 0], R[1, 1]])[None].expand(b, 2, 3, 3).float().contiguous()
    Tb = torch.stack([t[0, 0], t[1, 1]])[None].expand(b, 2, 3).float().contiguous()
    Kb = K[0].float()[None].expand(b, 3, 3).contiguous()
    w = torch.tensor([0.0, 1.0, 2.0, 3.0], device=DEV)
    smp = DiffusionSampler(m, timesteps=256, seed=9, device=torch.device(DEV))
    z = torch.randn(b, 3, 32, 32, device=DEV)
    for k in (100, 128, 200):
        za = smp.step(z, img[:, 0], Rb, Tb, Kb, w, k, shared=False)
        zb = smp.step(z, img[:, 0], Rb, Tb, Kb, w, k, shared=True)
        assert torch.isfinite(zb).all()
        assert rel(zb, za) < 1e-2, (k, rel(zb, za))


def test_full_model_64px_matches_fp32_oracle():
    """HIP bf16 X-UNet (full 136.7M architecture at 64x64, zero-init layers
    given random weights so every path carries signal) against the
    independent fp32 NCHW oracle models/reference.py: output and EVERY
    parameter gradient, by relative L2 error -- bounded in absolute terms and
    against the error of the plain PyTorch bf16 composition of the same model
    (MIOpen / hipBLASLt / ATen ops), i.e. the HIP kernels must be as exact
    as bf16 PyTorch itself."""
    from distributed_3d_diffusion_pytorch_amd import ops
    from distributed_3d_diffusion_pytorch_amd.models import XUNet, reference_forward_grad
    from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches
    torch.manual_seed(21)
    m = XUNet(H=64, W=64, ch=128).to(DEV)
    with torch.no_grad():
        for p in m.parameters():
            if p.abs().sum() == 0:
                p.normal_(0, 0.02)
    m.compute_dtype = BF
    m.eval()
    img, R, t, K = next(SyntheticBatches(2, 64, DEV, seed=4))
    batch = {"x": img[:, 0], "z": img[:, 1], "logsnr": torch.tensor([[20.0, 2.5], [20.0, -4.0]], device=DEV),
             "R": R, "t": t, "K": K}
    mask = torch.tensor([True, False], device=DEV)
    go = torch.randn(2, 3, 64, 64, device=DEV)
    sd = {n: p.detach().clone().float().requires_grad_(True) for n, p in m.named_parameters()}
    ref = reference_forward_grad(sd, batch, mask)
    (ref * go).sum().backward()
    r2 = lambda a, b: ((a.float() - b).norm() / b.norm().clamp_min(1e-12)).item()  # noqa: E731
    res = {}
    for be in ("hip", "torch"):
        ops.set_backend(be)
        try:
            m.zero_grad(set_to_none=True)
            out = m(batch, cond_mask=mask)
            (out.float() * go).sum().backward()
        finally:
            ops.set_backend(None)
        res[be] = (r2(out, ref), {n: r2(p.grad, sd[n].grad) for n, p in m.named_parameters()
                                  if p.grad is not None and sd[n].grad.norm() > 0})
    (oh, gh), (ot, gt) = res["hip"], res["torch"]
    from distributed_3d_diffusion_pytorch_amd.ops import hip_impl
    assert hip_impl.FALLBACKS == {}, hip_impl.FALLBACKS     # the HIP run never left the native kernels
    odir = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out")
    os.makedirs(odir, exist_ok=True)
    with open(os.path.join(odir, "oracle64_errors.txt"), "w") as f:
        f.write(f"output rel-L2 hip {oh:.4e} torch-bf16 {ot:.4e}\n")
        f.write("hip_relL2 torch_bf16_relL2 parameter\n")
        for n in sorted(gh, key=lambda k: -gh[k]):
            f.write(f"{gh[n]:.4e} {gt.get(n, float('nan')):.4e} {n}\n")
    assert len(gh) == len(list(m.parameters()))
    assert oh < 2e-2 and oh < 1.5 * ot + 2e-3, (oh, ot)
    hv, tv = sorted(gh.values()), sorted(gt.values())
    med_h, med_t = hv[len(hv) // 2], tv[len(tv) // 2]
    assert hv[-1] < 0.12, max(gh.items(), key=lambda kv: kv[1])
    assert med_h < 1.5 * med_t + 5e-3, (med_h, med_t)


def test_sync_check_mode(H):
    """D3D_SYNC_CHECK debug mode: every native launch is synchronised and
    recorded; results are unchanged."""
    torch.manual_seed(3)
    x = torch.randn(2, 16, 16, 128, device=DEV).to(BF)
    w = torch.randn(128, 128, 3, 3, device=DEV) / 34
    ref = H.conv3x3(x, w, None)
    H.set_sync_check(True)
    try:
        y = H.conv3x3(x, w, None)
        g = H.group_norm(y, torch.ones(128, device=DEV), torch.zeros(128, device=DEV), 32, 1e-5, True)
    finally:
        H.set_sync_check(False)
    assert torch.equal(y, ref) and torch.isfinite(g.float()).all()
    names = H.recent_launches()
    assert "conv" in names and "gn_apply2" in names, names


@pytest.mark.parametrize("N,L,C", [(4, 256, 256), (8, 64, 512), (2, 64, 128)])
def test_linear_residual_fused_gn_stats(H, no_gn_img, N, L, C):
    """Attention-output epilogue (residual + scale) emitting the consuming
    GroupNorm's partial statistics == the statistics pass (GN+SiLU and
    GN-FiLM), and the output itself == the plain epilogue."""
    torch.manual_seed(17)
    x = torch.randn(N, L, C, device=DEV).to(BF)
    w = torch.randn(C, C, device=DEV) / math.sqrt(C)
    b = torch.randn(C, device=DEV) * 0.2
    r = torch.randn(N, L, C, device=DEV).to(BF)
    y = H.linear(x, w, b, r, 1 / math.sqrt(2), gn_groups=32)
    y0 = H.linear(x, w, b, r, 1 / math.sqrt(2))
    assert torch.equal(y, y0)
    assert hasattr(y, "_d3d_gnpart")
    Hh = int(math.isqrt(L))
    y4 = H.carry_gn_stats(y, y.reshape(N, Hh, Hh, C))
    plain = y4.detach().clone()
    gam = torch.rand(C, device=DEV) + 0.5
    bet = torch.randn(C, device=DEV) * 0.1
    a1 = H.group_norm(y4, gam, bet, 32, 1e-5, True)
    r1 = H.group_norm(plain, gam, bet, 32, 1e-5, True)
    assert rel(a1, r1) < 1e-2, rel(a1, r1)
    ss = (torch.randn(N, Hh, Hh, 2 * C, device=DEV) * 0.5).to(BF)
    a2 = H.gn_film(y4, gam, bet, ss, 32, 1e-5, 0.0, False, 0)
    r2 = H.gn_film(plain, gam, bet, ss, 32, 1e-5, 0.0, False, 0)
    assert rel(a2, r2) < 1e-2, rel(a2, r2)


@pytest.mark.parametrize("graph", [False, True])
def test_fused_update_matches_separate(graph, monkeypatch):
    """Adam fused with the bf16 operand repack (adam_update_all: tile kernel
    for the packed weights, range kernel for the rest, pack_all for casts /
    slices) == Adam over the flat buffer + the separate batched repack:
    parameters, moments, and the forward through the repacked operands."""
    from distributed_3d_diffusion_pytorch_amd.config import make_config
    from distributed_3d_diffusion_pytorch_amd.engine import Trainer
    from distributed_3d_diffusion_pytorch_amd.engine import optim as O, graphs as Gm
    from distributed_3d_diffusion_pytorch_amd.parallel import DistContext
    from distributed_3d_diffusion_pytorch_amd.data import SyntheticBatches
    ctx = DistContext(device=torch.device("cuda", 0))
    data = SyntheticBatches(4, 32, "cuda", seed=6)
    batches = [next(data) for _ in range(3)]

    def run(fused):
        monkeypatch.setattr(O, "FUSED_UPDATE", fused)
        monkeypatch.setattr(Gm, "_FUSED_UPDATE", fused)
        cfg = make_config(None, {"model.H": 32, "model.W": 32, "model.dropout": 0.0, "data.imgsize": 32,
                                 "global_batch": 4, "data.synthetic": True, "log_every": 0, "ckpt_every": 0,
                                 "graph": graph, "optim.warmup_examples": 0, "optim.lr": 1e-3})
        tr = Trainer(cfg, ctx)
        for b in batches:
            tr.train_step(*b)
        tr.sync()
        img, R, t, K = batches[0]
        batch = {"x": img[:, 0], "z": img[:, 1], "logsnr": torch.full((4, 2), 1.5, device=DEV), "R": R, "t": t,
                 "K": K}
        with torch.no_grad():
            y = tr.model(batch, cond_mask=torch.ones(4, dtype=torch.bool, device=DEV)).float()
        out = (tr.flat.data.clone(), tr.optim.exp_avg_sq.clone(), y)
        from distributed_3d_diffusion_pytorch_amd.ops import hip_impl
        hip_impl.set_device_seed(None)
        return out

    a, b = run(False), run(True)
    for u, w in zip(a, b):
        d = (u - w).abs().max().item()
        assert d <= 1e-6 * max(1.0, u.abs().max().item()), d


@pytest.mark.parametrize("R", [32, 128, 200])
def test_logsnr_mlp(H, R):
    """K10: fused posenc + Linear-SiLU-Linear (csrc/mlp.hip) vs the fp32 torch
    composition, forward and all four parameter gradients (sink off)."""
    torch.manual_seed(0)
    E = 1024
    logsnr = (torch.rand(R // 2, 2, device=DEV) * 50 - 25)      # includes clipped values
    w1 = torch.randn(E, E, device=DEV) / 32
    b1 = torch.randn(E, device=DEV) * 0.1
    w2 = torch.randn(E, E, device=DEV) / 32
    b2 = torch.randn(E, device=DEV) * 0.1
    go = torch.randn(R, E, device=DEV)
    ph = [leaf(t) for t in (w1, b1, w2, b2)]
    pr = [leaf(t) for t in (w1, b1, w2, b2)]
    yh = H.logsnr_mlp(logsnr, *ph)
    yr = T.logsnr_mlp(logsnr, *pr)
    assert H.FALLBACKS.get(f"logsnr_mlp: E={E}") is None
    yh.backward(go)
    yr.backward(go)
    assert yh.shape == yr.shape == (R, E)
    # fp32 throughout; the posenc arguments reach 2e4 rad, where one ulp of the
    # device vs host exp() of a frequency moves sin/cos by ~1e-3
    assert rel(yh, yr) < 1e-2
    for a, b in zip(ph, pr):
        assert rel(a.grad, b.grad) < 1e-2


@pytest.mark.parametrize("rescale", [0, 128])
def test_ray_conditioning_prep(H, rescale):
    """One-launch conditioning prep (inverse intrinsics, mask, origin posenc;
    rays.hip cond_prep_k) + direction image == the torch composition."""
    from distributed_3d_diffusion_pytorch_amd import ops
    torch.manual_seed(3)
    B, Hh, W = 5, 32, 32
    A = torch.randn(B, 2, 3, 3, device=DEV)
    R = torch.linalg.qr(A)[0].contiguous()
    t = torch.randn(B, 2, 3, device=DEV) * 2
    K = torch.tensor([[60.0, 0.0, 16.0], [0.0, 58.0, 15.5], [0.0, 0.0, 1.0]], device=DEV).repeat(B, 1, 1)
    K[:, 0, 0] += torch.rand(B, device=DEV) * 5
    mask = torch.tensor([True, False, True, True, False], device=DEV)
    dh, oh = H.ray_conditioning(R, t, K, Hh, W, mask, rescale)
    dr = T.ray_posenc_dir(R, t, K, Hh, W, mask, rescale)
    orr = T.ray_origin_pe(t, mask)
    assert oh.shape == orr.shape == (2 * B, 93)
    assert (oh - orr).abs().max().item() < 1e-5
    assert dh.shape == dr.shape == (2 * B, Hh, W, 64)
    assert rel(dh, dr) < 1e-2
    assert dh[..., 51:].abs().max().item() == 0.0


def test_kernels_bitwise_under_coresidency():
    """Race screen: the dense-layer GEMM, convs, weight
    gradients, attention and GroupNorm kernels give bit-identical results
    alone and while another HIP stream keeps LDS-heavy kernels (the per-pixel
    weight gradients of the side stream) resident on the same CUs
    (tools/stress_concurrent.py; a missing LDS-read retirement in the GEMM
    produced wrong outputs only in this situation)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import stress_concurrent as S
    side = torch.cuda.Stream()
    noise = S.noise_setup("wgrad1x1")
    bad = []
    for name, f in S.cases():
        ref = f().clone()
        torch.cuda.synchronize()
        for i in range(6):
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                noise()
            for _ in range(i % 3):
                torch.empty(1, device=DEV).zero_()
            o = f()
            torch.cuda.current_stream().wait_stream(side)
            torch.cuda.synchronize()
            if not torch.equal(o, ref):
                bad.append(name)
                break
    assert not bad, bad


def test_conv_operands_beyond_2gib(H):
    """Large-operand path (128x128 images at one micro-batch of 128): a 3x3
    conv whose input exceeds the kernels' 32-bit buffer offsets runs as
    image chunks at full speed (d3d_conv2), and the weight gradient over a
    > 1 GiB input stays on the descriptor-rebased fast kernels; both against
    the fp32 torch composition."""
    torch.manual_seed(0)
    N, Hh, IC, OC = 132, 128, 512, 64                  # input 2.2 GB bf16
    x = (torch.randn(N, Hh, Hh, IC, device=DEV) * 0.5).to(BF)
    w = torch.randn(OC, IC, 3, 3, device=DEV) * 0.02
    b = torch.randn(OC, device=DEV) * 0.1
    y = H.conv3x3(x, w, b)
    for sl in (slice(0, 3), slice(125, 132)):          # both chunks
        ref = F.conv2d(x[sl].permute(0, 3, 1, 2).float(), w, b, padding=1).permute(0, 2, 3, 1)
        assert rel(y[sl], ref) < 1e-2, rel(y[sl], ref)
    del y
    # weight gradient over a 1.07 GB input (128 channels, 256 frames of 128x128)
    N2, C2 = 256, 128
    x2 = (torch.randn(N2, Hh, Hh, C2, device=DEV) * 0.5).to(BF)
    g2 = (torch.randn(N2, Hh, Hh, C2, device=DEV) * 0.5).to(BF)
    dW, db = H._wgrad(g2, x2, C2, C2, N2, Hh, Hh, Hh, Hh, 1, 9, want_bias=True)
    ref = torch.zeros(C2, C2, 3, 3, device=DEV)
    for s in range(0, N2, 32):
        ref += torch.nn.grad.conv2d_weight(x2[s:s + 32].permute(0, 3, 1, 2).float(), (C2, C2, 3, 3),
                                           g2[s:s + 32].permute(0, 3, 1, 2).float(), padding=1)
    assert rel(dW.reshape(C2, C2, 3, 3), ref) < 1e-3, rel(dW.reshape(C2, C2, 3, 3), ref)
    rb = g2.float().sum((0, 1, 2))
    assert (db - rb).abs().max().item() <= 1e-3 * rb.abs().max().item() + 1e-2


def test_colsum_jobs_batched(H):
    """Batched column sums (reduce.hip colsum_jobs_k): 20 jobs of mixed row
    counts / widths (two launches, one output accumulated twice across
    them) against torch sums; interleaved pairs split into two outputs."""
    torch.manual_seed(7)
    specs, refs, outs = [], [], []
    shared0 = torch.randn(256, device=DEV)
    shared1 = torch.randn(256, device=DEV)
    base0, base1 = shared0.clone(), shared1.clone()
    acc0, acc1 = torch.zeros(256, device=DEV), torch.zeros(256, device=DEV)
    for i in range(20):
        R, C = (32, 256) if i % 3 else (256, 512 if i % 2 else 128)
        x = torch.randn(R, 2 * C, device=DEV)
        if i in (3, 17):            # two jobs accumulate into one shared output pair (C = 256)
            x = torch.randn(R, 512, device=DEV)
            o0, o1 = shared0, shared1
            acc0 += x[:, 0::2].sum(0)
            acc1 += x[:, 1::2].sum(0)
            specs.append(H._ColJob(x.data_ptr(), o0.data_ptr(), o1.data_ptr(), R, 512, 1, 0))
            outs.append(x)
            continue
        o0 = torch.full((C,), 5.0, device=DEV)
        o1 = torch.full((C,), 5.0, device=DEV)
        specs.append(H._ColJob(x.data_ptr(), o0.data_ptr(), o1.data_ptr(), R, 2 * C, 0, 0))
        refs.append((o0, o1, x[:, 0::2].sum(0), x[:, 1::2].sum(0)))
        outs.append(x)
    H.colsum_group_run(specs)
    torch.cuda.synchronize()
    for o0, o1, r0, r1 in refs:
        assert torch.allclose(o0, r0, rtol=1e-5, atol=1e-4)
        assert torch.allclose(o1, r1, rtol=1e-5, atol=1e-4)
    assert torch.allclose(shared0, base0 + acc0, rtol=1e-5, atol=1e-4)
    assert torch.allclose(shared1, base1 + acc1, rtol=1e-5, atol=1e-4)
