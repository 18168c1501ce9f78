"""Winograd F(2,3) band conv (droid_conv_wino_f16, csrc/conv_kernels.hip:
conv_wino_kernel) and the two-workgroups-per-CU direct tile (conv_band2_kernel,
the default for the plain 3x3 convs at W = 64) against the fp32 conv of the
same fp16 operands (the reference runs these convs through cuDNN under
autocast: droid_net.py:84-103, modules/gru.py:19-32)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from gpu_util import host

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _ref(xs, w, bias=None, bb=None):
    xin = torch.cat([x.float() for x in xs], -1).permute(0, 3, 1, 2)
    y = F.conv2d(xin, w.half().float(), bias, padding=1)
    if bb is not None:
        y = y + bb[:, :, None, None]
    return y.permute(0, 2, 3, 1)


@pytest.mark.parametrize("B,H,splits,cout,act", [(3, 8, [128], 128, 1), (2, 4, [128, 96, 64], 256, 0),
                                                  (1, 48, [128], 384, 0), (2, 12, [64, 8], 128, 1)])
def test_wino_act_matches_fp32_conv(B, H, splits, cout, act, ab_backends):
    """EPI_ACT (bias, optional ReLU) at W = 64: partial channel chunks (96, 8),
    several sources, one-tile images (H = 4), several output tiles; the error
    bound is the fp16 class (an fp16 ulp of each transformed operand + the fp16
    output rounding) and within 3x of the direct conv's own error."""
    droid_backends = ab_backends   # the Winograd tile ships in the A/B build only
    from droid_mi355x.fused import pack_conv, pack_conv_wino
    W = 64
    g = torch.Generator(device=DEV).manual_seed(31 + H)
    xs = [torch.randn((B, H, W, c), generator=g, device=DEV).half() for c in splits]
    cin = sum(splits)
    w = torch.randn((cout, cin, 3, 3), generator=g, device=DEV) / (cin * 9) ** 0.5
    bias = torch.randn(cout, generator=g, device=DEV)
    srcs = [(x, 0, c) for x, c in zip(xs, splits)]
    out = torch.full((B, H, W, cout), float("nan"), dtype=torch.float16, device=DEV)
    droid_backends.conv_wino_f16(srcs, pack_conv_wino(w, splits), cout, bias=bias, act=act, out=out)
    ref = _ref(xs, w, bias)
    if act:
        ref = torch.relu(ref)
    err = (out.float() - ref).abs().max().item()
    assert np.isfinite(err) and err < 6e-3, err
    # the direct conv (at W = 64 an EPI_ACT conv runs on the two-workgroups-per-CU
    # tile, conv_band2_kernel): the fp16 output rounding is its only error
    direct = torch.empty_like(out)
    droid_backends.conv_nhwc_f16(srcs, pack_conv(w, splits), cout, 3, bias=bias, act=act, out=direct)
    derr = (direct.float() - ref).abs().max().item()
    assert derr < 4e-3, derr
    assert err < 3 * derr + 1e-3, (err, derr)
    # bias-free mean error: no systematic offset from the transform
    assert abs((out.float() - ref).mean().item()) < 1e-4


def test_wino_image_edges_and_zero_rows(ab_backends):
    """x = -1 / x = 64 neighbours and the rows above / below each image are zero:
    a delta input at every edge position reproduces the clipped kernel exactly."""
    droid_backends = ab_backends   # the Winograd tile ships in the A/B build only
    from droid_mi355x.fused import pack_conv_wino
    B, H, W, C = 2, 8, 64, 64
    x = torch.zeros((B, H, W, C), dtype=torch.float16, device=DEV)
    for (b, y, xx) in [(0, 0, 0), (0, 0, 63), (0, 7, 0), (1, 7, 63), (1, 3, 31), (1, 4, 32), (0, 3, 1), (1, 0, 62)]:
        x[b, y, xx, 5] = 1.0
    w = torch.zeros((128, C, 3, 3), device=DEV)
    w[:, 5] = torch.arange(1, 10, device=DEV, dtype=torch.float32).view(3, 3) / 16   # exact in fp16
    w[:, 5] *= torch.linspace(0.5, 1.0, 128, device=DEV).view(128, 1, 1)
    out = torch.empty((B, H, W, 128), dtype=torch.float16, device=DEV)
    droid_backends.conv_wino_f16([(x, 0, C)], pack_conv_wino(w, [C]), 128, act=0, out=out)
    ref = _ref([x], w)
    np.testing.assert_allclose(host(out.float()), host(ref), atol=2e-3, rtol=2e-3)
    # nothing leaks across images or tile rows: pixels with no input in their 3x3 window are exactly 0
    mask = F.max_pool2d(x[..., 5].float().unsqueeze(1), 3, 1, 1).squeeze(1) == 0
    assert (out.float()[mask] == 0).all()


@pytest.mark.parametrize("B,H", [(3, 8), (2, 48)])
def test_wino_gru_pre_epilogues(B, H, ab_backends):
    """z|r and q gates with the per-source-frame term (EPI_GRU_ZR / EPI_GRU_Q on
    the Winograd tile) vs torch fp32 over the full 448-channel input, at the
    bounds of the direct band kernel's own test (test_gpu_fused.py::test_conv_gru_pre_epilogues)."""
    droid_backends = ab_backends   # the Winograd tile ships in the A/B build only
    from droid_backends import EPI_GRU_Q, EPI_GRU_ZR
    from droid_mi355x.fused import pack_conv_wino
    W = 64
    g = torch.Generator(device=DEV).manual_seed(17)
    mk = lambda n, c: torch.randn((n, H, W, c), generator=g, device=DEV).half()
    F_ = 2
    idx = torch.tensor([1, 0, 1, 0][:B], dtype=torch.int64, device=DEV)
    inp_f = mk(F_, 128)
    h = torch.tanh(mk(B, 128).float()).half()
    cf, ff = mk(B, 128), mk(B, 64)
    xs = [h, inp_f[idx].contiguous(), cf, ff]
    wzr = torch.randn((256, 448, 3, 3), generator=g, device=DEV) / (448 * 9) ** 0.5
    wq = torch.randn((128, 448, 3, 3), generator=g, device=DEV) / (448 * 9) ** 0.5
    bzr, bq = torch.randn(256, generator=g, device=DEV), torch.randn(128, generator=g, device=DEV)
    bbzr, bbq = torch.randn((B, 256), generator=g, device=DEV), torch.randn((B, 128), generator=g, device=DEV)
    keep = lambda w: torch.cat([w[:, :128], w[:, 256:]], 1)
    pre = torch.empty((F_, H, W, 384), dtype=torch.float16, device=DEV)
    droid_backends.conv_wino_f16([(inp_f, 0, 128)], pack_conv_wino(torch.cat([wzr[:, 128:256], wq[:, 128:256]]),
                                                                   [128]), 384, act=0, out=pre)
    z = torch.empty((B, H, W, 128), dtype=torch.float16, device=DEV)
    rn = torch.empty_like(z)
    droid_backends.conv_wino_f16([(h, 0, 128), (cf, 0, 128), (ff, 0, 64)], pack_conv_wino(keep(wzr), [128, 128, 64]),
                                 256, bzr, bbzr, epi=EPI_GRU_ZR, pre=pre, pre_idx=idx, pre_coff=0, h=h, zout=z,
                                 rnet=rn)
    gates = torch.sigmoid(_ref(xs, wzr, bzr, bbzr))
    np.testing.assert_allclose(host(z.float()), host(gates[..., :128]), atol=3e-3)
    np.testing.assert_allclose(host(rn.float()), host(gates[..., 128:] * h.float()), atol=3e-3)
    hn = torch.empty_like(z)
    droid_backends.conv_wino_f16([(rn, 0, 128), (cf, 0, 128), (ff, 0, 64)], pack_conv_wino(keep(wq), [128, 128, 64]),
                                 128, bq, bbq, epi=EPI_GRU_Q, pre=pre, pre_idx=idx, pre_coff=256, h=h, z=z, out=hn)
    q = torch.tanh(_ref([rn] + xs[1:], wq, bq, bbq))
    ref = (1 - z.float()) * h.float() + z.float() * q
    np.testing.assert_allclose(host(hn.float()), host(ref), atol=4e-3)


def test_wino_rejects_unsupported_shape(ab_backends):
    """W != 64 -> DROID_UNSUPPORTED raised (the caller runs the direct conv)."""
    droid_backends = ab_backends   # the Winograd tile ships in the A/B build only
    from droid_mi355x.fused import pack_conv_wino
    x = torch.zeros((1, 8, 32, 128), dtype=torch.float16, device=DEV)
    out = torch.empty_like(x)
    with pytest.raises(RuntimeError):
        droid_backends.conv_wino_f16([(x, 0, 128)], pack_conv_wino(torch.zeros((128, 128, 3, 3), device=DEV), [128]),
                                     128, act=1, out=out)


@pytest.mark.parametrize("B,H,splits", [(3, 8, [128]), (2, 12, [96, 64])])
def test_conv64_matches_fp32_conv(B, H, splits):
    """flow_encoder[2]'s shape (64 output channels, the 384x64 band tile at W = 64)
    vs the fp32 conv of the same fp16 operands: the fp16 output rounding is its
    only error.  (A 64-channel two-workgroups-per-CU tile measured 1.116 vs
    1.104 ms at C3 and was left out.)"""
    import droid_backends
    from droid_mi355x.fused import pack_conv
    W, cout = 64, 64
    g = torch.Generator(device=DEV).manual_seed(5 + H)
    xs = [torch.randn((B, H, W, c), generator=g, device=DEV).half() for c in splits]
    cin = sum(splits)
    w = torch.randn((cout, cin, 3, 3), generator=g, device=DEV) / (cin * 9) ** 0.5
    bias = torch.randn(cout, generator=g, device=DEV)
    out = torch.full((B, H, W, cout), float("nan"), dtype=torch.float16, device=DEV)
    droid_backends.conv_nhwc_f16([(x, 0, c) for x, c in zip(xs, splits)], pack_conv(w, splits), cout, 3, bias=bias,
                                 act=1, out=out)
    ref = torch.relu(_ref(xs, w, bias))
    np.testing.assert_allclose(host(out.float()), host(ref), atol=4e-3, rtol=1e-3)


@pytest.mark.parametrize("B,H,splits", [(3, 8, [128]), (2, 12, [96, 64]), (64, 48, [128]), (1, 24, [64])])
def test_conv64_two_tap_stages_bitwise(B, H, splits, ab_backends):
    """The 64-channel band tile's two-tap stages (the product's: 5 barriers per
    chunk, two tap blocks of weights per stage) sum the same products in the same
    order as its one-tap stages (A/B build, droid_conv_set_pair(0)): bitwise the
    same outputs, single- and multi-source, partial chunks, one-chunk inputs."""
    import ctypes
    import droid_backends
    from droid_mi355x.fused import pack_conv
    W, cout = 64, 64
    g = torch.Generator(device=DEV).manual_seed(7 + H)
    xs = [torch.randn((B, H, W, c), generator=g, device=DEV).half() for c in splits]
    cin = sum(splits)
    w = torch.randn((cout, cin, 3, 3), generator=g, device=DEV) / (cin * 9) ** 0.5
    bias = torch.randn(cout, generator=g, device=DEV)
    srcs = [(x, 0, c) for x, c in zip(xs, splits)]
    out = droid_backends.conv_nhwc_f16(srcs, pack_conv(w, splits), cout, 3, bias=bias, act=1,
                                       out=torch.empty((B, H, W, cout), dtype=torch.float16, device=DEV))
    set_pair = ab_backends.lib.droid_conv_set_pair
    set_pair.argtypes, set_pair.restype = [ctypes.c_int], ctypes.c_int
    prev = set_pair(0)
    try:
        one = ab_backends.conv_nhwc_f16(srcs, pack_conv(w, splits), cout, 3, bias=bias, act=1,
                                        out=torch.empty_like(out))
    finally:
        set_pair(prev)
    assert torch.equal(out, one)


@pytest.mark.parametrize("B,H,cstride,off,bias", [(3, 8, 128, 0, True), (2, 48, 136, 8, True), (5, 4, 128, 0, False),
                                                  (256, 48, 128, 0, True)])
def test_eta_conv_matches_fp32_conv(B, H, cstride, off, bias):
    """GraphAgg's eta head shape (3x3 128 -> 1, droid_net.py:48-50; eta_conv_kernel,
    the conv_nhwc_f16 path for Cout == 1 at W = 64) vs the fp32 conv of the same
    fp16 operands: image-edge taps zero, a strided / offset source, no bias, the
    C3 frame count; the fp16 output rounding is the only error."""
    import droid_backends
    from droid_mi355x.fused import pack_conv
    W = 64
    g = torch.Generator(device=DEV).manual_seed(B + H)
    xb = torch.randn((B, H, W, cstride), generator=g, device=DEV).half()
    x = xb[..., off:off + 128]
    w = torch.randn((1, 128, 3, 3), generator=g, device=DEV) / 34.0
    b = torch.randn(1, generator=g, device=DEV) if bias else None
    out = torch.full((B, H, W, 1), float("nan"), dtype=torch.float16, device=DEV)
    droid_backends.conv_nhwc_f16([(xb, off, 128)], pack_conv(w, [128]), 1, 3, bias=b, out=out)
    ref = _ref([x], w, b)
    err = (out.float() - ref).abs()
    assert float(err.max()) <= 2e-3 * max(1.0, float(ref.abs().max())), float(err.max())
    assert torch.equal(out, droid_backends.conv_nhwc_f16([(xb, off, 128)], pack_conv(w, [128]), 1, 3, bias=b,
                                                         out=torch.empty_like(out)))


def test_corr_lookup_ce0_cooperative_gather_deterministic():
    """The fused lookup's cooperative gather (csrc/corr_kernels.hip, DROID_CE0_COOP)
    parks each pixel's coordinates in LDS between its issue and bilinear steps:
    at E = 300 edges of 48x64 (4,608 tiles, each CU walking ~18 of them through
    both in-flight slots) three launches are bitwise equal and equal to the
    bit-exact oracle-pinned lookup followed by the 1x1 conv in fp32."""
    import droid_backends
    from droid_mi355x.corr import CorrBlock
    E, H, W = 300, 48, 64
    rng = np.random.default_rng(31)
    f1 = torch.from_numpy(rng.normal(size=(1, E, 128, H, W)).astype(np.float16)).to(DEV)
    f2 = torch.from_numpy(rng.normal(size=(1, E, 128, H, W)).astype(np.float16)).to(DEV)
    cbt = CorrBlock(f1, f2, tiled=True)
    coords = (np.stack(np.meshgrid(np.arange(W), np.arange(H)), -1)[None, None]
              + rng.normal(0, 6, (1, E, H, W, 2))).astype(np.float32)
    c = torch.from_numpy(coords).to(DEV).view(E, H, W, 2).contiguous()
    g = torch.Generator(device=DEV).manual_seed(32)
    w224 = torch.zeros((128, 224), device=DEV)
    w224[:, :196] = torch.randn((128, 196), generator=g, device=DEV) / 14.0
    w224 = w224.half().contiguous()
    b = torch.randn(128, generator=g, device=DEV) * 0.1
    with torch.no_grad():
        outs = [droid_backends.corr_lookup_ce0(cbt.corr_pyramid, c, w224, b, tiled_shapes=cbt.level_shapes)
                for _ in range(3)]
        for o in outs[1:]:
            assert torch.equal(o, outs[0])
        look = cbt(c.view(1, E, H, W, 2))[0].permute(0, 2, 3, 1).float()   # (E,H,W,196), bit-exact lookup
        ref = torch.relu(look @ w224[:, :196].float().t() + b)
    np.testing.assert_allclose(host(outs[0].float()), host(ref), atol=2e-3, rtol=2e-3)


@pytest.mark.parametrize("B,R,C,ldd", [(3, 196, 3072, 200), (2, 128, 3072, None), (2, 3072, 576, None),
                                       (1, 5, 7, 9), (4, 70, 130, 72)])
def test_transpose_f16(B, R, C, ldd):
    """droid_transpose_f16 (the reference-layout drop-in's NCHW <-> NHWC copies):
    bitwise the torch transpose, channels past R zero-padded up to ldd, ragged
    tile edges included."""
    import droid_backends
    g = torch.Generator(device=DEV).manual_seed(R + C)
    src = torch.randn((B, R, C), generator=g, device=DEV).half()
    out = droid_backends.transpose_f16(src, R, C, ldd)
    L = ldd or R
    ref = torch.zeros((B, C, L), dtype=torch.float16, device=DEV)
    ref[..., :R] = src.transpose(1, 2)
    assert torch.equal(out, ref)
