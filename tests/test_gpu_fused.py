"""MFMA implicit-GEMM conv and the fused update operator vs fp32 references."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from fill import det_fill
from gpu_util import host

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.mark.parametrize("ks,splits,cout,B,H,W", [(3, [128, 64], 128, 2, 16, 24), (1, [200], 128, 3, 8, 16),
                                                   (7, [8], 128, 2, 12, 16), (3, [256], 4, 2, 8, 16),
                                                   (3, [128, 128, 128, 64], 256, 1, 16, 16),
                                                   (3, [128], 64, 2, 16, 24), (3, [128], 1, 3, 8, 12),
                                                   (5, [8], 128, 3, 8, 12), (3, [64, 128], 16, 3, 8, 12),
                                                   (3, [64], 128, 3, 8, 12), (5, [128], 128, 2, 12, 20)])
def test_conv_matches_torch(ks, splits, cout, B, H, W):
    import droid_backends
    from droid_mi355x.fused import pack_conv
    g = torch.Generator(device=DEV).manual_seed(5)
    xs = [torch.randn((B, H, W, c), generator=g, device=DEV).half() for c in splits]
    w = (torch.randn((cout, sum(splits), ks, ks), generator=g, device=DEV) / (sum(splits) * ks * ks) ** 0.5)
    bias = torch.randn(cout, generator=g, device=DEV)
    bb = torch.randn((B, cout), generator=g, device=DEV)
    out = torch.empty((B, H, W, cout), dtype=torch.float16, device=DEV)
    droid_backends.conv_nhwc_f16([(x, 0, x.shape[-1]) for x in xs], pack_conv(w, splits), cout, ks, bias=bias,
                                 bbias=bb, act=1, out=out)
    xin = torch.cat([x.float() for x in xs], -1).permute(0, 3, 1, 2)
    ref = F.conv2d(xin, w.half().float(), bias, padding=ks // 2) + bb[:, :, None, None]
    ref = F.relu(ref).permute(0, 2, 3, 1)
    np.testing.assert_allclose(host(out.float()), host(ref), atol=2e-2, rtol=1e-2)


@pytest.mark.parametrize("H,W", [(16, 24), (24, 32)])   # generic kernels / band tiles + fused heads
def test_fused_update_matches_reference_module(H, W):
    from droid_mi355x.fused import FusedUpdateModule
    from droid_mi355x.update import UpdateModule
    E = 6
    m = UpdateModule().to(DEV).eval()
    det_fill(m)
    f = FusedUpdateModule(m)
    g = torch.Generator(device=DEV).manual_seed(9)
    net = torch.tanh(torch.randn((1, E, 128, H, W), generator=g, device=DEV)).half()
    inp = torch.relu(torch.randn((1, E, 128, H, W), generator=g, device=DEV)).half()
    corr = (2 * torch.randn((1, E, 196, H, W), generator=g, device=DEV)).half()
    flow = (4 * torch.randn((1, E, 4, H, W), generator=g, device=DEV)).clamp(-64, 64)
    ii = torch.tensor([0, 0, 1, 2, 2, 3], device=DEV)
    jj = torch.tensor([1, 2, 0, 1, 3, 2], device=DEV)
    with torch.no_grad():
        rn, rd, rw, re, _ = m(net.float(), inp.float(), corr.float(), flow, ii, jj)
        nhwc = lambda t: t[0].permute(0, 2, 3, 1).contiguous()
        c200 = torch.zeros((E, H, W, 200), dtype=torch.float16, device=DEV)
        c200[..., :196] = nhwc(corr)
        uq, inv = torch.unique(ii, return_inverse=True)
        fn, fd, fw, fe = f(nhwc(net), nhwc(inp), c200, flow[0], inv, len(uq))
    np.testing.assert_allclose(host(fn.float()), host(nhwc(rn)), atol=1.5e-2)
    np.testing.assert_allclose(host(fd), host(rd), atol=3e-2 * max(1.0, float(rd.abs().max())))
    np.testing.assert_allclose(host(fw), host(rw), atol=1.5e-2)
    np.testing.assert_allclose(host(fe), host(re), atol=1e-3 + 2e-2 * float(re.abs().max()))


def test_corr_lookup_nhwc_equals_nchw():
    import droid_backends
    from droid_mi355x.corr import CorrBlock
    rng = np.random.default_rng(4)
    E, H, W = 3, 16, 24
    f1 = torch.from_numpy(rng.normal(size=(1, E, 128, H, W)).astype(np.float16)).to(DEV)
    f2 = torch.from_numpy(rng.normal(size=(1, E, 128, H, W)).astype(np.float16)).to(DEV)
    cb = CorrBlock(f1, f2)
    coords = (np.stack(np.meshgrid(np.arange(W), np.arange(H)), -1)[None, None]
              + rng.normal(0, 3, (1, E, H, W, 2))).astype(np.float32)
    c = torch.from_numpy(coords).to(DEV)
    with torch.no_grad():
        a = cb(c)[0].permute(0, 2, 3, 1)
        b = cb.lookup_nhwc(c)
    np.testing.assert_array_equal(host(b[..., :196]).view(np.uint16), host(a.contiguous()).view(np.uint16))
    assert torch.all(b[..., 196:] == 0)


def test_factor_graph_update_fused_path():
    """FactorGraph.update() with the fused operator: finite, and BA parity on its inputs."""
    import droid_backends
    from droid_mi355x import DepthVideo, FactorGraph, UpdateModule, synthetic
    from droid_mi355x.fused import FusedUpdateModule
    from oracle import ba as oba
    rng = np.random.default_rng(33)
    n, H, W = 8, 16, 24
    video = DepthVideo(image_size=(8 * H, 8 * W), buffer=n, device=DEV)
    poses = synthetic.trajectory(n, rng)
    poses, disps = synthetic.perturb(poses, synthetic.smooth_disps(n, H, W, rng), rng)
    video.poses[:n] = torch.from_numpy(poses.astype(np.float32)).to(DEV)
    video.disps[:n] = torch.from_numpy(disps.astype(np.float32)).to(DEV)
    video.intrinsics[:n] = torch.tensor([[H / 1.5, H / 1.5, W / 2, H / 2]] * n, device=DEV)
    video.fmaps[:n] = torch.from_numpy(rng.normal(size=(n, 1, 128, H, W)).astype(np.float16)).to(DEV)
    video.nets[:n] = torch.from_numpy(np.tanh(rng.normal(size=(n, 128, H, W))).astype(np.float16)).to(DEV)
    video.inps[:n] = torch.from_numpy(np.maximum(rng.normal(size=(n, 128, H, W)), 0).astype(np.float16)).to(DEV)
    video.counter.value = n
    m = UpdateModule().to(DEV).eval()
    det_fill(m)
    g = FactorGraph(video, FusedUpdateModule(m), device=DEV)
    g.add_neighborhood_factors(0, n, r=2)
    captured = {}
    orig = droid_backends.ba

    def spy(*a, **k):
        captured["a"] = [x.detach().clone() if isinstance(x, torch.Tensor) else x for x in a]
        return orig(*a, **k)

    droid_backends.ba = spy
    try:
        with torch.no_grad():
            g.update()
            g.update()
    finally:
        droid_backends.ba = orig
    a = captured["a"]
    ref = oba.ba(poses=host(a[0]), disps=host(a[1]), intrinsics=host(a[2]), disps_sens=host(a[3]),
                 targets=host(a[4]), weights=host(a[5]), eta=host(a[6]), ii=host(a[7]), jj=host(a[8]), t0=a[9],
                 t1=a[10], iterations=a[11], lm=a[12], ep=a[13], motion_only=a[14])
    np.testing.assert_allclose(host(video.poses[:n]), ref["poses"][:n], atol=1e-4)
    np.testing.assert_allclose(host(video.disps[:n]), np.maximum(ref["disps"][:n], 1e-3), atol=1e-4)
    assert g.net.shape == (len(g._ii), H, W, 128) and torch.isfinite(g.net.float()).all()


def test_segment_mean_matches_scatter_mean():
    import droid_backends
    from droid_mi355x.fused import edge_segments
    from droid_mi355x.update import scatter_mean
    g = torch.Generator(device=DEV).manual_seed(3)
    E, H, W, C = 9, 8, 12, 128
    src = torch.randn((E, H, W, C), generator=g, device=DEV).half()
    inverse = np.array([2, 0, 2, 1, 0, 2, 3, 3, 0])
    U = 5   # slot 4 has no edges -> zeros (torch_scatter semantics)
    ptr, idx = edge_segments(inverse, U)
    out = droid_backends.segment_mean_f16(src, torch.as_tensor(ptr, device=DEV), torch.as_tensor(idx, device=DEV), U)
    ref = scatter_mean(src.float().view(E, -1), torch.as_tensor(inverse, device=DEV), 0, U).view(U, H, W, C)
    np.testing.assert_allclose(host(out.float()), host(ref), atol=2e-3, rtol=2e-3)
    dptr, didx = edge_segments(torch.as_tensor(inverse, device=DEV), U)
    assert np.array_equal(host(dptr), ptr) and np.array_equal(host(didx), idx)


# shapes that take the LDS-DMA band kernel (3x3, W % 16 == 0, whole-row tiles):
# <256,256> for Cout % 256 == 0 (W | 256, HW % 256 == 0), <384,128> for Cout % 128 == 0
BAND_CASES = [([128, 128, 128, 64], 256, 2, 8, 64),    # z|r-shaped, 256-tile, image rows 0 and H-1 in the tile
              ([128], 256, 3, 16, 32),                 # 256-tile with W = 32 (8 rows per tile)
              ([128, 128, 128, 64], 128, 2, 12, 64),   # q-shaped, 384-tile (6 rows)
              ([128], 128, 1, 48, 64),                 # the update operator's 48x64 maps
              ([96, 64], 128, 2, 24, 32),              # source narrower than its 64-channel chunk
              ([64], 256, 2, 16, 16),                  # 256-tile of 16 rows
              ([128], 64, 2, 12, 64)]                  # flow_encoder[2]-shaped, 384x64 tile


def _conv_ref(xs, w, bias, bb):
    xin = torch.cat([x.float() for x in xs], -1).permute(0, 3, 1, 2)
    return (F.conv2d(xin, w.half().float(), bias, padding=1) + bb[:, :, None, None]).permute(0, 2, 3, 1)


@pytest.mark.parametrize("splits,cout,B,H,W", BAND_CASES)
def test_conv_band_act(splits, cout, B, H, W):
    import droid_backends
    from droid_mi355x.fused import pack_conv
    g = torch.Generator(device=DEV).manual_seed(11)
    xs = [torch.randn((B, H, W, c), generator=g, device=DEV).half() for c in splits]
    w = torch.randn((cout, sum(splits), 3, 3), generator=g, device=DEV) / (sum(splits) * 9) ** 0.5
    bias = torch.randn(cout, generator=g, device=DEV)
    bb = torch.randn((B, cout), generator=g, device=DEV)
    out = torch.empty((B, H, W, cout), dtype=torch.float16, device=DEV)
    droid_backends.conv_nhwc_f16([(x, 0, x.shape[-1]) for x in xs], pack_conv(w, splits), cout, 3, bias=bias,
                                 bbias=bb, act=1, out=out)
    ref = F.relu(_conv_ref(xs, w, bias, bb))
    # fp16 output: |err| <= fp16 rounding of the value + fp32 accumulation-order noise
    np.testing.assert_allclose(host(out.float()), host(ref), atol=1e-2, rtol=1e-2)


@pytest.mark.parametrize("B,H,W", [(2, 8, 64), (2, 12, 64), (1, 16, 32)])
def test_conv_gru_epilogues(B, H, W):
    """z|r (sigmoid, r*h) and q (tanh, (1-z)h + zq) epilogues vs torch fp32 (modules/gru.py:19-32)."""
    import droid_backends
    from droid_backends import EPI_GRU_Q, EPI_GRU_ZR
    from droid_mi355x.fused import pack_conv
    g = torch.Generator(device=DEV).manual_seed(12)
    splits = [128, 128, 128, 64]
    mk = lambda c: torch.randn((B, H, W, c), generator=g, device=DEV).half()
    h = torch.tanh(mk(128).float()).half()
    xs = [h, mk(128), mk(128), mk(64)]
    wzr = torch.randn((256, 448, 3, 3), generator=g, device=DEV) / (448 * 9) ** 0.5
    wq = torch.randn((128, 448, 3, 3), generator=g, device=DEV) / (448 * 9) ** 0.5
    bzr, bq = torch.randn(256, generator=g, device=DEV), torch.randn(128, generator=g, device=DEV)
    bbzr, bbq = torch.randn((B, 256), generator=g, device=DEV), torch.randn((B, 128), generator=g, device=DEV)
    z = torch.empty((B, H, W, 128), dtype=torch.float16, device=DEV)
    rn = torch.empty_like(z)
    droid_backends.conv_nhwc_f16([(x, 0, x.shape[-1]) for x in xs], pack_conv(wzr, splits), 256, 3, bias=bzr,
                                 bbias=bbzr, epi=EPI_GRU_ZR, h=h, zout=z, rnet=rn)
    gates = torch.sigmoid(_conv_ref(xs, wzr, bzr, bbzr))
    np.testing.assert_allclose(host(z.float()), host(gates[..., :128]), atol=2e-3)
    np.testing.assert_allclose(host(rn.float()), host(gates[..., 128:] * h.float()), atol=2e-3)
    hn = torch.empty_like(z)
    xq = [rn] + xs[1:]
    droid_backends.conv_nhwc_f16([(x, 0, x.shape[-1]) for x in xq], pack_conv(wq, splits), 128, 3, bias=bq,
                                 bbias=bbq, epi=EPI_GRU_Q, h=h, z=z, out=hn)
    q = torch.tanh(_conv_ref(xq, wq, bq, bbq))
    ref = (1 - z.float()) * h.float() + z.float() * q
    np.testing.assert_allclose(host(hn.float()), host(ref), atol=3e-3)


@pytest.mark.parametrize("B,H,W", [(2, 8, 64), (3, 16, 32), (2, 32, 16), (1, 48, 64)])
def test_conv_dw_head_fused(B, H, W):
    """relu(conv3x3 128->256) -> block-diagonal conv3x3 256->4 in one launch vs torch fp32."""
    import droid_backends
    from droid_mi355x.fused import pack_conv, pack_head_taps
    g = torch.Generator(device=DEV).manual_seed(13)
    x = torch.randn((B, H, W, 128), generator=g, device=DEV).half()
    w0 = torch.randn((256, 128, 3, 3), generator=g, device=DEV) / (128 * 9) ** 0.5
    b0 = torch.randn(256, generator=g, device=DEV) * 0.1
    head = torch.zeros(4, 256, 3, 3, device=DEV)
    head[0:2, :128] = torch.randn((2, 128, 3, 3), generator=g, device=DEV) / (128 * 9) ** 0.5
    head[2:4, 128:] = torch.randn((2, 128, 3, 3), generator=g, device=DEV) / (128 * 9) ** 0.5
    out = torch.zeros((B, H, W, 4), dtype=torch.float32, device=DEV)
    droid_backends.conv_dw_head_f16([(x, 0, 128)], pack_conv(w0, [128]), b0, pack_head_taps(head), out)
    dw = F.relu(F.conv2d(x.float().permute(0, 3, 1, 2), w0.half().float(), b0, padding=1))
    dw = dw.half().float()   # the hidden map is fp16 (autocast), as in the reference
    ref = F.conv2d(dw, head.half().float(), None, padding=1).permute(0, 2, 3, 1)
    np.testing.assert_allclose(host(out), host(ref), atol=2e-3 * max(1.0, float(ref.abs().max())), rtol=1e-3)
    out2 = torch.zeros_like(out)
    droid_backends.conv_dw_head_f16([(x, 0, 128)], pack_conv(w0, [128]), b0, pack_head_taps(head), out2)
    assert torch.equal(out, out2), "dw/head fusion must be deterministic"


@pytest.mark.parametrize("E,H,W", [(3, 16, 24), (2, 8, 64)])
def test_corr_lookup_ce0_fused(E, H, W):
    """Lookup + corr_encoder[0] in one kernel == bit-exact lookup followed by the
    1x1 conv in fp32 (modules/corr.py:40-50, droid_net.py:84-86)."""
    import droid_backends
    from droid_mi355x.corr import CorrBlock
    rng = np.random.default_rng(21)
    f1 = torch.from_numpy(rng.normal(size=(1, E, 128, H, W)).astype(np.float16)).to(DEV)
    f2 = torch.from_numpy(rng.normal(size=(1, E, 128, H, W)).astype(np.float16)).to(DEV)
    cb = CorrBlock(f1, f2)
    coords = (np.stack(np.meshgrid(np.arange(W), np.arange(H)), -1)[None, None]
              + rng.normal(0, 4, (1, E, H, W, 2))).astype(np.float32)   # windows leave the volume at borders
    c = torch.from_numpy(coords).to(DEV)
    g = torch.Generator(device=DEV).manual_seed(22)
    w = torch.randn((128, 196), generator=g, device=DEV) / 14.0
    b = torch.randn(128, generator=g, device=DEV) * 0.1
    w224 = torch.zeros((128, 224), device=DEV)
    w224[:, :196] = w
    w224 = w224.half().contiguous()
    with torch.no_grad():
        out = droid_backends.corr_lookup_ce0(cb.corr_pyramid, c.view(E, H, W, 2).contiguous(), w224, b)
        look = cb.lookup_nhwc(c)[..., :196].float()
    ref = F.relu(look @ w224[:, :196].float().t() + b)
    np.testing.assert_allclose(host(out.float()), host(ref), atol=2e-3 * max(1.0, float(ref.abs().max())), rtol=2e-3)
    out2 = droid_backends.corr_lookup_ce0(cb.corr_pyramid, c.view(E, H, W, 2).contiguous(), w224, b)
    assert torch.equal(out, out2)


@pytest.mark.parametrize("E,H,W", [(3, 24, 64), (2, 48, 64), (2, 16, 32)])
def test_corr_lookup_ce0_tiled_volume_bitexact(E, H, W):
    """The 8x8-tiled volume (CorrBlock(tiled=True), droid_corr_lookup_ce0_tiled)
    gives bit-identical outputs to the reference row-major layout, including
    levels whose H2 is not a multiple of 8 (padded tile rows) and windows that
    leave the volume; (16, 32) has a W2 = 4 level, so the block stays row-major."""
    import droid_backends
    from droid_mi355x.corr import CorrBlock
    rng = np.random.default_rng(23)
    f1 = torch.from_numpy(rng.normal(size=(1, E, 128, H, W)).astype(np.float16)).to(DEV)
    f2 = torch.from_numpy(rng.normal(size=(1, E, 128, H, W)).astype(np.float16)).to(DEV)
    cb = CorrBlock(f1, f2)
    cbt = CorrBlock(f1, f2, tiled=True)
    assert cbt.tiled == all(w % 8 == 0 for _, w in cbt.level_shapes)
    for a, b in zip(cb.corr_pyramid, cbt.reference_pyramid()):
        assert torch.equal(a, b)
    coords = (np.stack(np.meshgrid(np.arange(W), np.arange(H)), -1)[None, None]
              + rng.normal(0, 6, (1, E, H, W, 2))).astype(np.float32)
    coords[0, 0, :4] = rng.uniform(-12, max(H, W) + 12, (4, W, 2))   # far outside at every level
    c = torch.from_numpy(coords).to(DEV).view(E, H, W, 2).contiguous()
    g = torch.Generator(device=DEV).manual_seed(24)
    w224 = torch.zeros((128, 224), device=DEV)
    w224[:, :196] = torch.randn((128, 196), generator=g, device=DEV) / 14.0
    w224 = w224.half().contiguous()
    b = torch.randn(128, generator=g, device=DEV) * 0.1
    with torch.no_grad():
        ref = droid_backends.corr_lookup_ce0(cb.corr_pyramid, c, w224, b)
        out = droid_backends.corr_lookup_ce0(cbt.corr_pyramid, c, w224, b,
                                             tiled_shapes=cbt.level_shapes if cbt.tiled else None)
        assert torch.equal(out, ref)
        # the generic lookups of a tiled block go through the reference layout
        assert torch.equal(cbt(c.view(1, E, H, W, 2)), cb(c.view(1, E, H, W, 2)))


@pytest.mark.parametrize("E,H,W", [(3, 8, 24), (2, 48, 64), (96, 48, 64), (600, 48, 64)])
def test_gru_global_context(E, H, W):
    """glo = mean_px sigmoid(conv1x1(h) + b) * h (modules/gru.py:24-26) vs torch fp32
    (one workgroup per edge, or several pixel ranges per edge for small graphs)."""
    import droid_backends
    g = torch.Generator(device=DEV).manual_seed(23)
    h = torch.tanh(torch.randn((E, H, W, 128), generator=g, device=DEV)).half()
    w = (torch.randn((128, 128), generator=g, device=DEV) / 11.3).half()
    b = torch.randn(128, generator=g, device=DEV) * 0.1
    out = droid_backends.gru_global_f16(h, w, b)
    hf = h.float().view(E, H * W, 128)
    ref = (torch.sigmoid(hf @ w.float().t() + b) * hf).mean(1)
    np.testing.assert_allclose(host(out), host(ref), atol=1e-4, rtol=1e-3)
    assert torch.equal(out, droid_backends.gru_global_f16(h, w, b))


@pytest.mark.parametrize("E,H,W", [(3, 8, 32), (2048, 48, 64), (5, 4, 16)])
def test_gru_global_ring_depths_bitwise(E, H, W, ab_backends):
    """gru_glo_kernel's tile ring (the product's 3 buffers, three workgroups per
    CU) changes only how many tiles are in flight: bitwise the sums of the
    round-4 ring of 5 and of a ring of 2 (A/B build, droid_glo_set_ring)."""
    import ctypes
    import droid_backends
    g = torch.Generator(device=DEV).manual_seed(29)
    h = torch.tanh(torch.randn((E, H, W, 128), generator=g, device=DEV)).half()
    w = (torch.randn((128, 128), generator=g, device=DEV) / 11.3).half()
    b = torch.randn(128, generator=g, device=DEV) * 0.1
    out = droid_backends.gru_global_f16(h, w, b)
    set_ring = ab_backends.lib.droid_glo_set_ring
    set_ring.argtypes, set_ring.restype = [ctypes.c_int], ctypes.c_int
    prev = set_ring(5)
    try:
        r5 = ab_backends.gru_global_f16(h, w, b)
        set_ring(2)
        r2 = ab_backends.gru_global_f16(h, w, b)
    finally:
        set_ring(prev)
    assert torch.equal(out, r5) and torch.equal(out, r2)


@pytest.mark.parametrize("E,H,W", [(3, 8, 32), (2, 48, 64), (2, 4, 128), (3, 4, 32), (5, 12, 32)])
def test_flow_encoder0(E, H, W):
    """relu(conv7x7(motn.half()) + b) (droid_net.py:88-90 under autocast) vs torch fp32.
    H*W % 256 == 0 runs the 256-pixel tile (flow_enc0_rw_kernel, weights in VGPRs),
    the (3, 4, 32) and (5, 12, 32) shapes the 128-pixel / 8-wave one."""
    import droid_backends
    from droid_mi355x.fused import pack_flow_enc0
    g = torch.Generator(device=DEV).manual_seed(24)
    motn = (8 * torch.randn((E, 4, H, W), generator=g, device=DEV)).clamp(-64, 64)
    w = torch.randn((128, 4, 7, 7), generator=g, device=DEV) / 14.0
    b = torch.randn(128, generator=g, device=DEV) * 0.1
    out = droid_backends.flow_enc0_f16(motn, pack_flow_enc0(w), b)
    ref = F.relu(F.conv2d(motn.half().float(), w.half().float(), b, padding=3)).permute(0, 2, 3, 1)
    np.testing.assert_allclose(host(out.float()), host(ref), atol=2e-3 * max(1.0, float(ref.abs().max())), rtol=2e-3)


@pytest.mark.parametrize("E,H,W", [(3, 8, 32), (2, 48, 64), (2, 4, 128), (3, 16, 16), (300, 48, 64)])
def test_flow_encoder0_resident_weights_bitwise(E, H, W, ab_backends):
    """flow_enc0_rw_kernel (the product's 256-pixel tile: 8 waves, weights in
    VGPRs) multiplies the same operands in the same K order as the round-4
    flow_enc0_kernel (16 waves, weights in LDS; A/B build, droid_fe_set_variant(0)):
    bitwise the same outputs, including a persistent walk over many tiles."""
    import ctypes
    import droid_backends
    from droid_mi355x.fused import pack_flow_enc0
    g = torch.Generator(device=DEV).manual_seed(25 + W)
    motn = (8 * torch.randn((E, 4, H, W), generator=g, device=DEV)).clamp(-64, 64)
    wp = pack_flow_enc0(torch.randn((128, 4, 7, 7), generator=g, device=DEV) / 14.0)
    b = torch.randn(128, generator=g, device=DEV) * 0.1
    out = droid_backends.flow_enc0_f16(motn, wp, b)
    set_v = ab_backends.lib.droid_fe_set_variant
    set_v.argtypes, set_v.restype = [ctypes.c_int], ctypes.c_int
    prev = set_v(0)
    try:
        ref = ab_backends.flow_enc0_f16(motn, wp, b)
    finally:
        set_v(prev)
    assert torch.equal(out, ref)
    assert torch.equal(out, ab_backends.flow_enc0_f16(motn, wp, b))


@pytest.mark.parametrize("noise,H,W,E", [(1.5, 16, 24, 6), (40.0, 16, 24, 6), (1.5, 48, 64, 300), (8.0, 48, 64, 300),
                                         (40.0, 48, 64, 48)])
def test_corr_alt_ce0_matches_volume_path(noise, H, W, E):
    """On-demand correlation (feature pyramid, MFMA) + corr_encoder[0] == the
    volume lookup + corr_encoder[0] up to fp16 rounding of the pooled levels
    (modules/corr.py: CorrBlock vs AltCorrBlock semantics).  Coherent windows /
    incoherent (half, quadrant and pixel fallbacks; at 48x64 with noise 40 for
    the product's pixel-major C and window table on every fallback path); at 48x64 with 300 edges
    every workgroup walks many tiles (the cross-tile pipeline)."""
    import droid_backends
    from droid_mi355x.corr import AltCorrBlock, CorrBlock
    rng = np.random.default_rng(31)
    NF = 4 if E <= 6 else 12
    fm = torch.from_numpy(rng.normal(size=(NF, 128, H, W)).astype(np.float16)).to(DEV)
    if E <= 6:
        ii = np.array([0, 1, 2, 3, 1, 2], np.int64)
        jj = np.array([1, 0, 3, 1, 1, 0], np.int64)
    else:
        ii = rng.integers(0, NF, E).astype(np.int64)
        jj = rng.integers(0, NF, E).astype(np.int64)
    cb = CorrBlock(fm[ii][None], fm[jj][None])
    pyr = [lv.view((-1,) + tuple(lv.shape[2:])) for lv in AltCorrBlock(fm[None]).pyramid]
    grid = np.stack(np.meshgrid(np.arange(W), np.arange(H)), -1)[None].astype(np.float32)
    coords = grid + rng.normal(0, noise, (E, H, W, 2)).astype(np.float32) + 2.0
    c = torch.from_numpy(coords).to(DEV).contiguous()
    g = torch.Generator(device=DEV).manual_seed(32)
    w224 = torch.zeros((128, 224), device=DEV)
    w224[:, :196] = torch.randn((128, 196), generator=g, device=DEV) / 14.0
    w224 = w224.half().contiguous()
    b = torch.randn(128, generator=g, device=DEV) * 0.1
    with torch.no_grad():
        ref = droid_backends.corr_lookup_ce0(cb.corr_pyramid, c, w224, b).float()
        out = droid_backends.corr_alt_ce0(pyr, torch.as_tensor(ii, dtype=torch.int32, device=DEV),
                                          torch.as_tensor(jj, dtype=torch.int32, device=DEV), c, w224, b).float()
    scale = float(ref.abs().max())
    err = (out - ref).abs()
    assert float(err.max()) < 2e-2 * scale, float(err.max()) / scale
    assert float(err.mean()) < 1e-3 * scale, float(err.mean()) / scale
    out2 = droid_backends.corr_alt_ce0(pyr, torch.as_tensor(ii, dtype=torch.int32, device=DEV),
                                       torch.as_tensor(jj, dtype=torch.int32, device=DEV), c, w224, b).float()
    assert torch.equal(out, out2)


@pytest.mark.parametrize("noise,H,W,E,far", [(1.5, 16, 24, 6, 0.0), (40.0, 16, 24, 6, 0.0), (1.5, 48, 64, 300, 0.0),
                                             (8.0, 48, 64, 300, 0.0), (4.0, 48, 64, 200, 0.1), (0.3, 32, 64, 64, 0.0)])
def test_corr_alt2_bitwise_equals_alt1(noise, H, W, E, far, ab_backends):
    """The round-4 corr_alt2_kernel (two 4-wave workgroups per CU, C in place,
    merged level-3/2/1 stage, group fallbacks; A/B variant 4) and its round-5
    pixel-major C layout alone (variant 6) compute every value with the same
    operations in the same order as corr_alt_ce0_kernel: outputs bitwise
    equal.  The product (pixel-major C + row-K lookup tile) is checked against
    them in test_corr_alt2_v3_matches_v2.  far: fraction of pixels thrown
    30-200 px off the map (windows partly or wholly outside, boxes over the
    region -> half / quadrant / pixel groups)."""
    droid_backends = ab_backends   # variants 1, 4 and 6 ship in the A/B build only
    from droid_mi355x.corr import AltCorrBlock
    rng = np.random.default_rng(41)
    NF = 8
    fm = torch.from_numpy(rng.normal(size=(NF, 128, H, W)).astype(np.float16)).to(DEV)
    ii = rng.integers(0, NF, E).astype(np.int32)
    jj = rng.integers(0, NF, E).astype(np.int32)
    pyr = [lv.view((-1,) + tuple(lv.shape[2:])) for lv in AltCorrBlock(fm[None]).pyramid]
    grid = np.stack(np.meshgrid(np.arange(W), np.arange(H)), -1)[None].astype(np.float32)
    coords = grid + rng.normal(0, noise, (E, H, W, 2)).astype(np.float32) + rng.uniform(-3, 3, (E, 1, 1, 2)).astype(np.float32)
    if far:
        m = rng.random((E, H, W)) < far
        coords[m] += rng.uniform(30, 200, (int(m.sum()), 2)).astype(np.float32) * rng.choice([-1, 1], (int(m.sum()), 2))
    c = torch.from_numpy(coords).to(DEV).contiguous()
    g = torch.Generator(device=DEV).manual_seed(42)
    w224 = torch.zeros((128, 224), device=DEV)
    w224[:, :196] = torch.randn((128, 196), generator=g, device=DEV) / 14.0
    w224 = w224.half().contiguous()
    b = torch.randn(128, generator=g, device=DEV) * 0.1
    f1, f2 = torch.as_tensor(ii, device=DEV), torch.as_tensor(jj, device=DEV)
    try:
        droid_backends.alt_set_variant(1)
        ref = droid_backends.corr_alt_ce0(pyr, f1, f2, c, w224, b)
        droid_backends.alt_set_variant(4)
        out = droid_backends.corr_alt_ce0(pyr, f1, f2, c, w224, b)
        droid_backends.alt_set_variant(6)
        out6 = droid_backends.corr_alt_ce0(pyr, f1, f2, c, w224, b)
    finally:
        droid_backends.alt_set_variant(2)
    torch.cuda.synchronize()
    diff = (out.float() - ref.float()).abs()
    assert torch.equal(out, ref), (float(diff.max()), int((diff > 0).sum()))
    assert torch.equal(out6, ref)


@pytest.mark.parametrize("noise,H,W,E,far", [(1.5, 16, 24, 6, 0.0), (40.0, 16, 24, 6, 0.0), (1.5, 48, 64, 300, 0.0),
                                             (4.0, 48, 64, 200, 0.1), (0.3, 32, 64, 64, 0.0)])
def test_corr_alt2_v3_matches_v2(noise, H, W, E, far, ab_backends):
    """The product corr_alt2_kernel (round 5: C pixel-major with 8-B C
    stores and dword window-row reads, lookup tile in the k = 8 iy + ix order with the encoder
    weights permuted to match) and the A/B kernels that share its lookup-tile
    order - V3 (box blocks split over the waves) and the row-K tile alone
    (variant 5) - are bitwise equal to each other: their C values and bilinear
    windows are the round-4 V2 values (variant 4), and only corr_encoder[0]'s
    fp32 summation order differs from V2 (a permuted K), so against V2 the fp16
    outputs agree to a few ulps and are mostly identical; every fallback
    (incoherent, off-map coordinates) included."""
    import droid_backends as product
    droid_backends = ab_backends   # variants 3, 4 and 5 ship in the A/B build only
    from droid_mi355x.corr import AltCorrBlock
    rng = np.random.default_rng(43)
    NF = 8
    fm = torch.from_numpy(rng.normal(size=(NF, 128, H, W)).astype(np.float16)).to(DEV)
    ii = rng.integers(0, NF, E).astype(np.int32)
    jj = rng.integers(0, NF, E).astype(np.int32)
    pyr = [lv.view((-1,) + tuple(lv.shape[2:])) for lv in AltCorrBlock(fm[None]).pyramid]
    grid = np.stack(np.meshgrid(np.arange(W), np.arange(H)), -1)[None].astype(np.float32)
    coords = grid + rng.normal(0, noise, (E, H, W, 2)).astype(np.float32) + rng.uniform(-3, 3, (E, 1, 1, 2)).astype(np.float32)
    if far:
        m = rng.random((E, H, W)) < far
        coords[m] += rng.uniform(30, 200, (int(m.sum()), 2)).astype(np.float32) * rng.choice([-1, 1], (int(m.sum()), 2))
    c = torch.from_numpy(coords).to(DEV).contiguous()
    g = torch.Generator(device=DEV).manual_seed(44)
    w224 = torch.zeros((128, 224), device=DEV)
    w224[:, :196] = torch.randn((128, 196), generator=g, device=DEV) / 14.0
    w224 = w224.half().contiguous()
    b = torch.randn(128, generator=g, device=DEV) * 0.1
    f1, f2 = torch.as_tensor(ii, device=DEV), torch.as_tensor(jj, device=DEV)
    try:
        droid_backends.alt_set_variant(4)
        ref = droid_backends.corr_alt_ce0(pyr, f1, f2, c, w224, b)
        droid_backends.alt_set_variant(3)
        out = droid_backends.corr_alt_ce0(pyr, f1, f2, c, w224, b)
        out2 = droid_backends.corr_alt_ce0(pyr, f1, f2, c, w224, b)
        droid_backends.alt_set_variant(5)
        out5 = droid_backends.corr_alt_ce0(pyr, f1, f2, c, w224, b)
    finally:
        droid_backends.alt_set_variant(2)
    prod = product.corr_alt_ce0(pyr, f1, f2, c, w224, b)   # the product library's corr_alt2_kernel
    torch.cuda.synchronize()
    assert torch.equal(out, out2)                      # deterministic
    assert torch.equal(out5, out)
    assert torch.equal(prod, out)
    assert bool(torch.isfinite(out.float()).all())
    scale = float(ref.float().abs().max())
    diff = (out.float() - ref.float()).abs()
    assert float(diff.max()) <= 4e-3 * scale, float(diff.max()) / scale
    assert float((diff == 0).float().mean()) > 0.9


def test_corr_alt_ordered_walk_is_bitwise_the_same(ab_backends):
    """droid_corr_alt_ce0_ordered: walking the tiles in an edge permutation
    (edges grouped by target frame, FactorGraph._alt_order) changes only which
    workgroup computes a tile - the outputs are the same bytes in the same
    places, for the default and the V3 kernel."""
    import droid_backends
    from droid_mi355x.corr import AltCorrBlock
    rng = np.random.default_rng(45)
    NF, H, W, E = 8, 48, 64, 40
    fm = torch.from_numpy(rng.normal(size=(NF, 128, H, W)).astype(np.float16)).to(DEV)
    ii = rng.integers(0, NF, E).astype(np.int32)
    jj = rng.integers(0, NF, E).astype(np.int32)
    pyr = [lv.view((-1,) + tuple(lv.shape[2:])) for lv in AltCorrBlock(fm[None]).pyramid]
    grid = np.stack(np.meshgrid(np.arange(W), np.arange(H)), -1)[None].astype(np.float32)
    coords = grid + rng.normal(0, 2.0, (E, H, W, 2)).astype(np.float32)
    c = torch.from_numpy(coords).to(DEV).contiguous()
    g = torch.Generator(device=DEV).manual_seed(46)
    w224 = torch.zeros((128, 224), device=DEV)
    w224[:, :196] = torch.randn((128, 196), generator=g, device=DEV) / 14.0
    w224 = w224.half().contiguous()
    b = torch.randn(128, generator=g, device=DEV) * 0.1
    f1, f2 = torch.as_tensor(ii, device=DEV), torch.as_tensor(jj, device=DEV)
    order = torch.as_tensor(np.argsort(jj, kind="stable").astype(np.int32), device=DEV)
    try:
        ref = droid_backends.corr_alt_ce0(pyr, f1, f2, c, w224, b)   # the product library
        out = droid_backends.corr_alt_ce0(pyr, f1, f2, c, w224, b, order=order)
        torch.cuda.synchronize()
        assert torch.equal(out, ref)
        for v in (2, 3):   # the A/B library: the product kernel and V3
            ab_backends.alt_set_variant(v)
            ref_v = ab_backends.corr_alt_ce0(pyr, f1, f2, c, w224, b)
            out = ab_backends.corr_alt_ce0(pyr, f1, f2, c, w224, b, order=order)
            torch.cuda.synchronize()
            ab_backends.alt_set_variant(2)
            assert torch.equal(out, ref_v), v
        # the XCD chunking of the walk (droid_alt_set_chunk, a testing hook):
        # interleaved, one edge, a chunk that does not divide the 40 edges, more than all of them
        for chunk in (0, 1, 3, 64):
            ab_backends.alt_set_chunk(chunk)
            for o in (None, order):
                out = ab_backends.corr_alt_ce0(pyr, f1, f2, c, w224, b, order=o)
                torch.cuda.synchronize()
                assert torch.equal(out, ref), (chunk, o is None)
    finally:
        ab_backends.alt_set_variant(2)
        ab_backends.alt_set_chunk(0)


def test_corr_volume_slot_pool_matches_fresh_block():
    """The tiled CorrBlock as a slot pool (frontend edge edits: append, drop,
    append again, pool growth) looked up in place through
    droid_corr_lookup_ce0_tiled_slots == a block built fresh from the final edge
    list (bitwise), and corr_pyramid gathers the same volumes in edge order."""
    import droid_backends
    from droid_mi355x.corr import CorrBlock
    rng = np.random.default_rng(51)
    H, W, NF = 16, 64, 6   # every level's width a multiple of 8 (the tiled layout)
    fm = torch.from_numpy(rng.normal(size=(NF, 128, H, W)).astype(np.float16)).to(DEV)
    frames = (fm.half() / 4.0).permute(0, 2, 3, 1).contiguous()
    def block(ii, jj):
        return CorrBlock.from_frames(frames, torch.as_tensor(ii, dtype=torch.int32, device=DEV),
                                     torch.as_tensor(jj, dtype=torch.int32, device=DEV), tiled=True)
    e1 = (np.array([0, 1, 2, 3, 4]), np.array([1, 2, 3, 4, 5]))
    e2 = (np.array([5, 0, 2]), np.array([0, 3, 5]))
    e3 = (np.array([1, 4, 3, 0, 2, 5, 1]), np.array([0, 2, 1, 5, 4, 3, 5]))
    cb = block(*e1).cat(block(*e2))                      # 8 edges (pool grows from 5)
    keep = np.array([1, 0, 1, 1, 0, 1, 0, 1], bool)
    cb.select(keep)                                      # 5 edges, 3 free rows
    cb.cat(block(*e3))                                   # 12 edges: fills 3 rows, grows
    ii = np.concatenate([e1[0], e2[0]])[keep].tolist() + e3[0].tolist()
    jj = np.concatenate([e1[1], e2[1]])[keep].tolist() + e3[1].tolist()
    ref = block(np.array(ii), np.array(jj))
    assert cb.slot_tensor() is not None and cb.num_edges() == len(ii)
    for a, b in zip(cb.corr_pyramid, ref.corr_pyramid):
        assert torch.equal(a, b)
    E = len(ii)
    grid = np.stack(np.meshgrid(np.arange(W), np.arange(H)), -1)[None].astype(np.float32)
    c = torch.from_numpy(grid + rng.normal(0, 2.0, (E, H, W, 2)).astype(np.float32)).to(DEV).contiguous()
    g = torch.Generator(device=DEV).manual_seed(52)
    w224 = torch.zeros((128, 224), device=DEV)
    w224[:, :196] = torch.randn((128, 196), generator=g, device=DEV) / 14.0
    w224 = w224.half().contiguous()
    b = torch.randn(128, generator=g, device=DEV) * 0.1
    out = droid_backends.corr_lookup_ce0(cb.pool_levels(), c, w224, b, tiled_shapes=cb.level_shapes,
                                         slots=cb.slot_tensor())
    exp = droid_backends.corr_lookup_ce0(ref.corr_pyramid, c, w224, b, tiled_shapes=ref.level_shapes)
    assert torch.equal(out, exp)


def test_head_finish_and_eta_damping_match_torch():
    """droid_head_finish_f32 (bias, sigmoid, coords1 + delta, BA-layout rows)
    and droid_eta_damping_f32 (0.01 softplus, the damping store, 0.2 d + EP
    gather) against the torch ops they replace (factor_graph.py:209-221)."""
    import droid_backends
    g = torch.Generator(device=DEV).manual_seed(61)
    E, H, W = 5, 8, 16
    head = torch.randn((E, H, W, 4), generator=g, device=DEV) * 3
    b = torch.randn(4, generator=g, device=DEV)
    base = torch.randn((E, H, W, 2), generator=g, device=DEV) * 20
    tba = torch.full((E + 3, 2, H, W), 7.0, device=DEV)
    wba = torch.full((E + 3, 2, H, W), 7.0, device=DEV)
    t, w = droid_backends.head_finish(head, b, base, tba, wba, 3)
    hb = head + b
    t_ref = base + hb[..., 0:2]
    w_ref = torch.sigmoid(hb[..., 2:4])
    assert torch.equal(t, t_ref)
    np.testing.assert_allclose(host(w), host(w_ref), rtol=0, atol=1e-7)
    assert torch.equal(tba[3:], t.permute(0, 3, 1, 2)) and torch.equal(wba[3:], w.permute(0, 3, 1, 2))
    assert bool((tba[:3] == 7.0).all()) and bool((wba[:3] == 7.0).all())
    d0, _ = droid_backends.head_finish(head, b)
    assert torch.equal(d0, hb[..., 0:2].contiguous())
    # eta / damping: frames 2, 5, 6 have eta rows 1, 0, -, frame 9 has row 2
    U, N = 3, 12
    er = (torch.randn((U, H, W, 1), generator=g, device=DEV) * 8).half()
    er[0, 0, 0, 0] = 30.0   # softplus' linear branch
    state = torch.rand((N, H, W), generator=g, device=DEV)
    frames = torch.tensor([2, 5, 6, 9], dtype=torch.int32, device=DEV)
    rows = torch.tensor([1, 0, -1, 2], dtype=torch.int32, device=DEV)
    ref_state = state.clone()
    eta = 0.01 * torch.nn.functional.softplus(er.float()).view(U, H, W)
    ref_state[torch.tensor([2, 5, 9], device=DEV)] = eta[torch.tensor([1, 0, 2], device=DEV)]
    ref_out = 0.2 * ref_state[frames.long()] + 1e-7
    out = droid_backends.eta_damping(er, rows, frames, state, 1e-7)
    np.testing.assert_allclose(host(state), host(ref_state), rtol=2e-7, atol=0)
    np.testing.assert_allclose(host(out), host(ref_out), rtol=2e-7, atol=0)


def test_factor_graph_update_pyramid_corr():
    """FactorGraph(corr_impl="pyramid"): no volume; update() finite and its BA
    matches the oracle on the inputs it hands over."""
    import droid_backends
    from droid_mi355x import DepthVideo, FactorGraph, UpdateModule, synthetic
    from droid_mi355x.fused import FusedUpdateModule
    from oracle import ba as oba
    rng = np.random.default_rng(34)
    n, H, W = 8, 16, 24
    video = DepthVideo(image_size=(8 * H, 8 * W), buffer=n, device=DEV)
    poses = synthetic.trajectory(n, rng)
    poses, disps = synthetic.perturb(poses, synthetic.smooth_disps(n, H, W, rng), rng)
    video.poses[:n] = torch.from_numpy(poses.astype(np.float32)).to(DEV)
    video.disps[:n] = torch.from_numpy(disps.astype(np.float32)).to(DEV)
    video.intrinsics[:n] = torch.tensor([[H / 1.5, H / 1.5, W / 2, H / 2]] * n, device=DEV)
    video.fmaps[:n] = torch.from_numpy(rng.normal(size=(n, 1, 128, H, W)).astype(np.float16)).to(DEV)
    video.nets[:n] = torch.from_numpy(np.tanh(rng.normal(size=(n, 128, H, W))).astype(np.float16)).to(DEV)
    video.inps[:n] = torch.from_numpy(np.maximum(rng.normal(size=(n, 128, H, W)), 0).astype(np.float16)).to(DEV)
    video.counter.value = n
    m = UpdateModule().to(DEV).eval()
    det_fill(m)
    g = FactorGraph(video, FusedUpdateModule(m), device=DEV, corr_impl="pyramid")
    g.add_neighborhood_factors(0, n, r=2)
    assert g.corr is None
    captured = {}
    orig = droid_backends.ba

    def spy(*a, **k):
        captured["a"] = [x.detach().clone() if isinstance(x, torch.Tensor) else x for x in a]
        return orig(*a, **k)

    droid_backends.ba = spy
    try:
        with torch.no_grad():
            g.update()
            g.update()
    finally:
        droid_backends.ba = orig
    a = captured["a"]
    ref = oba.ba(poses=host(a[0]), disps=host(a[1]), intrinsics=host(a[2]), disps_sens=host(a[3]),
                 targets=host(a[4]), weights=host(a[5]), eta=host(a[6]), ii=host(a[7]), jj=host(a[8]), t0=a[9],
                 t1=a[10], iterations=a[11], lm=a[12], ep=a[13], motion_only=a[14])
    np.testing.assert_allclose(host(video.poses[:n]), ref["poses"][:n], atol=1e-4)
    np.testing.assert_allclose(host(video.disps[:n]), np.maximum(ref["disps"][:n], 1e-3), atol=1e-4)
    assert torch.isfinite(g.net.float()).all()


@pytest.mark.parametrize("corr_impl", ["volume", "pyramid"])
def test_factor_graph_update_stereo(corr_impl):
    """Stereo video: neighbourhood edges skip |i-j| <= 1
    (factor_graph.py:334-337), one (i, i) edge per frame correlates against the
    right image (fmaps[i, 1], factor_graph.py:112-114) and BA uses the fixed
    stereo baseline for it.  Checks the stereo volume rows, then BA parity on the
    inputs update() hands over (as test_factor_graph_update_fused_path)."""
    import droid_backends
    from droid_mi355x import DepthVideo, FactorGraph, UpdateModule, synthetic
    from droid_mi355x.fused import FusedUpdateModule
    from oracle import ba as oba
    rng = np.random.default_rng(35)
    n, H, W = 8, 16, 24
    video = DepthVideo(image_size=(8 * H, 8 * W), buffer=n, stereo=True, device=DEV)
    poses = synthetic.trajectory(n, rng)
    poses, disps = synthetic.perturb(poses, synthetic.smooth_disps(n, H, W, rng), rng)
    video.poses[:n] = torch.from_numpy(poses.astype(np.float32)).to(DEV)
    video.disps[:n] = torch.from_numpy(disps.astype(np.float32)).to(DEV)
    video.intrinsics[:n] = torch.tensor([[H / 1.5, H / 1.5, W / 2, H / 2]] * n, device=DEV)
    fm = rng.normal(size=(n, 2, 128, H, W)).astype(np.float16)
    video.fmaps[:n] = torch.from_numpy(fm).to(DEV)
    video.nets[:n] = torch.from_numpy(np.tanh(rng.normal(size=(n, 128, H, W))).astype(np.float16)).to(DEV)
    video.inps[:n] = torch.from_numpy(np.maximum(rng.normal(size=(n, 128, H, W)), 0).astype(np.float16)).to(DEV)
    video.counter.value = n
    m = UpdateModule().to(DEV).eval()
    det_fill(m)
    g = FactorGraph(video, FusedUpdateModule(m), device=DEV, corr_impl=corr_impl)
    g.add_neighborhood_factors(0, n, r=3)
    d = np.abs(g._ii - g._jj)
    assert d.min() == 2 and d.max() == 3
    g.add_factors(np.arange(n), np.arange(n))
    stereo = np.nonzero(g._ii == g._jj)[0]
    assert len(stereo) == n
    if corr_impl == "volume":
        lv0 = g.corr.reference_pyramid()[0]
        for k in stereo[:3]:
            i = int(g._ii[k])
            f1 = fm[i, 0].astype(np.float32).reshape(128, -1) / 4
            f2 = fm[i, 1].astype(np.float32).reshape(128, -1) / 4
            want = (f1.T @ f2).reshape(H, W, H, W)
            np.testing.assert_allclose(host(lv0[k]).astype(np.float32), want, atol=2e-2, rtol=1e-2)
    captured = {}
    orig = droid_backends.ba

    def spy(*a, **k):
        captured["a"] = [x.detach().clone() if isinstance(x, torch.Tensor) else x for x in a]
        return orig(*a, **k)

    droid_backends.ba = spy
    try:
        with torch.no_grad():
            g.update()
            g.update()
    finally:
        droid_backends.ba = orig
    a = captured["a"]
    assert (host(a[7]) == host(a[8])).sum() == n   # stereo edges reach BA
    ref = oba.ba(poses=host(a[0]), disps=host(a[1]), intrinsics=host(a[2]), disps_sens=host(a[3]),
                 targets=host(a[4]), weights=host(a[5]), eta=host(a[6]), ii=host(a[7]), jj=host(a[8]), t0=a[9],
                 t1=a[10], iterations=a[11], lm=a[12], ep=a[13], motion_only=a[14])
    np.testing.assert_allclose(host(video.poses[:n]), ref["poses"][:n], atol=1e-4)
    np.testing.assert_allclose(host(video.disps[:n]), np.maximum(ref["disps"][:n], 1e-3), atol=1e-4)
    assert torch.isfinite(g.net.float()).all()


@pytest.mark.parametrize("B,H,W", [(3, 12, 64), (2, 24, 32), (4, 48, 16)])
def test_conv_gru_pre_epilogues(B, H, W):
    """Gates with the inp term factored per source frame (droid_conv_gru_pre_f16):
    conv3x3 over (h | corr | flow) + pre[pre_idx[b]] with pre = conv3x3(inp_frames)
    vs torch fp32 over the full 448-channel input (modules/gru.py:19-32)."""
    import droid_backends
    from droid_backends import EPI_GRU_Q, EPI_GRU_ZR
    from droid_mi355x.fused import pack_conv
    g = torch.Generator(device=DEV).manual_seed(13)
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
    droid_backends.conv_nhwc_f16([(inp_f, 0, 128)], pack_conv(torch.cat([wzr[:, 128:256], wq[:, 128:256]]), [128]),
                                 384, 3, out=pre)
    z = torch.empty((B, H, W, 128), dtype=torch.float16, device=DEV)
    rn = torch.empty_like(z)
    droid_backends.conv_gru_pre_f16([(h, 0, 128), (cf, 0, 128), (ff, 0, 64)], pack_conv(keep(wzr), [128, 128, 64]),
                                    256, bzr, bbzr, EPI_GRU_ZR, pre, idx, 0, h=h, zout=z, rnet=rn)
    gates = torch.sigmoid(_conv_ref(xs, wzr, bzr, bbzr))
    np.testing.assert_allclose(host(z.float()), host(gates[..., :128]), atol=3e-3)
    np.testing.assert_allclose(host(rn.float()), host(gates[..., 128:] * h.float()), atol=3e-3)
    hn = torch.empty_like(z)
    droid_backends.conv_gru_pre_f16([(rn, 0, 128), (cf, 0, 128), (ff, 0, 64)], pack_conv(keep(wq), [128, 128, 64]),
                                    128, bq, bbq, EPI_GRU_Q, pre, idx, 256, h=h, z=z, out=hn)
    q = torch.tanh(_conv_ref([rn] + xs[1:], wq, bq, bbq))
    ref = (1 - z.float()) * h.float() + z.float() * q
    np.testing.assert_allclose(host(hn.float()), host(ref), atol=4e-3)


def test_conv_gru_pre_rejects_unsupported_shape():
    """No band tile for the shape -> DROID_UNSUPPORTED raised, nothing silently computed."""
    import droid_backends
    from droid_backends import EPI_GRU_ZR
    from droid_mi355x.fused import pack_conv
    B, H, W = 1, 10, 24
    t = lambda c: torch.zeros((B, H, W, c), dtype=torch.float16, device=DEV)
    h, cf, ff = t(128), t(128), t(64)
    pre = torch.zeros((1, H, W, 384), dtype=torch.float16, device=DEV)
    w = pack_conv(torch.zeros((256, 320, 3, 3), device=DEV), [128, 128, 64])
    with pytest.raises(RuntimeError):
        droid_backends.conv_gru_pre_f16([(h, 0, 128), (cf, 0, 128), (ff, 0, 64)], w, 256, None, None, EPI_GRU_ZR,
                                        pre, torch.zeros(1, dtype=torch.int64, device=DEV), 0, h=h, zout=t(128),
                                        rnet=t(128))


def test_fused_update_inp_frames_matches_per_edge_inp():
    """FusedUpdateModule with per-frame context features (gate inp term per
    source frame) vs the same module on per-edge inp copies, and vs UpdateModule."""
    from droid_mi355x.fused import FusedUpdateModule
    from droid_mi355x.update import UpdateModule
    E, H, W = 6, 24, 32
    m = UpdateModule().to(DEV).eval()
    det_fill(m)
    f = FusedUpdateModule(m)
    g = torch.Generator(device=DEV).manual_seed(19)
    ii = torch.tensor([0, 0, 1, 2, 2, 3], device=DEV)
    jj = torch.tensor([1, 2, 0, 1, 3, 2], device=DEV)
    uq, inv = torch.unique(ii, return_inverse=True)
    net = torch.tanh(torch.randn((1, E, 128, H, W), generator=g, device=DEV)).half()
    inpf = torch.relu(torch.randn((len(uq), 128, H, W), generator=g, device=DEV)).half()
    inp = inpf[inv].unsqueeze(0)
    corr = (2 * torch.randn((1, E, 196, H, W), generator=g, device=DEV)).half()
    flow = (4 * torch.randn((1, E, 4, H, W), generator=g, device=DEV)).clamp(-64, 64)
    nhwc = lambda t: t[0].permute(0, 2, 3, 1).contiguous()
    c200 = torch.zeros((E, H, W, 200), dtype=torch.float16, device=DEV)
    c200[..., :196] = nhwc(corr)
    with torch.no_grad():
        rn, rd, rw, re, _ = m(net.float(), inp.float(), corr.float(), flow, ii, jj)
        an, ad, aw, ae = f(nhwc(net), nhwc(inp), c200, flow[0], inv, len(uq))
        bn, bd, bw, be = f(nhwc(net), None, c200, flow[0], inv, len(uq),
                           inp_frames=inpf.permute(0, 2, 3, 1).contiguous())
    np.testing.assert_allclose(host(bn.float()), host(an.float()), atol=4e-3)
    np.testing.assert_allclose(host(bd), host(ad), atol=1e-2 * max(1.0, float(ad.abs().max())))
    np.testing.assert_allclose(host(bw), host(aw), atol=4e-3)
    np.testing.assert_allclose(host(bn.float()), host(nhwc(rn)), atol=1.5e-2)
    np.testing.assert_allclose(host(bd), host(rd), atol=3e-2 * max(1.0, float(rd.abs().max())))
    np.testing.assert_allclose(host(bw), host(rw), atol=1.5e-2)
    np.testing.assert_allclose(host(be), host(re), atol=1e-3 + 2e-2 * float(re.abs().max()))


def test_fused_update_matches_reference_module_48x64():
    """The bench's feature-map size (48x64, the per-frame gate term, fused
    delta/weight heads) with E=10 edges over 4 source frames.  At this edge
    count the gate convs run on the two-workgroup tile (conv_band2_kernel);
    the 8-wave W=64 band tiles the C3 bench takes are covered at 192-256
    edges by tests/test_gpu_conv_c3.py."""
    from droid_mi355x.fused import FusedUpdateModule
    from droid_mi355x.update import UpdateModule
    E, H, W = 10, 48, 64
    m = UpdateModule().to(DEV).eval()
    det_fill(m)
    f = FusedUpdateModule(m)
    g = torch.Generator(device=DEV).manual_seed(19)
    net = torch.tanh(torch.randn((1, E, 128, H, W), generator=g, device=DEV)).half()
    ii = torch.tensor([0, 0, 0, 1, 1, 2, 2, 2, 3, 3], device=DEV)
    jj = torch.tensor([1, 2, 3, 0, 2, 0, 1, 3, 1, 2], device=DEV)
    inp_f = torch.relu(torch.randn((4, 128, H, W), generator=g, device=DEV)).half()
    inp = inp_f[ii][None]                                   # every edge of a frame shares its context
    corr = (2 * torch.randn((1, E, 196, H, W), generator=g, device=DEV)).half()
    flow = (4 * torch.randn((1, E, 4, H, W), generator=g, device=DEV)).clamp(-64, 64)
    with torch.no_grad():
        rn, rd, rw, re, _ = m(net.float(), inp.float(), corr.float(), flow, ii, jj)
        nhwc = lambda t: t[0].permute(0, 2, 3, 1).contiguous()
        c200 = torch.zeros((E, H, W, 200), dtype=torch.float16, device=DEV)
        c200[..., :196] = nhwc(corr)
        uq, inv = torch.unique(ii, return_inverse=True)
        from droid_mi355x.fused import edge_segments
        ptr, idx = edge_segments(inv.cpu().numpy(), len(uq))
        segs = (torch.as_tensor(ptr, device=DEV), torch.as_tensor(idx, device=DEV))
        inp_frames = nhwc(inp).index_select(0, torch.as_tensor(idx[ptr[:-1]], device=DEV))
        fn, fd, fw, fe = f(nhwc(net), nhwc(inp), c200, flow[0], inv, len(uq), segments=segs, inp_frames=inp_frames)
    np.testing.assert_allclose(host(fn.float()), host(nhwc(rn)), atol=1.5e-2)
    np.testing.assert_allclose(host(fd), host(rd), atol=3e-2 * max(1.0, float(rd.abs().max())))
    np.testing.assert_allclose(host(fw), host(rw), atol=1.5e-2)
    np.testing.assert_allclose(host(fe), host(re), atol=1e-3 + 2e-2 * float(re.abs().max()))


@pytest.mark.parametrize("H,W,E,per_frame", [(16, 24, 6, False), (48, 64, 10, False), (48, 64, 10, True)])
def test_reference_layout_module_matches_update_module(H, W, E, per_frame):
    """ReferenceLayoutUpdateModule is called exactly as the reference's
    factor_graph.update() calls UpdateModule (factor_graph.py:207-208: NCHW
    state, materialised 196-channel lookup, 5 outputs incl. upmask) and agrees
    with the torch module (pinned to the reference by update_module.npz) at
    fp16 tolerance; without ii it returns the 3-output form.  per_frame: inp
    gathered per source frame as the reference's graph builds it
    (factor_graph.py:118), so the drop-in takes the factored gates (checked,
    not assumed - random per-edge inp takes the per-edge gates)."""
    from droid_mi355x.fused import ReferenceLayoutUpdateModule
    from droid_mi355x.update import UpdateModule
    m = UpdateModule().to(DEV).eval()
    det_fill(m)
    d = ReferenceLayoutUpdateModule(m)
    g = torch.Generator(device=DEV).manual_seed(19)
    net = torch.tanh(torch.randn((1, E, 128, H, W), generator=g, device=DEV)).half()
    inp = torch.relu(torch.randn((1, E, 128, H, W), generator=g, device=DEV)).half()
    corr = (2 * torch.randn((1, E, 196, H, W), generator=g, device=DEV)).half()
    flow = (4 * torch.randn((1, E, 4, H, W), generator=g, device=DEV)).clamp(-64, 64)
    ii = torch.tensor([0, 0, 1, 2, 2, 3, 1, 3, 0, 2][:E], device=DEV)
    jj = torch.tensor([1, 2, 0, 1, 3, 2, 3, 0, 3, 0][:E], device=DEV)
    if per_frame:
        inp = inp[:, :4][:, ii].contiguous()
    with torch.no_grad():
        rn, rd, rw, re, ru = m(net.float(), inp.float(), corr.float(), flow, ii, jj)
        dn, dd, dw, de, du = d(net, inp, corr, flow, ii, jj)
        n3 = d(net, inp, corr, flow)
        with torch.autocast("cuda", enabled=True):   # the reference's update() runs under autocast
            an, ad, aw, ae, au = d(net, inp, corr, flow, ii, jj)
    assert dn.shape == rn.shape and dn.dtype == torch.float16
    assert dd.shape == rd.shape and dw.shape == rw.shape and de.shape == re.shape and du.shape == ru.shape
    np.testing.assert_allclose(host(dn.float()), host(rn), atol=1.5e-2)
    np.testing.assert_allclose(host(dd), host(rd), atol=3e-2 * max(1.0, float(rd.abs().max())))
    np.testing.assert_allclose(host(dw), host(rw), atol=1.5e-2)
    np.testing.assert_allclose(host(de), host(re), atol=1e-3 + 2e-2 * float(re.abs().max()))
    np.testing.assert_allclose(host(du.float()), host(ru), atol=3e-2 * max(1.0, float(ru.abs().max())))
    if not per_frame:
        assert len(n3) == 3 and torch.equal(n3[0], dn) and torch.equal(n3[1], dd) and torch.equal(n3[2], dw)
    assert (d._frames[3] is not None) == per_frame
    for a, b in ((an, dn), (ad, dd), (aw, dw), (ae, de), (au, du)):
        assert torch.equal(a, b)


def test_reference_layout_module_under_inference_mode():
    """The drop-in called under torch.inference_mode() (inference tensors carry
    no version counter, so its channels-last caches must not read one) gives
    the no_grad results bit for bit, on repeated calls and with the net it
    returned passed back."""
    from droid_mi355x.fused import FusedUpdateModule, ReferenceLayoutUpdateModule
    from droid_mi355x.update import UpdateModule
    E, H, W = 10, 48, 64
    m = UpdateModule().to(DEV).eval()
    det_fill(m)
    g = torch.Generator(device=DEV).manual_seed(41)
    net = torch.tanh(torch.randn((1, E, 128, H, W), generator=g, device=DEV)).half()
    inp = torch.relu(torch.randn((1, E, 128, H, W), generator=g, device=DEV)).half()
    corr = (2 * torch.randn((1, E, 196, H, W), generator=g, device=DEV)).half()
    flow = (4 * torch.randn((1, E, 4, H, W), generator=g, device=DEV)).clamp(-64, 64)
    ii = torch.tensor([0, 0, 1, 2, 2, 3, 1, 3, 0, 2], device=DEV)
    jj = torch.tensor([1, 2, 0, 1, 3, 2, 3, 0, 3, 0], device=DEV)
    with torch.no_grad():
        d = ReferenceLayoutUpdateModule(m)
        a1 = d(net, inp, corr, flow, ii, jj)
        a2 = d(a1[0], inp, corr, flow, ii, jj)
    with torch.inference_mode():
        d = ReferenceLayoutUpdateModule(m)
        ni, ip, co, fl = net.clone(), inp.clone(), corr.clone(), flow.clone()
        assert ni.is_inference()
        b1 = d(ni, ip, co, fl, ii, jj)
        checked = d._frames
        b2 = d(b1[0], ip, co, fl, ii, jj)
        # the per-frame content check ran once for this (inp, ii) pair
        assert d._frames is checked
        # the per-frame gate term on an inference inp_frames tensor
        f = FusedUpdateModule(m)
        nhwc = lambda t: t[0].permute(0, 2, 3, 1).contiguous()
        c200 = torch.zeros((E, H, W, 200), dtype=torch.float16, device=DEV)
        c200[..., :196] = nhwc(co)
        uq, inv = torch.unique(ii, return_inverse=True)
        inpf = nhwc(ip)[:4]
        r1 = f(nhwc(ni), None, c200, fl[0], inv, len(uq), inp_frames=inpf)
        r2 = f(nhwc(ni), None, c200, fl[0], inv, len(uq), inp_frames=inpf)
    for x, y in list(zip(a1, b1)) + list(zip(a2, b2)) + list(zip(r1, r2)):
        assert torch.equal(x, y)


def test_reference_layout_module_inference_refill_in_place():
    """under inference_mode the per-frame check is keyed on a
    content fingerprint, not identity alone.  Refilling the same inp buffer
    in place so that edges of one frame no longer share their rows must turn
    the factored gates off: the result equals a fresh module's on the new
    contents."""
    from droid_mi355x.fused import ReferenceLayoutUpdateModule
    from droid_mi355x.update import UpdateModule
    E, H, W = 6, 48, 64
    m = UpdateModule().to(DEV).eval()
    det_fill(m)
    g = torch.Generator(device=DEV).manual_seed(45)
    net = torch.tanh(torch.randn((1, E, 128, H, W), generator=g, device=DEV)).half()
    frm = torch.relu(torch.randn((3, 128, H, W), generator=g, device=DEV)).half()
    corr = (2 * torch.randn((1, E, 196, H, W), generator=g, device=DEV)).half()
    flow = (4 * torch.randn((1, E, 4, H, W), generator=g, device=DEV)).clamp(-64, 64)
    ii = torch.tensor([0, 0, 1, 1, 2, 2], device=DEV)
    jj = torch.tensor([1, 2, 0, 2, 0, 1], device=DEV)
    other = torch.relu(torch.randn((1, E, 128, H, W), generator=g, device=DEV)).half()   # per edge: no sharing
    with torch.inference_mode():
        d = ReferenceLayoutUpdateModule(m)
        inp = frm[ii].unsqueeze(0).contiguous()
        d(net, inp, corr, flow, ii, jj)
        assert d._frames[3] is not None          # shared rows: the factored gates
        inp.copy_(other)
        a = d(net, inp, corr, flow, ii, jj)
        assert d._frames[3] is None              # refilled: per-edge gates
        b = ReferenceLayoutUpdateModule(m)(net, other.clone(), corr, flow, ii, jj)
    for x, y in zip(a, b):
        assert torch.equal(x, y)


def test_fused_pre_term_follows_in_place_refill():
    """The per-frame gate-term cache is keyed on the inp_frames tensor's version:
    refilling the same buffer in place gives the term of the new contents."""
    from droid_mi355x.fused import FusedUpdateModule
    from droid_mi355x.update import UpdateModule
    E, H, W = 6, 48, 64
    m = UpdateModule().to(DEV).eval()
    det_fill(m)
    f = FusedUpdateModule(m)
    g = torch.Generator(device=DEV).manual_seed(43)
    net = torch.tanh(torch.randn((E, H, W, 128), generator=g, device=DEV)).half()
    c200 = (2 * torch.randn((E, H, W, 200), generator=g, device=DEV)).half()
    flow = (4 * torch.randn((E, 4, H, W), generator=g, device=DEV)).clamp(-64, 64)
    inv = torch.tensor([0, 0, 1, 1, 2, 2], device=DEV)
    buf = torch.relu(torch.randn((3, H, W, 128), generator=g, device=DEV)).half()
    other = torch.relu(torch.randn((3, H, W, 128), generator=g, device=DEV)).half()
    with torch.no_grad():
        f(net, None, c200, flow, inv, 3, inp_frames=buf)
        buf.copy_(other)
        a = f(net, None, c200, flow, inv, 3, inp_frames=buf)
        b = FusedUpdateModule(m)(net, None, c200, flow, inv, 3, inp_frames=other)
    for x, y in zip(a, b):
        assert torch.equal(x, y)


@pytest.mark.parametrize("E,C,H,W", [(3, 196, 48, 64), (2, 196, 16, 24), (5, 100, 8, 16)])
def test_conv1x1_nchw_matches_torch(E, C, H, W):
    """corr_encoder[0] straight from the NCHW lookup (droid_conv1x1_nchw_f16)
    vs torch fp32 (droid_net.py:84-86), and vs the channels-last 1x1 conv the
    fused path runs on the transposed tensor."""
    import droid_backends
    from droid_mi355x.fused import pack_conv
    g = torch.Generator(device=DEV).manual_seed(47)
    src = (2 * torch.randn((E, C, H, W), generator=g, device=DEV)).half()
    w = torch.randn((128, C), generator=g, device=DEV) / C ** 0.5
    b = torch.randn(128, generator=g, device=DEV)
    K = (C + 31) // 32 * 32
    wk = torch.zeros((128, K), device=DEV)
    wk[:, :C] = w
    out = droid_backends.conv1x1_nchw_f16(src, wk.half().contiguous(), b)
    ref = torch.relu(torch.einsum("oc,echw->ehwo", w.half().float(), src.float()) + b)
    np.testing.assert_allclose(host(out.float()), host(ref), atol=2e-2, rtol=1e-2)
    nhwc = torch.zeros((E, H, W, (C + 7) // 8 * 8), dtype=torch.float16, device=DEV)
    nhwc[..., :C] = src.permute(0, 2, 3, 1)
    cl = torch.empty((E, H, W, 128), dtype=torch.float16, device=DEV)
    wp = torch.zeros((128, nhwc.shape[-1], 1, 1), device=DEV)
    wp[:, :C, 0, 0] = w
    droid_backends.conv_nhwc_f16([(nhwc, 0, nhwc.shape[-1])], pack_conv(wp, [nhwc.shape[-1]]), 128, 1, bias=b, act=1,
                                 out=cl)
    assert float((out.float() - cl.float()).abs().max()) < 2e-3


@pytest.mark.parametrize("E,H,W", [(3, 8, 32), (2048, 48, 64), (96, 48, 64)])
def test_gru_global_packed_sum_matches_scalar(E, H, W, ab_backends):
    """gru_glo_kernel's sigmoid sum on packed fp32 (the product) vs the scalar
    form the A/B build keeps (droid_glo_set_pk(0)): the same values up to fp32
    rounding of the exp argument (one fma instead of an add and a multiply), and
    both vs torch fp32."""
    import ctypes
    import droid_backends
    g = torch.Generator(device=DEV).manual_seed(31)
    h = torch.tanh(torch.randn((E, H, W, 128), generator=g, device=DEV)).half()
    w = (torch.randn((128, 128), generator=g, device=DEV) / 11.3).half()
    b = torch.randn(128, generator=g, device=DEV) * 0.1
    out = droid_backends.gru_global_f16(h, w, b)
    set_pk = ab_backends.lib.droid_glo_set_pk
    set_pk.argtypes, set_pk.restype = [ctypes.c_int], ctypes.c_int
    prev = set_pk(1)
    try:
        pk = ab_backends.gru_global_f16(h, w, b)
        set_pk(0)
        scalar = ab_backends.gru_global_f16(h, w, b)
    finally:
        set_pk(prev)
    assert torch.equal(out, pk)
    np.testing.assert_allclose(host(out), host(scalar), atol=1e-7, rtol=1e-5)
    hf = h.float().view(E, H * W, 128)
    ref = (torch.sigmoid(hf @ w.float().t() + b) * hf).mean(1)
    np.testing.assert_allclose(host(out), host(ref), atol=1e-6, rtol=1e-4)
