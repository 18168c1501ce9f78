"""HIP correlation kernels vs the CPU oracle (through the C ABI)."""
import numpy as np
import pytest
import torch

from gpu_util import dev, host
from oracle import corr as oc

pytestmark = pytest.mark.gpu


def _coords(rng, B, H, W, H2, W2, spread=3.0):
    base = np.stack(np.meshgrid(np.arange(W) * W2 / W, np.arange(H) * H2 / H), 0)[None]
    c = base + rng.normal(0, spread, (B, 2, H, W))
    c[:, :, 0, 0] = -50.0            # far out of bounds
    c[:, 0, 0, 1] = W2 - 0.5         # right edge
    c[:, 1, 1, 0] = -0.25            # top edge
    return c.astype(np.float32)


@pytest.mark.parametrize("dtype", [np.float16, np.float32, np.float64])
@pytest.mark.parametrize("r", [3, 1])
def test_corr_index_forward_vs_oracle(dtype, r):
    import droid_backends
    rng = np.random.default_rng(11)
    B, H, W, H2, W2 = 3, 12, 16, 12, 16
    vol = rng.normal(size=(B, H, W, H2, W2)).astype(dtype)
    coords = _coords(rng, B, H, W, H2, W2)
    out, = droid_backends.corr_index_forward(dev(vol), dev(coords), r)
    ref = oc.corr_index_forward(vol, coords, r)
    got = host(out)
    assert got.dtype == ref.dtype and got.shape == ref.shape
    if dtype == np.float16:
        np.testing.assert_array_equal(got.view(np.uint16), ref.view(np.uint16))  # bit-exact at::Half semantics
    else:
        np.testing.assert_allclose(got, ref, rtol=1e-6 if dtype == np.float32 else 1e-12,
                                   atol=1e-6 if dtype == np.float32 else 1e-12)


def test_pyramid_lookup_bitexact_and_equals_per_level():
    """the fused 4-level kernel == 4 x corr_index_forward + cat, bit for bit, and == oracle."""
    import droid_backends
    from droid_mi355x.corr import CorrBlock
    rng = np.random.default_rng(12)
    E, C, H, W = 3, 128, 16, 24
    f1 = dev(rng.normal(size=(1, E, C, H, W)).astype(np.float16))
    f2 = dev(rng.normal(size=(1, E, C, H, W)).astype(np.float16))
    cb = CorrBlock(f1, f2)
    coords = np.stack(np.meshgrid(np.arange(W), np.arange(H)), -1)[None, None].astype(np.float32)
    coords = np.repeat(coords, E, axis=1) + rng.normal(0, 2.5, (1, E, H, W, 2)).astype(np.float32)
    coords[0, 0, 0, 0] = [-40.0, 100.0]
    with torch.no_grad():
        fused = cb(dev(coords))
    c2 = dev(coords).permute(0, 1, 4, 2, 3).reshape(E, 2, H, W).contiguous()
    per = torch.cat([droid_backends.corr_index_forward(cb.corr_pyramid[i], (c2 / 2 ** i).contiguous(), 3)[0]
                     .view(1, E, -1, H, W) for i in range(4)], dim=2)
    np.testing.assert_array_equal(host(fused).view(np.uint16), host(per).view(np.uint16))
    ref = oc.lookup_pyramid([host(v) for v in cb.corr_pyramid], coords, 3)
    np.testing.assert_array_equal(host(fused).view(np.uint16), ref.view(np.uint16))


def test_tiled_pool_lookup_bitexact():
    """CorrBlock.__call__ on the 8x8-tiled slot pool (droid_corr_pyramid_lookup_tiled,
    the reference operators' NCHW lookup) == the row-major lookup of a block built
    from the final edge list, bit for bit, after drop / append edits (rows freed
    and refilled, pool growth), at 48x64 (levels 2 and 3 are 12 and 6 rows: a
    partial tile row) with off-map coordinates; == the oracle."""
    from droid_mi355x.corr import CorrBlock
    rng = np.random.default_rng(14)
    C, H, W = 128, 48, 64
    feats = [dev(rng.normal(size=(1, 1, C, H, W)).astype(np.float16)) for _ in range(9)]
    pairs = [(0, 1), (1, 2), (2, 0), (3, 4), (4, 5)]
    with torch.no_grad():
        mk = lambda ps, tiled: CorrBlock(torch.cat([feats[a] for a, _ in ps], 1),
                                         torch.cat([feats[b] for _, b in ps], 1), tiled=tiled)
        cb = mk(pairs, True)
        assert cb.tiled
        keep = np.array([True, False, True, False, True])
        cb = cb.select(keep)
        more = [(5, 6), (6, 7), (7, 8), (8, 0)]
        cb = cb.cat(mk(more, True))
        final = [p for p, k in zip(pairs, keep) if k] + more
        ref_blk = mk(final, False)
        E = len(final)
        coords = np.stack(np.meshgrid(np.arange(W), np.arange(H)), -1)[None, None].astype(np.float32)
        coords = np.repeat(coords, E, axis=1) + rng.normal(0, 4.0, (1, E, H, W, 2)).astype(np.float32)
        coords[0, 0, 0, 0] = [-40.0, 100.0]
        coords[0, 1, 2, 3] = [63.7, 47.9]
        coords[0, 2, 5, 5] = [-3.5, -3.5]
        got = cb(dev(coords))
        ref = ref_blk(dev(coords))
    assert got.shape == (1, E, 196, H, W)
    np.testing.assert_array_equal(host(got).view(np.uint16), host(ref).view(np.uint16))
    ora = oc.lookup_pyramid([host(v)[:2] for v in ref_blk.corr_pyramid], coords[:, :2], 3)
    np.testing.assert_array_equal(host(got)[:, :2].view(np.uint16), ora.view(np.uint16))


def _ab_lookup(bk, blk, coords):
    """CorrBlock.__call__ (droid_mi355x/corr.py) through another instance of the module (bk)."""
    batch, num, ht, wd, _ = coords.shape
    c = coords.reshape(batch * num, ht, wd, 2).float().contiguous()
    if blk.tiled:
        out = bk.corr_pyramid_lookup_tiled(blk._pyr, blk.level_shapes, c, blk.slot_tensor())
    else:
        out = bk.corr_pyramid_lookup(blk.reference_pyramid(), c, blk.radius)
    return out.view(batch, num, -1, ht, wd)


def test_coop_lookup_bitwise_equals_per_thread_kernel(ab_backends):
    """droid_corr_pyramid_lookup(_tiled)'s cooperative NCHW kernel (a wave per
    64 pixels, staged 16-B stores) == the per-thread kernel (droid_lookup_set_coop(0)),
    bit for bit, on the row-major and the tiled volume, with coordinates far off
    the map and on the borders; a 40x56 image (H*W % 64 == 0, 35 waves) and a
    20x36 one (H*W % 64 != 0: the per-thread kernel either way).  The switch is
    a testing hook (A/B library); the product library's output is the same bytes."""
    import droid_backends as product
    droid_backends = ab_backends   # the coop switch ships in the testing builds only
    from droid_mi355x.corr import CorrBlock
    rng = np.random.default_rng(15)
    try:
        for H, W, E in ((40, 56, 12), (20, 40, 5)):
            f1 = dev(rng.normal(size=(1, E, 128, H, W)).astype(np.float16))
            f2 = dev(rng.normal(size=(1, E, 128, H, W)).astype(np.float16))
            coords = np.stack(np.meshgrid(np.arange(W), np.arange(H)), -1)[None, None].astype(np.float32)
            coords = np.repeat(coords, E, axis=1) + rng.normal(0, 6.0, (1, E, H, W, 2)).astype(np.float32)
            coords[0, 0, :4, :4] = [[-40.0, 100.0]]
            coords[0, 1, 2, 3] = [W - 0.3, H - 0.1]
            coords[0, 2, 5] = [-3.5, -3.5]
            coords[0, 3, 7] = [W + 2.5, 1.25]
            c = dev(coords)
            with torch.no_grad():
                for tiled in (False, True):
                    blk = CorrBlock(f1, f2, tiled=tiled)
                    prod = blk(c)   # the product library (cooperative kernel where it applies)
                    droid_backends.lookup_set_coop(1)
                    got = _ab_lookup(droid_backends, blk, c)
                    droid_backends.lookup_set_coop(0)
                    ref = _ab_lookup(droid_backends, blk, c)
                    torch.cuda.synchronize()
                    assert torch.equal(got, ref), (H, W, tiled)
                    assert torch.equal(prod, got), (H, W, tiled)
    finally:
        droid_backends.lookup_set_coop(1)


def test_corr_index_backward_vs_oracle():
    import droid_backends
    rng = np.random.default_rng(13)
    B, H, W, H2, W2 = 2, 8, 10, 8, 10
    vol = rng.normal(size=(B, H, W, H2, W2)).astype(np.float32)
    coords = _coords(rng, B, H, W, H2, W2, 2.0)
    g = rng.normal(size=(B, 7, 7, H, W)).astype(np.float32)
    out, = droid_backends.corr_index_backward(dev(vol), dev(coords), dev(g), 3)
    ref = oc.corr_index_backward(vol, coords, g, 3)
    np.testing.assert_allclose(host(out), ref, atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("dtype", [np.float32, np.float16])
def test_altcorr_forward_vs_oracle(dtype):
    import droid_backends
    rng = np.random.default_rng(14)
    B, S, H, W, H2, W2, C = 2, 1, 12, 16, 6, 8, 64
    f1 = rng.normal(size=(B, H, W, C)).astype(dtype)
    f2 = rng.normal(size=(B, H2, W2, C)).astype(dtype)
    coords = np.stack(np.meshgrid(np.arange(W) / 2, np.arange(H) / 2), -1)[None, None]
    coords = (np.repeat(np.repeat(coords, B, 0), S, 1) + rng.normal(0, 1.5, (B, S, H, W, 2))).astype(np.float32)
    out, = droid_backends.altcorr_forward(dev(f1), dev(f2), dev(coords), 3)
    ref = oc.altcorr_forward(f1, f2, coords, 3)
    tol = 2e-4 if dtype == np.float32 else 2e-2
    np.testing.assert_allclose(host(out).astype(np.float64), ref, atol=tol * np.abs(ref).max(), rtol=tol)


def test_altcorr_matches_volume_lookup():
    """alt path == volume path on the same features (level 0, fp32)."""
    import droid_backends
    from droid_mi355x.corr import AltCorrBlock, CorrBlock
    rng = np.random.default_rng(15)
    C, H, W = 32, 16, 16
    fm = rng.normal(size=(1, 2, C, H, W)).astype(np.float32)
    vol = CorrBlock(dev(fm[:, :1]), dev(fm[:, 1:]))
    alt = AltCorrBlock(dev(fm))
    coords = (np.stack(np.meshgrid(np.arange(W), np.arange(H)), -1)[None, None]
              + rng.normal(0, 2, (1, 1, H, W, 2))).astype(np.float32)
    with torch.no_grad():
        a = vol(dev(coords))
        b = alt(dev(coords), torch.tensor([0], device="cuda"), torch.tensor([1], device="cuda"))
    np.testing.assert_allclose(host(a), host(b), atol=2e-4)


def test_altcorr_backward_vs_oracle():
    import droid_backends
    rng = np.random.default_rng(16)
    B, S, H, W, H2, W2, C = 1, 1, 6, 8, 6, 8, 16
    f1 = rng.normal(size=(B, H, W, C)).astype(np.float32)
    f2 = rng.normal(size=(B, H2, W2, C)).astype(np.float32)
    coords = (np.stack(np.meshgrid(np.arange(W), np.arange(H)), -1)[None, None]
              + rng.normal(0, 1.0, (B, S, H, W, 2))).astype(np.float32)
    g = rng.normal(size=(B, S, 49, H, W)).astype(np.float32)
    g1, g2, gc = droid_backends.altcorr_backward(dev(f1), dev(f2), dev(coords), dev(g), 3)
    r1, r2, rc = oc.altcorr_backward(f1, f2, coords, g, 3)
    np.testing.assert_allclose(host(g1), r1, atol=1e-4, rtol=1e-4)
    np.testing.assert_allclose(host(g2), r2, atol=1e-4, rtol=1e-4)
    assert np.all(host(gc) == 0)


# --- CorrBlock pyramid construction (droid_corr_volume_pyramid) -------------
def test_volume_pyramid_matches_reference_golden(golden_dir):
    """The hand-written pyramid kernel vs the reference's own CorrBlock
    (tests/golden/corr_pyramid.npz, fp32 on the CPU): fp16 inputs and outputs,
    so the tolerance is fp16 rounding of values of magnitude ~|level|."""
    import os
    from droid_mi355x.corr import CorrBlock
    g = np.load(os.path.join(golden_dir, "corr_pyramid.npz"))
    with torch.no_grad():
        cb = CorrBlock(dev(g["fmap1"]).half(), dev(g["fmap2"]).half())
    for i in range(4):
        ref = g["level%d" % i]
        got = host(cb.corr_pyramid[i].float()).reshape(ref.shape)
        np.testing.assert_allclose(got, ref, atol=4e-3 * max(1.0, np.abs(ref).max()), rtol=2e-3)


def test_volume_pyramid_levels_are_avg_pools_and_tiles():
    """Level l+1 is exactly F.avg_pool2d(2) of level l's fp16 values (the
    reference's pooling arithmetic), level 0 is the fp32-accumulated GEMM
    rounded to fp16, and the 8x8-tiled output is tile8 of the plain one, bit
    for bit; stereo-style indices (f2 = another rig slot) included."""
    import torch.nn.functional as F
    import droid_backends
    from droid_mi355x.corr import tile8
    rng = np.random.default_rng(5)
    NF, H, W = 5, 48, 64
    f = torch.from_numpy((rng.normal(size=(NF, H, W, 128)) / 4).astype(np.float16)).cuda()
    f1 = torch.tensor([0, 1, 2, 3, 4, 2], dtype=torch.int32, device="cuda")
    f2 = torch.tensor([1, 0, 3, 3, 2, 4], dtype=torch.int32, device="cuda")
    plain = droid_backends.corr_volume_pyramid(f, f1, f2, tiled=False)
    tiled = droid_backends.corr_volume_pyramid(f, f1, f2, tiled=True)
    E = f1.numel()
    a = f[f1.long()].reshape(E, H * W, 128).float()
    b = f[f2.long()].reshape(E, H * W, 128).float()
    v0 = torch.bmm(a, b.transpose(1, 2)).reshape(E, H, W, H, W)
    np.testing.assert_allclose(host(plain[0].float()), host(v0), atol=1e-3, rtol=1e-3)
    for i in range(3):
        lv = plain[i]
        h2, w2 = lv.shape[3:]
        pooled = F.avg_pool2d(lv.reshape(-1, 1, h2, w2), 2, stride=2).reshape(plain[i + 1].shape)
        assert torch.equal(pooled, plain[i + 1]), "level %d pooling" % (i + 1)
    for i in range(4):
        assert torch.equal(tile8(plain[i]), tiled[i]), "level %d tiling" % i
