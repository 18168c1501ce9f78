"""FactorGraph.update() at the benchmark's full size: C3's
256 keyframes / 2048 edges and C4's stereo 128 keyframes / 984 edges, both at
the 48x64 feature maps of a 384x512 image.

Two graphs are built on identical DepthVideo states: one runs the reference's
structure with the torch UpdateModule under autocast (factor_graph.py:196-242 -
CorrBlock lookup, the module, coords1 + delta), the other the MI355X fast path
(FusedUpdateModule: the lookup fused with corr_encoder[0] on the tiled volume,
the 8-wave W=64 gate tiles these edge counts select, fused heads, per-frame
gate term).  The fast path's net / target / weight / damping must agree with
the torch module's at fp16 tolerance over every pixel of every edge, and the BA
it runs - on the inputs it built - must agree with the oracle at the north
star's 1e-4.  (The oracle composition of the whole update at this size would
take minutes on the host; the module is pinned to the reference by
update_module.npz, the lookup bit-exactly, the BA here.)"""
import numpy as np
import pytest
import torch

from fill import det_fill
from gpu_util import host
from oracle import ba as oba

pytestmark = pytest.mark.gpu

H, W = 48, 64


def _video(config, seed):
    from droid_mi355x import DepthVideo, synthetic
    n = 256 if config == "C3" else 128
    stereo = config == "C4"
    rng = np.random.default_rng(seed)
    video = DepthVideo(image_size=(8 * H, 8 * W), buffer=n, stereo=stereo, device="cuda")
    gt = synthetic.trajectory(n, rng)
    poses, disps = synthetic.perturb(gt, synthetic.smooth_disps(n, H, W, rng), rng)
    video.poses[:n] = torch.from_numpy(poses.astype(np.float32)).cuda()
    video.disps[:n] = torch.from_numpy(disps.astype(np.float32)).cuda()
    video.intrinsics[:n] = torch.from_numpy(np.tile(synthetic.INTRINSICS, (n, 1))).cuda()
    g = torch.Generator(device="cuda").manual_seed(seed)
    video.fmaps[:n] = torch.randn((n, 2 if stereo else 1, 128, H, W), generator=g, device="cuda").half()
    video.nets[:n] = torch.tanh(torch.randn((n, 128, H, W), generator=g, device="cuda")).half()
    video.inps[:n] = torch.relu(torch.randn((n, 128, H, W), generator=g, device="cuda")).half()
    video.counter.value = n
    return video


def _edges(config):
    from droid_mi355x import synthetic
    if config == "C3":
        return synthetic.c3_edges(256, 2048, rng=np.random.default_rng(1003))
    return synthetic.c4_edges(128, rng=np.random.default_rng(1004))


def _state(g, E):
    """net (E,H,W,128), target / weight (E,H*W*2), damping, in one layout for both paths."""
    net = g.net.float()
    if net.dim() == 5:                      # reference layout (1,E,128,H,W)
        net = net[0].permute(0, 2, 3, 1)
    return dict(net=host(net), target=host(g.target.reshape(E, -1)), weight=host(g.weight.reshape(E, -1)),
                damping=host(g.damping))


def _err(a, b):
    d = np.abs(a.astype(np.float64) - b.astype(np.float64))
    return float(d.max()), float(np.percentile(d, 99.99)), float(d.mean())


@pytest.mark.parametrize("config", ["C3", "C4"])
def test_update_full_size_matches_reference_module(config):
    import droid_backends
    from droid_mi355x import FactorGraph, UpdateModule
    from droid_mi355x.fused import FusedUpdateModule
    ii, jj = _edges(config)
    E = len(ii)
    m = UpdateModule().to("cuda").eval()
    det_fill(m)

    # the reference's structure: CorrBlock lookup + the torch module under autocast
    va = _video(config, 77)
    ga = FactorGraph(va, m, device="cuda", corr_impl="volume")
    with torch.no_grad():
        ga.add_factors(ii, jj)
        ga.update()
    torch.cuda.synchronize()
    ref = _state(ga, E)
    ref_poses = host(va.poses[:va.counter.value])
    del ga, va
    torch.cuda.empty_cache()

    # the fast path, with a spy on the BA it calls
    vb = _video(config, 77)
    gb = FactorGraph(vb, FusedUpdateModule(m), device="cuda")
    assert gb.fused
    captured = {}
    orig = droid_backends.ba

    def spy(*a, **k):
        captured["a"] = [x.detach().clone() if isinstance(x, torch.Tensor) else x for x in a]
        return orig(*a, **k)

    droid_backends.ba = spy
    try:
        with torch.no_grad():
            gb.add_factors(ii, jj)
            coords0 = host(vb.reproject(ii, jj)[0]).reshape(E, -1)   # coords1 before the update's BA
            gb.update()
    finally:
        droid_backends.ba = orig
    torch.cuda.synchronize()
    got = _state(gb, E)
    n = vb.counter.value

    for k, tol in (("net", 2e-2), ("weight", 2e-2)):
        mx, p, mean = _err(got[k], ref[k])
        print("%s %s: max %.3g, p99.99 %.3g, mean %.3g" % (config, k, mx, p, mean))
        assert mx <= 2 * tol and p <= tol and mean <= tol / 20, k
    # target = coords1 + delta: the delta head's scale sets the fp16 tolerance
    dmax = max(1.0, float(np.abs(ref["target"] - coords0).max()))
    mx, p, mean = _err(got["target"], ref["target"])
    print("%s target: max %.3g, p99.99 %.3g, mean %.3g (delta scale %.3g)" % (config, mx, p, mean, dmax))
    assert mx <= 6e-2 * dmax and p <= 3e-2 * dmax and mean <= 1.5e-3 * dmax
    u = np.unique(ii)
    dd = np.abs(got["damping"][u] - ref["damping"][u]).max()
    assert dd <= 1e-3 + 2e-2 * np.abs(ref["damping"][u]).max(), dd

    # the BA update() ran, on the inputs it built, against the oracle (1e-4)
    a = captured["a"]
    np.testing.assert_array_equal(host(a[7]), ii)
    np.testing.assert_array_equal(host(a[8]), jj)
    ba_ref = oba.ba(poses=host(a[0]), disps=host(a[1]), intrinsics=host(a[2]), disps_sens=host(a[3]),
                    targets=host(a[4]), weights=host(a[5]), eta=host(a[6]), ii=host(a[7]), jj=host(a[8]), t0=a[9],
                    t1=a[10], iterations=a[11], lm=a[12], ep=a[13], motion_only=a[14])
    np.testing.assert_allclose(host(vb.poses[:n]), ba_ref["poses"][:n], atol=1e-4)
    np.testing.assert_allclose(host(vb.disps[:n]), np.maximum(ba_ref["disps"][:n], 0.001), atol=1e-4)
    # and the two paths' poses after their own BA stay close (different fp16 inputs)
    print("%s poses after update: max |fused - reference| %.3g" % (config, np.abs(host(vb.poses[:n]) - ref_poses).max()))
    np.testing.assert_allclose(host(vb.poses[:n]), ref_poses, atol=5e-3)
