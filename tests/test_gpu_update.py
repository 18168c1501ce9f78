"""Update operator and FactorGraph.update() on the GPU."""
import os

import numpy as np
import pytest
import torch

from fill import det_fill, det_state_dict
from gpu_util import dev, host
from oracle import ba as oba
from oracle import update_module as oum

pytestmark = pytest.mark.gpu


def test_update_module_matches_reference_golden(golden_dir):
    from droid_mi355x.update import UpdateModule
    u = np.load(os.path.join(golden_dir, "update_module.npz"))
    m = UpdateModule().to("cuda")
    det_fill(m)
    with torch.no_grad():
        out = m(dev(u["net"]), dev(u["inp"]), dev(u["corr"]), dev(u["flow"]), dev(u["ii"]), dev(u["jj"]))
    for name, o in zip(["net_out", "delta", "weight", "eta", "upmask"], out):
        np.testing.assert_allclose(host(o), u[name], atol=2e-4, rtol=2e-3)


def _graph(E_pairs=None, n_kf=8, H=16, W=24, seed=31):
    from droid_mi355x import DepthVideo, FactorGraph, UpdateModule, synthetic
    rng = np.random.default_rng(seed)
    video = DepthVideo(image_size=(8 * H, 8 * W), buffer=n_kf + 2, device="cuda")
    poses = synthetic.trajectory(n_kf, rng)
    poses, disps = synthetic.perturb(poses, synthetic.smooth_disps(n_kf, H, W, rng), rng)
    video.poses[:n_kf] = dev(poses.astype(np.float32))
    video.disps[:n_kf] = dev(disps.astype(np.float32))
    video.intrinsics[:n_kf] = dev(np.array([[H / 1.5, H / 1.5, W / 2, H / 2]] * n_kf, np.float32))
    video.fmaps[:n_kf] = dev(rng.normal(size=(n_kf, 1, 128, H, W)).astype(np.float16))
    video.nets[:n_kf] = dev(np.tanh(rng.normal(size=(n_kf, 128, H, W))).astype(np.float16))
    video.inps[:n_kf] = dev(np.maximum(rng.normal(size=(n_kf, 128, H, W)), 0).astype(np.float16))
    video.counter.value = n_kf
    net = UpdateModule().to("cuda").eval()
    det_fill(net)
    g = FactorGraph(video, net, device="cuda")
    g.add_neighborhood_factors(0, n_kf, r=2)
    return video, g


def test_factor_graph_update_end_to_end():
    """update(): lookup + update_op + BA.  BA parity is checked on the very
    inputs update() handed it (captured), and corr parity on the lookup."""
    import droid_backends
    video, g = _graph()
    captured = {}
    orig = droid_backends.ba

    def spy(*a, **k):
        captured["args"] = [x.detach().clone() if isinstance(x, torch.Tensor) else x for x in a]
        captured["kw"] = dict(k)
        return orig(*a, **k)

    droid_backends.ba = spy
    try:
        with torch.no_grad():
            g.update(itrs=2)
    finally:
        droid_backends.ba = orig
    torch.cuda.synchronize()
    a = captured["args"]
    poses0, disps0 = host(a[0]), host(a[1])
    prob = dict(poses=poses0, disps=disps0, intrinsics=host(a[2]), disps_sens=host(a[3]), targets=host(a[4]),
                weights=host(a[5]), eta=host(a[6]), ii=host(a[7]), jj=host(a[8]), t0=a[9], t1=a[10])
    ref = oba.ba(**prob, iterations=a[11], lm=a[12], ep=a[13], motion_only=a[14])
    n = video.counter.value
    np.testing.assert_allclose(host(video.poses[:n]), ref["poses"][:n], atol=1e-4)
    np.testing.assert_allclose(host(video.disps[:n]), np.maximum(ref["disps"][:n], 0.001), atol=1e-4)
    assert np.isfinite(host(g.net.float())).all()
    assert g.target.shape == (1, len(g._ii), 16, 24, 2)


def test_update_lowmem_runs():
    video, g = _graph(seed=32)
    with torch.no_grad():
        g.update_lowmem(steps=1)
    assert np.isfinite(host(video.poses)).all() and np.isfinite(host(video.disps)).all()


def _c2_video(H=48, W=64, seed=51, stereo=False, n=16, buffer=None):
    """C2 frontend shape: 16-KF buffer, fmaps/net/inp ~ N / tanh / relu."""
    from droid_mi355x import DepthVideo, synthetic
    rng = np.random.default_rng(seed)
    video = DepthVideo(image_size=(8 * H, 8 * W), buffer=buffer or n, stereo=stereo, device="cuda")
    gt = synthetic.trajectory(n, rng)
    poses, disps = synthetic.perturb(gt, synthetic.smooth_disps(n, H, W, rng), rng)
    video.poses[:n] = dev(poses.astype(np.float32))
    video.disps[:n] = dev(disps.astype(np.float32))
    video.intrinsics[:n] = dev(np.tile(synthetic.INTRINSICS * np.float32(W / 64.0), (n, 1)))
    video.fmaps[:n] = dev(rng.normal(size=(n, 2 if stereo else 1, 128, H, W)).astype(np.float16))
    video.nets[:n] = dev(np.tanh(rng.normal(size=(n, 128, H, W))).astype(np.float16))
    video.inps[:n] = dev(np.maximum(rng.normal(size=(n, 128, H, W)), 0).astype(np.float16))
    video.counter.value = n
    return video


def test_update_unit_matches_oracle_composition():
    """FactorGraph.update() as a unit (factor_graph.py:196-242) against the
    oracle composition (oracle/factor_graph.py: reproject -> lookup ->
    UpdateModule fp32 -> coords1 + delta -> damping scatter -> inactive-edge
    concat -> BA) on a C2-shaped graph at 48x64 with use_inactive=True: the
    fused operator (W=64 band tiles, fused lookup + corr_encoder[0] on the
    tiled volume, fused delta/weight heads) for target, weight, damping and
    net at fp16 tolerance; the BA inputs it builds (edge lists exactly); and
    the BA result on those inputs at the north star's 1e-4."""
    from droid_mi355x import synthetic
    ii, jj = synthetic.c2_edges()
    _update_unit_vs_oracle(_c2_video(48, 64), ii, jj)


def test_update_unit_stereo_matches_oracle_composition():
    """The same unit check on a stereo graph (SURVEY.md §8d C4 shape at 48x64):
    every frame of the window has its (i, i) edge, whose correlation volume is
    built against the RIGHT image (factor_graph.py:112-114) and whose BA rows
    carry depth terms only (droid_kernels.cu:219-229, 319-323), plus temporal
    and loop edges; use_inactive=True after the older edges are stored."""
    ii, jj = _stereo_edges(16, lo=4, loops=[(15, 5), (5, 15), (13, 6), (6, 13), (12, 4), (4, 12)])
    _update_unit_vs_oracle(_c2_video(48, 64, seed=53, stereo=True), ii, jj)


def _stereo_edges(n, lo, loops):
    es = [(i, i) for i in range(lo, n)]
    es += [(i, j) for i in range(lo, n) for j in range(lo, n) if i != j and abs(i - j) <= 3]
    es += [e for e in loops if e not in es]
    e = np.asarray(es, np.int64)
    return e[:, 0], e[:, 1]


def _update_unit_vs_oracle(video, ii, jj, store_below=7):
    import droid_backends
    from droid_mi355x import FactorGraph, UpdateModule
    from droid_mi355x.fused import FusedUpdateModule
    from oracle import factor_graph as ofg
    m = UpdateModule().to("cuda").eval()
    det_fill(m)
    g = FactorGraph(video, FusedUpdateModule(m), device="cuda")
    with torch.no_grad():
        g.add_factors(ii, jj)
        g.update()                                  # non-trivial targets / weights / damping
        g.rm_factors(g.ii < store_below, store=True)   # device-tensor mask, as droid_frontend.py:42 passes
    assert len(g._ii_inac) > 0 and g._ii.min() == store_below
    n = video.counter.value
    st = dict(poses=host(video.poses[:n]), disps=host(video.disps[:n]), disps_sens=host(video.disps_sens[:n]),
              intrinsics=host(video.intrinsics[:n]), fmaps=host(video.fmaps[:n].float()),
              ii=g._ii.copy(), jj=g._jj.copy(), net=host(g.net.float()).transpose(0, 3, 1, 2),
              inp=host(g.inp.float()).transpose(0, 3, 1, 2), target=host(g.target[0]), weight=host(g.weight[0]),
              damping=host(g.damping[:n]))
    inactive = (g._ii_inac.copy(), g._jj_inac.copy(), host(g.target_inac[0]), host(g.weight_inac[0]))
    params = {k: host(v.float()) for k, v in m.state_dict().items()}
    captured = {}
    orig = droid_backends.ba

    def spy(*a, **k):
        captured["a"] = [x.detach().clone() if isinstance(x, torch.Tensor) else x for x in a]
        return orig(*a, **k)

    droid_backends.ba = spy
    try:
        with torch.no_grad():
            g.update(use_inactive=True)
    finally:
        droid_backends.ba = orig
    torch.cuda.synchronize()
    ref = ofg.update(params, st["poses"], st["disps"], st["disps_sens"], st["intrinsics"], st["fmaps"], st["ii"],
                     st["jj"], st["net"], st["inp"], st["target"], st["weight"], st["damping"], use_inactive=True,
                     inactive=inactive)
    # the update operator's outputs (fp16 storage / fp16 convs vs fp32)
    np.testing.assert_allclose(host(g.net.float()).transpose(0, 3, 1, 2), ref["net"], atol=2e-2)
    dmax = max(1.0, float(np.abs(ref["target"] - ref["coords1"]).max()))
    np.testing.assert_allclose(host(g.target[0]), ref["target"], atol=3e-2 * dmax)
    np.testing.assert_allclose(host(g.weight[0]), ref["weight"], atol=1.5e-2)
    u = np.unique(st["ii"])
    np.testing.assert_allclose(host(g.damping[u]), ref["damping"][u], atol=1e-3 + 2e-2 * np.abs(ref["damping"][u]).max())
    untouched = np.setdiff1d(np.arange(n), u)
    np.testing.assert_array_equal(host(g.damping[untouched]), st["damping"][untouched])
    # the BA call it makes: inactive edges with ii, jj >= t0 - 3 first, then the active ones
    a = captured["a"]
    tgt, wgt, eta, ii_ba, jj_ba, t0, t1 = ref["ba_in"]
    np.testing.assert_array_equal(host(a[7]), ii_ba)
    np.testing.assert_array_equal(host(a[8]), jj_ba)
    assert (a[9], a[10]) == (t0, t1) and (a[11], a[12], a[13]) == (2, 1e-4, 0.1)
    assert len(ii_ba) > len(st["ii"])               # some inactive edges joined
    np.testing.assert_allclose(host(a[4]), tgt, atol=3e-2 * dmax)
    np.testing.assert_allclose(host(a[5]), wgt, atol=1.5e-2)
    np.testing.assert_allclose(host(a[6]), eta, atol=1e-3 + 2e-2 * np.abs(eta).max())
    # BA on the inputs update() built (the 1e-4 bar) and the disparity clamp
    ba_ref = oba.ba(poses=host(a[0]), disps=host(a[1]), intrinsics=host(a[2]), disps_sens=host(a[3]),
                    targets=host(a[4]), weights=host(a[5]), eta=host(a[6]), ii=host(a[7]), jj=host(a[8]), t0=a[9],
                    t1=a[10], iterations=a[11], lm=a[12], ep=a[13], motion_only=a[14])
    np.testing.assert_allclose(host(video.poses[:n]), ba_ref["poses"][:n], atol=1e-4)
    np.testing.assert_allclose(host(video.disps[:n]), np.maximum(ba_ref["disps"][:n], 0.001), atol=1e-4)
    # and the whole composition lands close to the oracle's own BA result
    np.testing.assert_allclose(host(video.poses[:n]), ref["poses"][:n], atol=2e-3)
    return g, ref


def test_update_motion_only_unit_matches_oracle():
    """update(N, N + M, motion_only=True) as the trajectory filler calls it
    (trajectory_filler.py:64-72): M new frames appended after N keyframes
    (fmaps only, poses interpolated), edges from each frame's bracketing
    keyframes t0 / t1 to it, motion-only BA over poses [N, N+M) - no Schur
    step, no depth update.  Update-operator outputs at fp16 tolerance vs the
    oracle composition, BA 1e-4 on the inputs update() handed over, 6
    iterations as the filler runs."""
    import droid_backends
    from droid_mi355x import FactorGraph, UpdateModule
    from droid_mi355x.fused import FusedUpdateModule
    from oracle import factor_graph as ofg
    H, W = 48, 64
    video = _c2_video(H, W, seed=54)
    N, M = 12, 4
    m = UpdateModule().to("cuda").eval()
    det_fill(m)
    # the filler's new frames: interpolated poses (here: the neighbours' plus noise), fmaps, counter += M
    rng = np.random.default_rng(55)
    t0 = np.array([8, 9, 10, 10])
    t1 = np.minimum(t0 + 1, N - 1)
    with torch.no_grad():
        video.poses[N:N + M] = video.poses[dev(t0)] + dev(rng.normal(0, 0.01, (M, 7)).astype(np.float32)) * \
            dev(np.array([1, 1, 1, 0, 0, 0, 0], np.float32))
        video.fmaps[N:N + M] = dev(rng.normal(size=(M, 1, 128, H, W)).astype(np.float16))
        video.disps[N:N + M] = 1.0
    params = {k: host(v.float()) for k, v in m.state_dict().items()}
    g = FactorGraph(video, FusedUpdateModule(m), device="cuda")
    with torch.no_grad():
        g.add_factors(t0, np.arange(N, N + M))
        g.add_factors(t1, np.arange(N, N + M))
    n = N + M
    for it in range(6):
        st = dict(poses=host(video.poses[:n]), disps=host(video.disps[:n]), disps_sens=host(video.disps_sens[:n]),
                  intrinsics=host(video.intrinsics[:n]), fmaps=host(video.fmaps[:n].float()),
                  net=host(g.net.float()).transpose(0, 3, 1, 2), inp=host(g.inp.float()).transpose(0, 3, 1, 2),
                  target=host(g.target[0]), weight=host(g.weight[0]), damping=host(g.damping[:n]))
        captured = {}
        orig = droid_backends.ba

        def spy(*a, **k):
            captured["a"] = [x.detach().clone() if isinstance(x, torch.Tensor) else x for x in a]
            return orig(*a, **k)

        droid_backends.ba = spy
        try:
            with torch.no_grad():
                g.update(N, N + M, motion_only=True)
        finally:
            droid_backends.ba = orig
        torch.cuda.synchronize()
        ref = ofg.update(params, st["poses"], st["disps"], st["disps_sens"], st["intrinsics"], st["fmaps"], g._ii,
                         g._jj, st["net"], st["inp"], st["target"], st["weight"], st["damping"], t0=N, t1=N + M,
                         motion_only=True)
        np.testing.assert_allclose(host(g.net.float()).transpose(0, 3, 1, 2), ref["net"], atol=2e-2)
        dmax = max(1.0, float(np.abs(ref["target"] - ref["coords1"]).max()))
        np.testing.assert_allclose(host(g.target[0]), ref["target"], atol=3e-2 * dmax)
        np.testing.assert_allclose(host(g.weight[0]), ref["weight"], atol=1.5e-2)
        a = captured["a"]
        assert (a[9], a[10], a[14]) == (N, N + M, True)
        ba_ref = oba.ba(poses=host(a[0]), disps=host(a[1]), intrinsics=host(a[2]), disps_sens=host(a[3]),
                        targets=host(a[4]), weights=host(a[5]), eta=host(a[6]), ii=host(a[7]), jj=host(a[8]),
                        t0=a[9], t1=a[10], iterations=a[11], lm=a[12], ep=a[13], motion_only=True)
        np.testing.assert_allclose(host(video.poses[:n]), ba_ref["poses"][:n], atol=1e-4)
        # motion-only: keyframe poses [0, N) and every disparity stay as they were
        np.testing.assert_array_equal(host(video.poses[:N]), st["poses"][:N])
        np.testing.assert_array_equal(host(video.disps[:n]), np.maximum(st["disps"], 0.001))
        np.testing.assert_allclose(host(video.poses[:n]), ref["poses"][:n], atol=2e-3)
    assert np.abs(host(video.poses[N:n]) - host(video.poses[dev(t0)])).max() > 1e-3


def test_update_lowmem_matches_oracle_composition():
    """update_lowmem (factor_graph.py:245-290, the global-BA backend's step) on
    the fused path - on-demand correlation (corr_alt_ce0) + factored gates, all
    edges in one pass - against the oracle composition with the backend's BA
    parameters (t0=1, t1=counter, lm=1e-5, ep=1e-2), at 48x64."""
    from droid_mi355x import FactorGraph, UpdateModule, synthetic
    from droid_mi355x.fused import FusedUpdateModule
    from oracle import factor_graph as ofg
    H, W = 48, 64
    video = _c2_video(H, W, seed=52)
    m = UpdateModule().to("cuda").eval()
    det_fill(m)
    g = FactorGraph(video, FusedUpdateModule(m), device="cuda", corr_impl="alt")
    # the backend's graph covers every frame (unique(ii) must be unique([1, t) U ii), the eta rows)
    ii, jj = synthetic.c3_edges(16, 96, rng=np.random.default_rng(7))
    with torch.no_grad():
        g.add_factors(ii, jj)
    n = video.counter.value
    st = dict(poses=host(video.poses[:n]), disps=host(video.disps[:n]), disps_sens=host(video.disps_sens[:n]),
              intrinsics=host(video.intrinsics[:n]), fmaps=host(video.fmaps[:n].float()),
              net=host(g.net.float()).transpose(0, 3, 1, 2), target=host(g.target[0]), weight=host(g.weight[0]),
              damping=host(g.damping[:n]))
    inp = host(video.inps[:n].float())[g._ii]
    params = {k: host(v.float()) for k, v in m.state_dict().items()}
    import droid_backends
    from oracle import ba as oba
    captured = {}
    orig = droid_backends.ba

    def spy(*a, **k):
        captured["a"] = [x.detach().clone() if isinstance(x, torch.Tensor) else x for x in a]
        return orig(*a, **k)

    droid_backends.ba = spy
    try:
        with torch.no_grad():
            g.update_lowmem(steps=1)
    finally:
        droid_backends.ba = orig
    torch.cuda.synchronize()
    # the BA update_lowmem drives, on the very inputs it handed over, within the
    # north star's 1e-4 of the oracle (the composition below is looser: its
    # targets come from the fp32 operator, the device's from the fp16 one)
    a = captured["a"]
    assert (a[9], a[10], a[12], a[13], a[14]) == (1, n, 1e-5, 1e-2, False)
    ba_ref = oba.ba(poses=host(a[0]), disps=host(a[1]), intrinsics=host(a[2]), disps_sens=host(a[3]),
                    targets=host(a[4]), weights=host(a[5]), eta=host(a[6]), ii=host(a[7]), jj=host(a[8]),
                    t0=a[9], t1=a[10], iterations=a[11], lm=a[12], ep=a[13], motion_only=False)
    np.testing.assert_allclose(host(video.poses[:n]), ba_ref["poses"][:n], atol=1e-4)
    np.testing.assert_allclose(host(video.disps[:n]), np.maximum(ba_ref["disps"][:n], 1e-3), atol=1e-4)
    ref = ofg.update(params, st["poses"], st["disps"], st["disps_sens"], st["intrinsics"], st["fmaps"], g._ii,
                     g._jj, st["net"], inp, st["target"], st["weight"], st["damping"], t0=1, t1=n, lm=1e-5, ep=1e-2)
    np.testing.assert_allclose(host(g.net.float()).transpose(0, 3, 1, 2), ref["net"], atol=2e-2)
    dmax = max(1.0, float(np.abs(ref["target"] - ref["coords1"]).max()))
    np.testing.assert_allclose(host(g.target[0]), ref["target"], atol=3e-2 * dmax)
    np.testing.assert_allclose(host(g.weight[0]), ref["weight"], atol=1.5e-2)
    u = np.unique(g._ii)
    np.testing.assert_allclose(host(g.damping[u]), ref["damping"][u], atol=1e-3 + 2e-2 * np.abs(ref["damping"][u]).max())
    np.testing.assert_allclose(host(video.poses[:n]), ref["poses"][:n], atol=2e-3)
    np.testing.assert_allclose(host(video.disps[:n]), ref["disps"][:n], atol=2e-2)


def test_reference_update_structure_with_dropin_module():
    """The reference's update() structure (FactorGraph's NCHW path: materialised
    lookup, update_op(net, inp, corr, motn, ii, jj) under autocast, BA) with the
    MI355X UpdateModule drop-in (ReferenceLayoutUpdateModule) vs the torch
    UpdateModule on identical state at 48x64: targets, weights, damping and
    the hidden state agree at fp16 tolerance, and the BA it drives matches the
    oracle on the inputs it handed over."""
    import droid_backends
    from droid_mi355x.fused import ReferenceLayoutUpdateModule
    va, ga = _graph(H=48, W=64, seed=41)
    vb, gb = _graph(H=48, W=64, seed=41)
    gb.update_op = ReferenceLayoutUpdateModule(gb.update_op)
    assert not gb.fused
    captured = {}
    orig = droid_backends.ba

    def spy(*a, **k):
        captured["args"] = [x.detach().clone() if isinstance(x, torch.Tensor) else x for x in a]
        return orig(*a, **k)

    with torch.no_grad():
        ga.update(itrs=2)
        droid_backends.ba = spy
        try:
            gb.update(itrs=2)
        finally:
            droid_backends.ba = orig
    torch.cuda.synchronize()
    np.testing.assert_allclose(host(gb.net.float()), host(ga.net.float()), atol=2e-2)
    np.testing.assert_allclose(host(gb.target), host(ga.target), atol=5e-2 * max(1.0, float(ga.target.abs().max())))
    np.testing.assert_allclose(host(gb.weight), host(ga.weight), atol=2e-2)
    n = va.counter.value
    np.testing.assert_allclose(host(gb.damping[:n]), host(ga.damping[:n]), atol=1e-4 + 3e-2 * float(ga.damping[:n].abs().max()))
    a = captured["args"]
    prob = dict(poses=host(a[0]), disps=host(a[1]), intrinsics=host(a[2]), disps_sens=host(a[3]), targets=host(a[4]),
                weights=host(a[5]), eta=host(a[6]), ii=host(a[7]), jj=host(a[8]), t0=a[9], t1=a[10])
    ref = oba.ba(**prob, iterations=a[11], lm=a[12], ep=a[13], motion_only=a[14])
    np.testing.assert_allclose(host(vb.poses[:n]), ref["poses"][:n], atol=1e-4)
    np.testing.assert_allclose(host(vb.disps[:n]), np.maximum(ref["disps"][:n], 0.001), atol=1e-4)


def test_update_graph_replay_matches_eager():
    """update() replayed from a captured HIP graph (FactorGraph.graphs,
    DROID_UPDATE_GRAPHS=1) gives the eager body's results bit for bit, across
    replays, an edge edit (graph dropped, eager, re-captured), use_inactive and
    a keyframe removal (the capture's safety rules)."""
    from droid_mi355x import FactorGraph, UpdateModule, synthetic
    from droid_mi355x.fused import FusedUpdateModule
    m = UpdateModule().to("cuda").eval()
    det_fill(m)
    ii, jj = synthetic.c2_edges()
    runs = []
    for graphs in (True, False):
        video = _c2_video(48, 64, seed=57)
        g = FactorGraph(video, FusedUpdateModule(m), device="cuda")
        g.graphs = graphs
        g.graph_strict = True
        with torch.no_grad():
            g.add_factors(ii, jj)
            for _ in range(4):
                g.update()
            g.rm_factors(g._ii < 7, store=True)
            for _ in range(3):
                g.update(use_inactive=True)
            g.add_factors(np.array([15, 4]), np.array([4, 15]))
            for _ in range(3):
                g.update(use_inactive=True)
            g.rm_keyframe(12)
            for _ in range(3):
                g.update(use_inactive=True)
        torch.cuda.synchronize()
        runs.append((g, video))
    (ga, va), (gb, vb) = runs
    assert ga.graphs and ga._graph is not None and gb._graph is None
    for x, y in ((va.poses, vb.poses), (va.disps, vb.disps), (ga.net, gb.net), (ga.target, gb.target),
                 (ga.weight, gb.weight), (ga.damping, gb.damping), (ga.age, gb.age)):
        np.testing.assert_array_equal(host(x), host(y))
