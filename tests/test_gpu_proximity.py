"""Proximity edges on the device (droid_proximity_select via
droid_mi355x.factor_graph.proximity_edge_list / FactorGraph.add_proximity_factors)
vs the reference's own add_proximity_factors (tests/golden/proximity.npz) and
the oracle restatement (oracle/factor_graph.py:proximity_edges).  Edge lists
must be identical (integer work)."""
import os
import time

import numpy as np
import pytest
import torch

from gpu_util import dev
from oracle.factor_graph import proximity_edges
from test_oracle_golden import _proximity_case

pytestmark = pytest.mark.gpu


def test_proximity_matches_reference_fixture(golden_dir):
    from droid_mi355x.factor_graph import proximity_edge_list
    z = np.load(os.path.join(golden_dir, "proximity.npz"))
    for c in range(int(z["ncases"])):
        args, ref = _proximity_case(z, c)
        args["d"] = dev(args["d"])
        np.testing.assert_array_equal(proximity_edge_list(**args), ref, err_msg="case %d" % c)


def _lap_distances(rng, t0, t1, t, lap=24, nan=0):
    gi, gj = np.meshgrid(np.arange(t0, t), np.arange(t1, t), indexing="ij")
    d = (40.0 * np.abs(np.sin(np.pi * (gi - gj) / lap)) + rng.uniform(0, 8.0, gi.shape)).astype(np.float32).reshape(-1)
    if nan:
        d[rng.choice(d.size, nan, replace=False)] = np.nan
    return d


@pytest.mark.parametrize("t,t0,t1,rad,nms,stereo,max_factors,nan", [
    (256, 0, 0, 2, 2, False, 16 * 256, 0),        # the backend's call: whole video, max_factors = 16 t
    (300, 40, 10, 2, 2, True, 10 ** 7, 5),        # offsets, stereo, NaN distances, no cap
    (200, 0, 0, 3, 3, False, 900, 0),             # the cap hits early
    (96, 8, 8, 2, 0, False, 10 ** 6, 0),          # nms = 0: only exact hits suppressed
])
def test_proximity_matches_oracle(t, t0, t1, rad, nms, stereo, max_factors, nan):
    from droid_mi355x.factor_graph import proximity_edge_list
    rng = np.random.default_rng(t + t0)
    d = _lap_distances(rng, t0, t1, t, nan=nan)
    ne = 4 * t
    ei = rng.integers(0, t, ne)
    ej = np.clip(ei + rng.integers(-30, 31, ne), 0, t - 1)
    ref = proximity_edges(d, t0, t1, t, rad, nms, 16.0, ei, ej, stereo, max_factors)
    got = proximity_edge_list(dev(d), t0, t1, t, rad, nms, 16.0, ei, ej, stereo, max_factors)
    np.testing.assert_array_equal(got, ref)


def test_add_proximity_factors_on_video():
    """FactorGraph.add_proximity_factors end to end (frame_distance on the
    device, then the walk) vs the oracle walk over the same distances."""
    from droid_mi355x import DepthVideo, FactorGraph, synthetic
    n, H, W = 96, 12, 16
    rng = np.random.default_rng(77)
    video = DepthVideo(image_size=(8 * H, 8 * W), buffer=n, device="cuda:0")
    poses = synthetic.trajectory_laps(n, 24, rng)
    video.poses[:n] = torch.from_numpy(poses.astype(np.float32)).cuda()
    video.disps[:n] = torch.from_numpy(synthetic.smooth_disps(n, H, W, rng).astype(np.float32)).cuda()
    video.intrinsics[:n] = torch.from_numpy(np.tile(synthetic.INTRINSICS / 4, (n, 1)).astype(np.float32)).cuda()
    video.counter.value = n
    graph = FactorGraph(video, None, device="cuda:0", corr_impl="none", max_factors=16 * n)
    ii, jj = synthetic.c3_edges(n, 300, rng=np.random.default_rng(5))
    graph._ii, graph._jj = ii, jj
    got = []
    graph.add_factors = lambda a, b, remove=False: got.append(np.stack([a, b], 1))
    graph.add_proximity_factors(t0=0, t1=0, rad=2, nms=2, beta=0.25, thresh=16.0)
    gi, gj = np.meshgrid(np.arange(n), np.arange(n), indexing="ij")
    d = video.distance(dev(gi.reshape(-1)), dev(gj.reshape(-1)), beta=0.25).cpu().numpy()
    ref = proximity_edges(d, 0, 0, n, 2, 2, 16.0, ii, jj, False, 16 * n)
    assert len(ref) > 2 * (3 * n - 6)        # proximity pairs beyond the static edges
    np.testing.assert_array_equal(got[0], ref)


def test_proximity_c5_scale_timing():
    """The global backend at C5 scale: 2048 keyframes, the whole grid (4.2 M
    candidates), max_factors = 16 t; the device walk against the oracle."""
    from droid_mi355x.factor_graph import proximity_edge_list
    t = 2048
    rng = np.random.default_rng(2048)
    d = _lap_distances(rng, 0, 0, t, lap=256)
    ei = rng.integers(0, t, 8 * t)
    ej = np.clip(ei + rng.integers(-3, 4, 8 * t), 0, t - 1)
    dd = dev(d)
    proximity_edge_list(dd, 0, 0, t, 2, 2, 16.0, ei, ej, False, 16 * t)
    torch.cuda.synchronize()
    t_0 = time.perf_counter()
    got = proximity_edge_list(dd, 0, 0, t, 2, 2, 16.0, ei, ej, False, 16 * t)
    ms = 1000 * (time.perf_counter() - t_0)
    ref = proximity_edges(d, 0, 0, t, 2, 2, 16.0, ei, ej, False, 16 * t)
    np.testing.assert_array_equal(got, ref)
    print("proximity walk, 2048 KF full grid: %.2f ms (%d edges)" % (ms, len(got)))
