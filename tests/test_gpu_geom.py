"""HIP geometry kernels vs the CPU oracle."""
import numpy as np
import pytest
import torch

from droid_mi355x import synthetic
from gpu_util import dev, host
from oracle import geometry as og

pytestmark = pytest.mark.gpu


def _state(seed=21, N=6, H=12, W=16):
    rng = np.random.default_rng(seed)
    poses = synthetic.trajectory(N, rng)
    poses, disps = synthetic.perturb(poses, synthetic.smooth_disps(N, H, W, rng), rng)
    disps[0, 0, 0] = 20.0  # a point that projects behind / very close
    intr = np.array([[14.0, 15.0, 8.0, 6.0]] * N) + rng.normal(0, 0.1, (N, 4))
    return poses.astype(np.float32), disps.astype(np.float32), intr.astype(np.float32)


def test_projective_transform_and_motion_features():
    import droid_backends
    poses, disps, intr = _state()
    ii = np.array([0, 1, 2, 3, 4, 5, 2, 3], np.int64)
    jj = np.array([1, 0, 3, 2, 5, 4, 2, 0], np.int64)   # includes a stereo edge (2,2)
    E, H, W = len(ii), disps.shape[1], disps.shape[2]
    target = np.random.default_rng(1).normal(8, 10, (E, H, W, 2)).astype(np.float32)
    coords, valid, motn = droid_backends.projective_transform(dev(poses), dev(disps), dev(intr), dev(ii), dev(jj),
                                                              target=dev(target))
    rc, rv = og.projective_transform(poses, disps, intr, ii, jj)
    np.testing.assert_allclose(host(coords), rc, atol=2e-4, rtol=1e-4)
    assert np.mean(host(valid) == rv) > 0.999
    grid = og.coords_grid(H, W)
    ref_m = np.concatenate([rc - grid, target - rc], -1).transpose(0, 3, 1, 2).clip(-64, 64)
    np.testing.assert_allclose(host(motn), ref_m, atol=3e-4, rtol=1e-4)


def test_frame_distance_projmap_iproj():
    import droid_backends
    poses, disps, intr = _state(22)
    k = intr[0]
    ii = np.array([0, 1, 2, 4, 5], np.int64)
    jj = np.array([1, 2, 0, 3, 5], np.int64)
    d = droid_backends.frame_distance(dev(poses), dev(disps), dev(k), dev(ii), dev(jj), 0.3)
    np.testing.assert_allclose(host(d), og.frame_distance(poses, disps, k, ii, jj, 0.3), rtol=1e-4, atol=1e-3)
    c, v = droid_backends.projmap(dev(poses), dev(disps), dev(k), dev(ii), dev(jj))
    rc, rv = og.projmap(poses, disps, k, ii, jj)
    np.testing.assert_allclose(host(c), rc, atol=2e-3, rtol=1e-4)
    np.testing.assert_array_equal(host(v), rv)
    p = droid_backends.iproj(dev(poses), dev(disps), dev(k))
    np.testing.assert_allclose(host(p), og.iproj(poses, disps, k), rtol=1e-4, atol=1e-4)


def test_depth_filter():
    import droid_backends
    poses, disps, intr = _state(23, N=8)
    k = intr[0]
    ix = np.array([0, 3, 4, 7], np.int64)
    thresh = np.array([0.05, 0.2, 0.5, 1.0], np.float32)
    cnt = droid_backends.depth_filter(dev(poses), dev(disps), dev(k), dev(ix), dev(thresh))
    ref = og.depth_filter(poses, disps, k, ix, thresh)
    assert np.mean(host(cnt) == ref) > 0.995


def test_projective_transform_matches_reference_fixture(golden_dir):
    """The fused HIP reprojection vs the reference's own geom/projective_ops.py
    output (tests/golden/projective_ops.npz, lietorch SE3 stand-in): per-frame
    intrinsics, a stereo edge, the Z clamp and the valid mask."""
    import os
    import droid_backends
    g = np.load(os.path.join(golden_dir, "projective_ops.npz"))
    coords, valid = droid_backends.projective_transform(dev(g["poses"]), dev(g["disps"]), dev(g["intrinsics"]),
                                                        dev(g["ii"]), dev(g["jj"]))
    np.testing.assert_allclose(host(coords), g["coords"], rtol=1e-5, atol=2e-4)
    np.testing.assert_array_equal(host(valid), g["valid"])
