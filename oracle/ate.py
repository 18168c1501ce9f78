"""Absolute trajectory error (ATE) restated from the TartanAir tools vendored
in the reference (TEST INFRASTRUCTURE ONLY, see oracle/__init__.py):

  ATEEvaluator.evaluate   thirdparty/tartanair_tools/evaluation/evaluator_base.py:33-55
  align (Horn / Umeyama)  thirdparty/tartanair_tools/evaluation/evaluate_ate_scale.py:46-100

The reference aligns the ground-truth positions ("model") onto the estimate
("data"): rotation from the SVD of the centred cross-covariance, with the
reflection fixed; with `scale` the ESTIMATE is scaled by
s = sum |model_c|^2 / sum <data_c, R model_c> (evaluate_ate_scale.py:72-83, the
"scale the est to the gt" variant), the translation t = s mean(data) -
R mean(model), and the ATE is the RMS of |R model + t - s data|.
Pinned by tests/test_oracle_golden.py against the reference's own fixture
pair (pose_gt.txt / pose_est.txt, 734 poses, tests/golden/tartanair_poses.npz):
0.8344983411575012 with scale (s = 1.0782526734172067), 1.204507439280004
without.
"""
import numpy as np


def align(gt_xyz, est_xyz, scale):
    """gt_xyz, est_xyz (n, 3) -> (R (3,3), t (3,), per-pose error (n,), s)."""
    m = np.asarray(gt_xyz, np.float64)
    d = np.asarray(est_xyz, np.float64)
    mc = m - m.mean(0)
    dc = d - d.mean(0)
    cov = dc.T @ mc                          # = W^T with W = sum_k mc_k dc_k^T
    U, _, Vh = np.linalg.svd(cov)
    fix = np.eye(3)
    if np.linalg.det(U) * np.linalg.det(Vh) < 0:
        fix[2, 2] = -1.0
    R = U @ fix @ Vh
    s = float(np.sum(mc * mc) / np.sum(dc * (mc @ R.T))) if scale else 1.0
    t = s * d.mean(0) - R @ m.mean(0)
    err = np.linalg.norm(m @ R.T + t - s * d, axis=1)
    return R, t, err, s


def ate(gt_traj, est_traj, scale):
    """ATEEvaluator.evaluate's error on (n, 7) [t, q] trajectories (positions only)
    -> (rmse, s)."""
    _, _, err, s = align(np.asarray(gt_traj)[:, :3], np.asarray(est_traj)[:, :3], scale)
    return float(np.sqrt(np.mean(err * err))), s


def camera_centres(poses):
    """world->camera [t, q_xyzw] poses (DepthVideo.poses) -> camera centres
    c = -R^T t in the world frame (the trajectory the evaluation scripts
    compare: droid.py:terminate returns the inverted poses)."""
    p = np.asarray(poses, np.float64)
    t, q = p[:, :3], p[:, 3:]
    qv, qw = -q[:, :3], q[:, 3:]             # conjugate = inverse rotation
    uv = 2.0 * np.cross(qv, t)
    return -(t + qw * uv + np.cross(qv, uv))
