"""Pin the BA oracle (a restatement of ba_cuda, which cannot be built here)
against an independent formulation: residuals written with 4x4 matrices and
torch.linalg.matrix_exp, Jacobians by autograd, the full fp64 normal
equations, and an explicit Schur complement."""
import numpy as np
import pytest
import torch
from scipy.spatial.transform import Rotation

from droid_mi355x import synthetic
from oracle import ba as oba
from oracle import se3


def _mat(pose):
    T = torch.eye(4, dtype=torch.float64)
    T[:3, :3] = torch.from_numpy(Rotation.from_quat(pose[3:]).as_matrix())
    T[:3, 3] = torch.from_numpy(pose[:3].astype(np.float64))
    return T


def _exp(xi):
    A = torch.zeros(4, 4, dtype=torch.float64)
    tau, phi = xi[:3], xi[3:]
    A[0, 1], A[0, 2], A[1, 2] = -phi[2], phi[1], -phi[0]
    A[1, 0], A[2, 0], A[2, 1] = phi[2], -phi[1], phi[0]
    A[:3, 3] = tau
    return torch.linalg.matrix_exp(A)


def independent_step(prob, lm, ep):
    poses, disps = prob["poses"].astype(np.float64), prob["disps"].astype(np.float64)
    fx, fy, cx, cy = prob["intrinsics"].astype(np.float64)
    ii, jj, t0, t1 = prob["ii"], prob["jj"], prob["t0"], prob["t1"]
    N, H, W = disps.shape
    HW = H * W
    P = t1 - t0
    kx = np.unique(np.concatenate([np.arange(t0, t1), ii]))
    kpos = {int(f): k for k, f in enumerate(kx)}
    K = len(kx)
    Ts = [_mat(p) for p in poses]
    v, u = np.meshgrid(np.arange(H, dtype=np.float64), np.arange(W, dtype=np.float64), indexing="ij")
    xr = torch.from_numpy(((u - cx) / fx).reshape(-1))
    yr = torch.from_numpy(((v - cy) / fy).reshape(-1))
    tg = torch.from_numpy(prob["targets"].astype(np.float64)).reshape(len(ii), 2, HW)
    wt = torch.from_numpy(prob["weights"].astype(np.float64)).reshape(len(ii), 2, HW)

    def proj_all(x):
        xi = x[:6 * P].reshape(P, 6)
        dz = x[6 * P:].reshape(K, HW)
        out = []
        for e, (i, j) in enumerate(zip(ii, jj)):
            d = torch.from_numpy(disps[i].reshape(-1)) + dz[kpos[int(i)]]
            if i == j:
                Tij = torch.eye(4, dtype=torch.float64)
                Tij[0, 3] = -0.1
            else:
                Ti = _exp(xi[i - t0]) @ Ts[i] if t0 <= i < t1 else Ts[i]
                Tj = _exp(xi[j - t0]) @ Ts[j] if t0 <= j < t1 else Ts[j]
                Tij = Tj @ torch.linalg.inv(Ti)
            X = Tij[:3, :3] @ torch.stack([xr, yr, torch.ones_like(xr)]) + Tij[:3, 3:4] * d
            out.append(torch.stack([fx * X[0] / X[2] + cx, fy * X[1] / X[2] + cy]))
            out.append(X[2:3].expand(2, -1))
        return torch.stack(out[0::2]), torch.stack(out[1::2])

    x0 = torch.zeros(6 * P + K * HW, dtype=torch.float64)
    proj0, Z0 = proj_all(x0)
    J = torch.autograd.functional.jacobian(lambda x: proj_all(x)[0], x0).reshape(-1, x0.numel())
    w = (0.001 * wt * (Z0 >= 0.25)).reshape(-1)
    r = (tg - proj0).reshape(-1)
    Hf = J.T @ (w[:, None] * J)
    g = J.T @ (w * r)
    n = 6 * P
    A, B, Cz = Hf[:n, :n], Hf[:n, n:], Hf[n:, n:]
    off = Cz - torch.diag(torch.diagonal(Cz))
    assert off.abs().max() < 1e-9 * max(1.0, Cz.abs().max())
    c = torch.diagonal(Cz).clone()
    bz = g[n:].clone()
    ds = torch.from_numpy(prob["disps_sens"][kx].astype(np.float64).reshape(-1))
    dd = torch.from_numpy(disps[kx].reshape(-1))
    eta = torch.from_numpy(prob["eta"].astype(np.float64).reshape(-1))
    m = (ds > 0).double()
    c = c + m * 0.05 + (1 - m) * eta
    bz = bz - m * 0.05 * (dd - ds)
    Q = 1.0 / c
    S = A - B @ (Q[:, None] * B.T)
    rhs = g[:n] - B @ (Q * bz)
    S = S + torch.diag(ep + lm * torch.diagonal(S))
    dx = torch.linalg.solve(S, rhs)
    dz = Q * (bz - B.T @ dx)
    return dx.numpy().reshape(P, 6), dz.numpy().reshape(K, HW)


def small_problem(seed=7, stereo=False, sens=0.0):
    ii = np.array([1, 2, 2, 3, 3, 4, 1, 4, 0, 2], dtype=np.int64)
    jj = np.array([2, 1, 3, 2, 4, 3, 3, 2, 1, 4], dtype=np.int64)
    if stereo:
        ii = np.concatenate([ii, [2, 3]])
        jj = np.concatenate([jj, [2, 3]])
    return synthetic.ba_problem("X", H=4, W=6, seed=seed, edges=(ii, jj), num_frames=5, t0=1, t1=5,
                                sens_fraction=sens)


@pytest.mark.parametrize("stereo,sens", [(False, 0.0), (True, 0.0), (False, 0.5)])
def test_oracle_matches_independent_formulation(stereo, sens):
    prob = small_problem(stereo=stereo, sens=sens)
    lm, ep = 1e-4, 0.1
    ref_dx, ref_dz = independent_step(prob, lm, ep)
    out = oba.ba(**{k: prob[k] for k in ("poses", "disps", "intrinsics", "disps_sens", "targets", "weights",
                                          "eta", "ii", "jj", "t0", "t1")},
                 iterations=1, lm=lm, ep=ep, motion_only=False, skip_t0_backsub=False)
    np.testing.assert_allclose(out["dx"], ref_dx, atol=1e-7, rtol=1e-6)
    np.testing.assert_allclose(out["dz"], ref_dz, atol=1e-7, rtol=1e-6)


def test_t0_backsub_quirk_only_touches_rows_of_pose_t0():
    """EvT6x1 skips rows with jj - t0 <= 0 (droid_kernels.cu:1105): dz differs
    from the exact Schur back-substitution exactly in frames that have a row
    whose pose is t0; dx is unaffected."""
    prob = small_problem()
    args = {k: prob[k] for k in ("poses", "disps", "intrinsics", "disps_sens", "targets", "weights", "eta",
                                 "ii", "jj", "t0", "t1")}
    a = oba.ba(**args, iterations=1, lm=1e-4, ep=0.1, motion_only=False, skip_t0_backsub=True)
    b = oba.ba(**args, iterations=1, lm=1e-4, ep=0.1, motion_only=False, skip_t0_backsub=False)
    np.testing.assert_array_equal(a["dx"], b["dx"])
    t0 = prob["t0"]
    affected = set(prob["ii"][prob["jj"] == t0].tolist()) | {t0}
    for k, f in enumerate(a["kx"]):
        same = np.allclose(a["dz"][k], b["dz"][k], atol=1e-14)
        assert same == (int(f) not in affected), f


def test_motion_only_and_failure():
    prob = small_problem()
    args = {k: prob[k] for k in ("poses", "disps", "intrinsics", "disps_sens", "targets", "weights", "eta",
                                 "ii", "jj", "t0", "t1")}
    out = oba.ba(**args, iterations=1, lm=1e-4, ep=0.1, motion_only=True)
    assert out["dz"] is None and out["dx"].shape == (4, 6)
    np.testing.assert_array_equal(out["disps"], prob["disps"].astype(np.float64))
    # negative damping -> not positive definite -> dx = 0 (SparseBlock::solve :1207-1210)
    bad = oba.ba(**args, iterations=1, lm=0.0, ep=-1e9, motion_only=False)
    assert not bad["ok"] and np.all(bad["dx"] == 0)


def test_se3_against_scipy():
    rng = np.random.default_rng(3)
    q = Rotation.random(20, random_state=4).as_quat()
    X = rng.normal(size=(20, 3))
    np.testing.assert_allclose(se3.act_so3(q, X), Rotation.from_quat(q).apply(X), atol=1e-12)
    a, b = Rotation.random(20, random_state=5).as_quat(), Rotation.random(20, random_state=6).as_quat()
    np.testing.assert_allclose(Rotation.from_quat(se3.quat_mul(a, b)).as_matrix(),
                               (Rotation.from_quat(a) * Rotation.from_quat(b)).as_matrix(), atol=1e-12)
    xi = rng.normal(scale=0.3, size=(20, 6))
    t, qq = se3.exp_se3(xi)
    for k in range(20):
        T = _exp(torch.from_numpy(xi[k])).numpy()
        np.testing.assert_allclose(Rotation.from_quat(qq[k]).as_matrix(), T[:3, :3], atol=1e-9)
        np.testing.assert_allclose(t[k], T[:3, 3], atol=1e-9)
    tiny = np.array([[1e-3, 0, 0, 1e-6, 0, 0]])
    t, qq = se3.exp_se3(tiny)
    np.testing.assert_allclose(t[0], tiny[0, :3], atol=1e-12)


def test_projective_transform_matches_ba_linearisation():
    """pops semantics vs the kernel's: both map the same pixel to the same place
    (away from the depth clamps)."""
    from oracle import geometry as og
    prob = small_problem()
    ii, jj = prob["ii"], prob["jj"]
    intr = np.tile(prob["intrinsics"][None], (5, 1))
    coords, valid = og.projective_transform(prob["poses"], prob["disps"], intr, ii, jj)
    ref = synthetic.reproject_np(prob["poses"].astype(np.float64), prob["disps"].astype(np.float64),
                                 prob["intrinsics"].astype(np.float64), ii, jj)
    np.testing.assert_allclose(coords.transpose(0, 3, 1, 2), ref, atol=1e-9)
