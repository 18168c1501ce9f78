"""Dense bundle adjustment restated from `ba_cuda` (numpy, fp64).

Follows /root/reference/src/droid_kernels.cu:
  linearize()  projective_transform_kernel        :176-424
  accum        accum_cuda / accum_kernel          :854-874, :948-998
  schur        schur_block / EEt6x6 / Ev6x1       :1001-1093, :1222-1311
  solve        SparseBlock::solve (SimplicialLLT) :1192-1213 -> dense Cholesky
  backsub      EvT6x1_kernel                      :1095-1115, :1408-1417
  retract      pose_retr_kernel / disp_retr       :877-946
  driver       ba_cuda                            :1314-1434

Quirks reproduced: MIN_DEPTH 0.25, w = 0.001*weight, stereo
tij = (-0.1,0,0) with pose terms zeroed but C/bz kept, damping
`diag += ep + lm*diag` applied to (A - S), back-substitution skips rows whose
pose is t0 (`jj - t0 <= 0`), depth prior alpha=0.05 where disps_sens > 0,
dx = 0 if the factorisation fails, disps updated for every frame of kx.
Sparse-vs-dense: Eigen's SimplicialLLT (AMD ordering) and a dense Cholesky are
the same exact factorisation up to fp64 roundoff.
"""
import os

import numpy as np

from .se3 import adj_se3, act_se3, rel_se3, retr_se3

MIN_DEPTH = 0.25
ALPHA = 0.05


def _threads():
    """worker threads for the per-chunk linearisation (numpy releases the GIL
    in its array kernels): the CPU quota of this process, at most 16."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def linearize(poses, disps, intrinsics, targets, weights, ii, jj, chunk=64):
    """Per-edge Hessian blocks and per-pixel Schur terms (droid_kernels.cu:176-424).

    Returns Hs (4,E,6,6), vs (2,E,6), Eii/Eij (E,6,HW), Cii/bz (E,HW).  Edge
    chunks are independent and linearised on worker threads; the results are
    the same arrays as a serial pass.
    """
    E = len(ii)
    if E > chunk:
        from concurrent.futures import ThreadPoolExecutor
        job = lambda s: _linearize(poses, disps, intrinsics, targets[s:s + chunk], weights[s:s + chunk],
                                   np.asarray(ii)[s:s + chunk], np.asarray(jj)[s:s + chunk])
        with ThreadPoolExecutor(_threads()) as ex:
            parts = list(ex.map(job, range(0, E, chunk)))
        return (np.concatenate([p[0] for p in parts], axis=1), np.concatenate([p[1] for p in parts], axis=1),
                *[np.concatenate([p[k] for p in parts], axis=0) for k in range(2, 6)])
    return _linearize(poses, disps, intrinsics, targets, weights, ii, jj)


def jacobians(poses, disps, intrinsics, ii, jj):
    """Per-pixel reprojection and Jacobians of projective_transform_kernel
    (droid_kernels.cu:281-330): Xj = Tij Xi, d = 1/z (0 where z < MIN_DEPTH),
    Jj rows for u and v, Ji = -Adj(Tij)^T Jj (adjSE3 :147-175), Jz.  Stereo
    edges use Tij = (-0.1,0,0 | identity).  Arrays are (E,HW[,6]); pinned
    against the reference's geom/projective_ops.py (jacobian=True) by
    tests/golden/projective_ops.npz."""
    E = len(ii)
    _, H, W = disps.shape
    HW = H * W
    fx, fy, cx, cy = [float(v) for v in intrinsics]
    ii = np.asarray(ii)
    jj = np.asarray(jj)
    tij, qij = rel_se3(poses[ii, :3], poses[ii, 3:], poses[jj, :3], poses[jj, 3:])
    stereo = ii == jj
    tij[stereo] = [-0.1, 0.0, 0.0]
    qij[stereo] = [0.0, 0.0, 0.0, 1.0]

    v, u = np.meshgrid(np.arange(H, dtype=np.float64), np.arange(W, dtype=np.float64), indexing="ij")
    u = u.reshape(-1)
    v = v.reshape(-1)
    Xi = np.zeros((E, HW, 4))
    Xi[..., 0] = (u - cx) / fx
    Xi[..., 1] = (v - cy) / fy
    Xi[..., 2] = 1.0
    Xi[..., 3] = disps[ii].reshape(E, HW)
    T = tij[:, None, :]
    Q = qij[:, None, :]
    Xj = act_se3(np.broadcast_to(T, (E, HW, 3)), np.broadcast_to(Q, (E, HW, 4)), Xi)
    x, y, z, h = Xj[..., 0], Xj[..., 1], Xj[..., 2], Xj[..., 3]
    bad = z < MIN_DEPTH
    with np.errstate(divide="ignore"):
        d = np.where(bad, 0.0, 1.0 / np.where(bad, 1.0, z))
    d2 = d * d
    zero = np.zeros_like(d)
    Jj_u = fx * np.stack([h * d, zero, -x * h * d2, -x * y * d2, 1 + x * x * d2, -y * d], axis=-1)
    Jj_v = fy * np.stack([zero, h * d, -y * h * d2, -1 - y * y * d2, x * y * d2, x * d], axis=-1)
    Jz_u = fx * (tij[:, 0:1] * d - tij[:, 2:3] * (x * d2))
    Jz_v = fy * (tij[:, 1:2] * d - tij[:, 2:3] * (y * d2))
    TT = np.broadcast_to(T, (E, HW, 3))
    QQ = np.broadcast_to(Q, (E, HW, 4))
    Ji_u = -adj_se3(TT, QQ, Jj_u)
    Ji_v = -adj_se3(TT, QQ, Jj_v)
    return dict(x=x, y=y, z=z, h=h, d=d, bad=bad, stereo=stereo, Jj_u=Jj_u, Jj_v=Jj_v, Ji_u=Ji_u, Ji_v=Ji_v,
                Jz_u=Jz_u, Jz_v=Jz_v, coords=np.stack([fx * d * x + cx, fy * d * y + cy], -1))


def _linearize(poses, disps, intrinsics, targets, weights, ii, jj):
    E = len(ii)
    _, H, W = disps.shape
    HW = H * W
    fx, fy, cx, cy = [float(v) for v in intrinsics]
    J = jacobians(poses, disps, intrinsics, ii, jj)
    x, y, d, bad, stereo = J["x"], J["y"], J["d"], J["bad"], J["stereo"]
    Jj_u, Jj_v, Ji_u, Ji_v, Jz_u, Jz_v = J["Jj_u"], J["Jj_v"], J["Ji_u"], J["Ji_v"], J["Jz_u"], J["Jz_v"]
    tg = targets.reshape(E, 2, HW)
    wt = weights.reshape(E, 2, HW)
    wu = np.where(bad, 0.0, 0.001 * wt[:, 0])
    wv = np.where(bad, 0.0, 0.001 * wt[:, 1])
    ru = tg[:, 0] - (fx * d * x + cx)
    rv = tg[:, 1] - (fy * d * y + cy)

    Cii = wu * Jz_u * Jz_u + wv * Jz_v * Jz_v
    bz = wu * ru * Jz_u + wv * rv * Jz_v

    wu = np.where(stereo[:, None], 0.0, wu)
    wv = np.where(stereo[:, None], 0.0, wv)

    Ju = np.concatenate([Ji_u, Jj_u], axis=-1)   # (E,HW,12)
    Jv = np.concatenate([Ji_v, Jj_v], axis=-1)
    # sum_p w_p J_p J_p^T as batched matmuls (same sums as the reference's per-pixel accumulation)
    H12 = np.matmul((wu[..., None] * Ju).transpose(0, 2, 1), Ju) + np.matmul((wv[..., None] * Jv).transpose(0, 2, 1), Jv)
    v12 = np.matmul((wu * ru)[:, None, :], Ju)[:, 0] + np.matmul((wv * rv)[:, None, :], Jv)[:, 0]

    Hs = np.stack([H12[:, :6, :6], H12[:, :6, 6:], H12[:, 6:, :6], H12[:, 6:, 6:]], axis=0)
    vs = np.stack([v12[:, :6], v12[:, 6:]], axis=0)

    Eii = (wu * Jz_u)[..., None] * Ji_u + (wv * Jz_v)[..., None] * Ji_v   # (E,HW,6)
    Eij = (wu * Jz_u)[..., None] * Jj_u + (wv * Jz_v)[..., None] * Jj_v
    return Hs, vs, Eii.transpose(0, 2, 1), Eij.transpose(0, 2, 1), Cii, bz


def accum(data, ix, jx):
    """accum_cuda droid_kernels.cu:948-998: out[j] = sum_{e: ix[e]==jx[j]} data[e]."""
    out = np.zeros((len(jx),) + data.shape[1:])
    pos = {int(f): k for k, f in enumerate(jx)}
    for e, f in enumerate(np.asarray(ix)):
        k = pos.get(int(f))
        if k is not None:
            out[k] += data[e]
    return out


def _add_blocks(A, blocks, ii, jj, P):
    """SparseBlock::update_lhs :1131-1156 (drops negative block indices)."""
    for n in range(len(ii)):
        i, j = int(ii[n]), int(jj[n])
        if 0 <= i < P and 0 <= j < P:
            A[6 * i:6 * i + 6, 6 * j:6 * j + 6] += blocks[n]


def _add_rhs(b, vecs, ii, P):
    """SparseBlock::update_rhs :1158-1173."""
    for n in range(len(ii)):
        i = int(ii[n])
        if 0 <= i < P:
            b[6 * i:6 * i + 6] += vecs[n]


def solve(A, b, lm, ep):
    """SparseBlock::solve :1192-1213: diag += ep + lm*diag, LLT; dx = 0 on failure.
    (LAPACK potrf + two triangular solves: the same exact factorisation as
    Eigen's SimplicialLLT up to fp64 roundoff, whatever the ordering.)"""
    from scipy.linalg import LinAlgError, cho_factor, cho_solve
    L = A.copy()
    idx = np.arange(A.shape[0])
    L[idx, idx] += ep + lm * L[idx, idx]
    if A.shape[0] == 0:
        return np.zeros(0), True
    try:
        c = cho_factor(L, lower=True, overwrite_a=True, check_finite=False)
    except LinAlgError:
        return np.zeros(A.shape[0]), False
    return cho_solve(c, b, check_finite=False), True


def ba(poses, disps, intrinsics, disps_sens, targets, weights, eta, ii, jj, t0, t1,
       iterations, lm, ep, motion_only, return_system=False, skip_t0_backsub=True):
    """Restatement of ba_cuda (droid_kernels.cu:1314-1434).

    Inputs mirror droid_backends.ba; poses/disps are NOT mutated - updated copies
    are returned.  Returns dict(dx (P,6), dz (K,HW) or None, poses, disps, kx, ok).
    """
    poses = np.array(poses, dtype=np.float64)
    disps = np.array(disps, dtype=np.float64)
    disps_sens = np.asarray(disps_sens, dtype=np.float64)
    targets = np.asarray(targets, dtype=np.float64)
    weights = np.asarray(weights, dtype=np.float64)
    eta = np.asarray(eta, dtype=np.float64)
    ii = np.asarray(ii, dtype=np.int64)
    jj = np.asarray(jj, dtype=np.int64)
    N, H, W = disps.shape
    HW = H * W
    P = t1 - t0
    ts = np.arange(t0, t1)
    ii_exp = np.concatenate([ts, ii])
    jj_exp = np.concatenate([ts, jj])
    kx, kk_exp = np.unique(ii_exp, return_inverse=True)
    dx = dz = None
    ok = True
    system = None
    for _ in range(iterations):
        Hs, vs, Eii, Eij, Cii, bz = linearize(poses, disps, intrinsics, targets, weights, ii, jj)
        A = np.zeros((6 * P, 6 * P))
        b = np.zeros(6 * P)
        _add_blocks(A, Hs.reshape(-1, 6, 6), np.concatenate([ii, ii, jj, jj]) - t0,
                    np.concatenate([ii, jj, ii, jj]) - t0, P)
        _add_rhs(b, vs.reshape(-1, 6), np.concatenate([ii, jj]) - t0, P)
        if motion_only:
            dx, ok = solve(A, b, lm, ep)
            dx = dx.reshape(P, 6)
            t, q = retr_se3(dx, poses[t0:t1, :3], poses[t0:t1, 3:])
            poses[t0:t1] = np.concatenate([t, q], axis=-1)
            system = (A, b)
            continue

        m = (disps_sens[kx] > 0).astype(np.float64).reshape(-1, HW)
        eta2 = eta.reshape(-1, HW)
        if eta2.shape[0] != len(kx) and eta2.shape[0] != 1:
            raise ValueError("eta rows (%d) must equal len(unique([t0,t1) U ii)) = %d"
                             % (eta2.shape[0], len(kx)))
        C = accum(Cii, ii, kx) + m * ALPHA + (1 - m) * eta2
        w = accum(bz, ii, kx) - m * ALPHA * (disps[kx] - disps_sens[kx]).reshape(-1, HW)
        Q = 1.0 / C
        Ei = accum(Eii.reshape(len(ii), 6 * HW), ii, ts).reshape(P, 6, HW)   # (explicit: E may be 0)
        Erows = np.concatenate([Ei, Eij], axis=0)     # (P+E, 6, HW)

        # schur_block :1222-1311 -- pairs of rows sharing a depth map
        S = np.zeros((6 * P, 6 * P))
        rowpose = jj_exp - t0
        live = (jj_exp >= t0) & (jj_exp < t1)
        for k in range(len(kx)):
            rows = np.nonzero((kk_exp == k) & live)[0]
            if len(rows) == 0:
                continue
            Ek = Erows[rows]                          # (r,6,HW)
            Ef = Ek.reshape(-1, Ek.shape[-1])                 # (r*6, HW)
            G = ((Ef * Q[k]) @ Ef.T).reshape(len(rows), 6, len(rows), 6).transpose(0, 2, 1, 3)
            for a, ra in enumerate(rows):
                for c, rc in enumerate(rows):
                    i, j = rowpose[ra], rowpose[rc]
                    S[6 * i:6 * i + 6, 6 * j:6 * j + 6] += G[a, c]
        vS = np.einsum("rnp,rp->rn", Erows, (Q * w)[kk_exp])
        bS = np.zeros(6 * P)
        _add_rhs(bS, vS, rowpose, P)

        dxf, ok = solve(A - S, b - bS, lm, ep)
        dx = dxf.reshape(P, 6)
        system = (A - S, b - bS)

        # EvT6x1 :1095-1115 -- rows with pose index <= 0 (i.e. pose t0) skipped
        use = ((rowpose > 0) if skip_t0_backsub else (rowpose >= 0)) & (rowpose < P)
        dw = np.zeros((len(rowpose), HW))
        dw[use] = np.einsum("rnp,rn->rp", Erows[use], dx[rowpose[use]])
        dz = Q * (w - accum(dw, ii_exp, kx))

        t, q = retr_se3(dx, poses[t0:t1, :3], poses[t0:t1, 3:])
        poses[t0:t1] = np.concatenate([t, q], axis=-1)
        disps[kx] += dz.reshape(-1, H, W)

    out = dict(dx=dx, dz=dz, poses=poses, disps=disps, kx=kx, ok=ok)
    if return_system:
        out["system"] = system
    return out
