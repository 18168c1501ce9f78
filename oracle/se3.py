"""SE3 / quaternion arithmetic of the reference device code, vectorised numpy.

Layout: pose = [tx, ty, tz, qx, qy, qz, qw] (lietorch convention, scalar-last
Hamilton quaternion), twist = [tau(3), phi(3)].  Each function follows the
CUDA helper it names in /root/reference/src/droid_kernels.cu.
"""
import numpy as np


def cross(a, b):
    return np.stack([a[..., 1] * b[..., 2] - a[..., 2] * b[..., 1],
                     a[..., 2] * b[..., 0] - a[..., 0] * b[..., 2],
                     a[..., 0] * b[..., 1] - a[..., 1] * b[..., 0]], axis=-1)


def act_so3(q, X):
    """actSO3 droid_kernels.cu:58-68 (also Eigen's _transformVector used by lietorch)."""
    qv, qw = q[..., :3], q[..., 3:4]
    uv = 2.0 * cross(qv, X)
    return X + qw * uv + cross(qv, uv)


def act_se3(t, q, X4):
    """actSE3 droid_kernels.cu:70-77: homogeneous point [X, W] -> [R X + t W, W]."""
    Y = act_so3(q, X4[..., :3]) + X4[..., 3:4] * t
    return np.concatenate([Y, X4[..., 3:4]], axis=-1)


def quat_conj(q):
    return np.concatenate([-q[..., :3], q[..., 3:4]], axis=-1)


def quat_mul(a, b):
    """Hamilton product a (x) b, scalar-last."""
    av, aw = a[..., :3], a[..., 3:4]
    bv, bw = b[..., :3], b[..., 3:4]
    v = aw * bv + bw * av + cross(av, bv)
    w = aw * bw - np.sum(av * bv, axis=-1, keepdims=True)
    return np.concatenate([v, w], axis=-1)


def rel_se3(ti, qi, tj, qj):
    """relSE3 droid_kernels.cu:96-107: Tij = Tj * Ti^-1 with qij = qj (x) qi^-1,
    tij = tj - R(qij) ti."""
    qij = quat_mul(qj, quat_conj(qi))
    tij = tj - act_so3(qij, ti)
    return tij, qij


def adj_se3(t, q, X):
    """adjSE3 droid_kernels.cu:79-94 (maps a 6-vector of Jj rows to Ji rows)."""
    qinv = quat_conj(q)
    Y0 = act_so3(qinv, X[..., :3])
    Y1 = act_so3(qinv, X[..., 3:])
    u = np.stack([t[..., 2] * X[..., 1] - t[..., 1] * X[..., 2],
                  t[..., 0] * X[..., 2] - t[..., 2] * X[..., 0],
                  t[..., 1] * X[..., 0] - t[..., 0] * X[..., 1]], axis=-1)
    return np.concatenate([Y0, Y1 + act_so3(qinv, u)], axis=-1)


def exp_so3(phi):
    """expSO3 droid_kernels.cu:110-132 (Taylor branch for theta^2 < 1e-8)."""
    th2 = np.sum(phi * phi, axis=-1, keepdims=True)
    th4 = th2 * th2
    th = np.sqrt(th2)
    small = th2 < 1e-8
    with np.errstate(invalid="ignore", divide="ignore"):
        imag = np.where(small, 0.5 - th2 / 48.0 + th4 / 3840.0, np.sin(0.5 * th) / np.where(small, 1.0, th))
    real = np.where(small, 1.0 - th2 / 8.0 + th4 / 384.0, np.cos(0.5 * th))
    return np.concatenate([imag * phi, real], axis=-1)


def exp_se3(xi):
    """expSE3 droid_kernels.cu:147-175: left-Jacobian translation, applied only
    when theta > 1e-4."""
    q = exp_so3(xi[..., 3:])
    tau, phi = xi[..., :3], xi[..., 3:]
    th2 = np.sum(phi * phi, axis=-1, keepdims=True)
    th = np.sqrt(th2)
    big = th > 1e-4
    safe_th = np.where(big, th, 1.0)
    a = (1.0 - np.cos(safe_th)) / (safe_th * safe_th)
    b = (safe_th - np.sin(safe_th)) / (safe_th * safe_th * safe_th)
    c1 = cross(phi, tau)
    c2 = cross(phi, c1)
    t = tau + np.where(big, a * c1 + b * c2, 0.0)
    return t, q


def retr_se3(xi, t, q):
    """retrSE3 droid_kernels.cu:877-895: T <- Exp(xi) * T (left retraction)."""
    dt, dq = exp_se3(xi)
    q1 = quat_mul(dq, q)
    t1 = act_so3(dq, t) + dt
    return t1, q1


def pose_mul(a, b):
    """lietorch SE3 composition a * b on [t, q] vectors."""
    return np.concatenate([a[..., :3] + act_so3(a[..., 3:], b[..., :3]),
                           quat_mul(a[..., 3:], b[..., 3:])], axis=-1)


def pose_inv(a):
    qi = quat_conj(a[..., 3:])
    return np.concatenate([-act_so3(qi, a[..., :3]), qi], axis=-1)
