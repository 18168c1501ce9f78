"""The differentiable bundle adjustment of the training path (geom/ba.py:31-158,
geom/chol.py, geom/projective_ops.py:18-125) on torch-ROCm, lietorch-free
(droid_mi355x.lie.SE3): the same Jacobians, damping, Schur complement, LLT
solve with the implicit backward (CholeskySolver) and retraction, so gradients
flow from the BA's poses / disparities back to the update operator's targets,
weights and damping as in DroidNet.forward.  The inference path never uses
it (droid_backends.ba is the fused device solve); the torch_scatter
scatter_sum the reference imports is restated as index_add.
"""
import torch

from .lie import SE3

MIN_DEPTH = 0.2


def _scatter_sum(src, index, dim, dim_size):
    shape = list(src.shape)
    shape[dim] = dim_size
    return torch.zeros(shape, dtype=src.dtype, device=src.device).index_add_(dim, index, src)


# ---- projective_ops.py:18-125 -------------------------------------------------
def _intr(intrinsics):
    return intrinsics[..., None, None, :].unbind(dim=-1)


def iproj(disps, intrinsics, jacobian=False):
    ht, wd = disps.shape[2:]
    fx, fy, cx, cy = _intr(intrinsics)
    y, x = torch.meshgrid(torch.arange(ht, device=disps.device, dtype=disps.dtype),
                          torch.arange(wd, device=disps.device, dtype=disps.dtype), indexing="ij")
    i = torch.ones_like(disps)
    pts = torch.stack([(x - cx) / fx, (y - cy) / fy, i, disps], dim=-1)
    if jacobian:
        J = torch.zeros_like(pts)
        J[..., -1] = 1.0
        return pts, J
    return pts, None


def proj(Xs, intrinsics, jacobian=False):
    fx, fy, cx, cy = _intr(intrinsics)
    X, Y, Z, D = Xs.unbind(dim=-1)
    Z = torch.where(Z < 0.5 * MIN_DEPTH, torch.ones_like(Z), Z)
    d = 1.0 / Z
    coords = torch.stack([fx * (X * d) + cx, fy * (Y * d) + cy], dim=-1)
    if jacobian:
        B, N, H, W = d.shape
        o = torch.zeros_like(d)
        J = torch.stack([fx * d, o, -fx * X * d * d, o, o, fy * d, -fy * Y * d * d, o], dim=-1).view(B, N, H, W, 2, 4)
        return coords, J
    return coords, None


def actp(Gij, X0, jacobian=False):
    X1 = Gij[:, :, None, None] * X0
    if jacobian:
        X, Y, Z, d = X1.unbind(dim=-1)
        o = torch.zeros_like(d)
        B, N, H, W = d.shape
        Ja = torch.stack([d, o, o, o, Z, -Y,
                          o, d, o, -Z, o, X,
                          o, o, d, Y, -X, o,
                          o, o, o, o, o, o], dim=-1).view(B, N, H, W, 4, 6)
        return X1, Ja
    return X1, None


def projective_transform(poses, depths, intrinsics, ii, jj, jacobian=False):
    """map points from ii -> jj (stereo edges ii == jj use the fixed rig baseline)."""
    X0, Jz = iproj(depths[:, ii], intrinsics[:, ii], jacobian=jacobian)
    gd = (poses[:, jj] * poses[:, ii].inv()).data
    stereo = (ii == jj).to(gd.device)
    if bool(stereo.any()):
        rig = torch.as_tensor([-0.1, 0.0, 0.0, 0.0, 0.0, 0.0, 1.0], device=gd.device, dtype=gd.dtype)
        gd = torch.where(stereo[None, :, None], rig, gd)
    Gij = SE3(gd)
    X1, Ja = actp(Gij, X0, jacobian=jacobian)
    x1, Jp = proj(X1, intrinsics[:, jj], jacobian=jacobian)
    valid = ((X1[..., 2] > MIN_DEPTH) & (X0[..., 2] > MIN_DEPTH)).to(x1.dtype).unsqueeze(-1)
    if jacobian:
        Jj = torch.matmul(Jp, Ja)
        Ji = -Gij[:, :, None, None, None].adjT(Jj)
        Jz = Gij[:, :, None, None] * Jz
        Jz = torch.matmul(Jp, Jz.unsqueeze(-1))
        return x1, valid, (Ji, Jj, Jz)
    return x1, valid


# ---- chol.py ---------------------------------------------------------------
class CholeskySolver(torch.autograd.Function):
    """x = H^-1 b with the implicit backward: dz = H^-1 grad, dH = -x dz^T;
    a failed factorisation returns zeros and no gradient (chol.py:5-31)."""

    @staticmethod
    def forward(ctx, H, b):
        U, info = torch.linalg.cholesky_ex(H)
        ctx.failed = bool((info != 0).any())
        if ctx.failed:
            return torch.zeros_like(b)
        xs = torch.cholesky_solve(b, U)
        ctx.save_for_backward(U, xs)
        return xs

    @staticmethod
    def backward(ctx, grad_x):
        if ctx.failed:
            return None, None
        U, xs = ctx.saved_tensors
        dz = torch.cholesky_solve(grad_x, U)
        return -torch.matmul(xs, dz.transpose(-1, -2)), dz


def block_solve(H, b, ep=0.1, lm=0.0001):
    B, N, _, D, _ = H.shape
    I = torch.eye(D, device=H.device, dtype=H.dtype)
    H = H + (ep + lm * H) * I
    H = H.permute(0, 1, 3, 2, 4).reshape(B, N * D, N * D)
    x = CholeskySolver.apply(H, b.reshape(B, N * D, 1))
    return x.reshape(B, N, D)


def schur_solve(H, E, C, v, w, ep=0.1, lm=0.0001, sless=False):
    B, P, M, D, HW = E.shape
    H = H.permute(0, 1, 3, 2, 4).reshape(B, P * D, P * D)
    E = E.permute(0, 1, 3, 2, 4).reshape(B, P * D, M * HW)
    Q = (1.0 / C).view(B, M * HW, 1)
    I = torch.eye(P * D, device=H.device, dtype=H.dtype)
    H = H + (ep + lm * H) * I
    v = v.reshape(B, P * D, 1)
    w = w.reshape(B, M * HW, 1)
    Et = E.transpose(1, 2)
    S = H - torch.matmul(E, Q * Et)
    v = v - torch.matmul(E, Q * w)
    dx = CholeskySolver.apply(S, v)
    if sless:
        return dx.reshape(B, P, D)
    dz = Q * (w - Et @ dx)
    return dx.reshape(B, P, D), dz.reshape(B, M, HW)


# ---- ba.py -------------------------------------------------------------------
def safe_scatter_add_mat(A, ii, jj, n, m):
    v = (ii >= 0) & (jj >= 0) & (ii < n) & (jj < m)
    return _scatter_sum(A[:, v], ii[v] * m + jj[v], 1, n * m)


def safe_scatter_add_vec(b, ii, n):
    v = (ii >= 0) & (ii < n)
    return _scatter_sum(b[:, v], ii[v], 1, n)


def disp_retr(disps, dz, ii):
    return disps + _scatter_sum(dz, ii.to(dz.device), 1, disps.shape[1])


def pose_retr(poses, dx, ii):
    return poses.retr(_scatter_sum(dx, ii.to(dx.device), 1, poses.shape[1]))


def _linearise(target, weight, poses, disps, intrinsics, ii, jj):
    B, P, ht, wd = disps.shape
    N = ii.shape[0]
    D = SE3.manifold_dim
    coords, valid, (Ji, Jj, Jz) = projective_transform(poses, disps, intrinsics, ii, jj, jacobian=True)
    r = (target - coords).view(B, N, -1, 1)
    w = .001 * (valid * weight).view(B, N, -1, 1)
    Ji = Ji.reshape(B, N, -1, D)
    Jj = Jj.reshape(B, N, -1, D)
    wJiT = (w * Ji).transpose(2, 3)
    wJjT = (w * Jj).transpose(2, 3)
    return B, P, ht, wd, N, D, r, w, Ji, Jj, Jz, wJiT, wJjT


def BA(target, weight, eta, poses, disps, intrinsics, ii, jj, fixedp=1, rig=1):
    """Full bundle adjustment (ba.py:31-106): one damped Gauss-Newton step on
    poses (SE3, (B, P)) and disparities (B, P, ht, wd)."""
    B, P, ht, wd, N, D, r, w, Ji, Jj, Jz, wJiT, wJjT = _linearise(target, weight, poses, disps, intrinsics, ii, jj)
    Jz = Jz.reshape(B, N, ht * wd, -1)
    Hii, Hij = torch.matmul(wJiT, Ji), torch.matmul(wJiT, Jj)
    Hji, Hjj = torch.matmul(wJjT, Ji), torch.matmul(wJjT, Jj)
    vi = torch.matmul(wJiT, r).squeeze(-1)
    vj = torch.matmul(wJjT, r).squeeze(-1)
    Ei = (wJiT.view(B, N, D, ht * wd, -1) * Jz[:, :, None]).sum(dim=-1)
    Ej = (wJjT.view(B, N, D, ht * wd, -1) * Jz[:, :, None]).sum(dim=-1)
    w = w.view(B, N, ht * wd, -1)
    r = r.view(B, N, ht * wd, -1)
    wk = torch.sum(w * r * Jz, dim=-1)
    Ck = torch.sum(w * Jz * Jz, dim=-1)
    kx, kk = torch.unique(ii, return_inverse=True)
    M = kx.shape[0]
    P = P // rig - fixedp
    ii = ii // rig - fixedp
    jj = jj // rig - fixedp
    H = (safe_scatter_add_mat(Hii, ii, ii, P, P) + safe_scatter_add_mat(Hij, ii, jj, P, P) +
         safe_scatter_add_mat(Hji, jj, ii, P, P) + safe_scatter_add_mat(Hjj, jj, jj, P, P))
    E = safe_scatter_add_mat(Ei, ii, kk, P, M) + safe_scatter_add_mat(Ej, jj, kk, P, M)
    v = safe_scatter_add_vec(vi, ii, P) + safe_scatter_add_vec(vj, jj, P)
    C = safe_scatter_add_vec(Ck, kk, M)
    w = safe_scatter_add_vec(wk, kk, M)
    C = C + eta.view(*C.shape) + 1e-7
    H = H.view(B, P, P, D, D)
    E = E.view(B, P, M, D, ht * wd)
    dx, dz = schur_solve(H, E, C, v, w)
    poses = pose_retr(poses, dx, torch.arange(P, device=dx.device) + fixedp)
    disps = disp_retr(disps, dz.view(B, -1, ht, wd), kx)
    disps = torch.where(disps > 10, torch.zeros_like(disps), disps)
    return poses, disps.clamp(min=0.0)


def MoBA(target, weight, eta, poses, disps, intrinsics, ii, jj, fixedp=1, rig=1):
    """Motion-only bundle adjustment (ba.py:108-158)."""
    B, P, ht, wd, N, D, r, w, Ji, Jj, Jz, wJiT, wJjT = _linearise(target, weight, poses, disps, intrinsics, ii, jj)
    Hii, Hij = torch.matmul(wJiT, Ji), torch.matmul(wJiT, Jj)
    Hji, Hjj = torch.matmul(wJjT, Ji), torch.matmul(wJjT, Jj)
    vi = torch.matmul(wJiT, r).squeeze(-1)
    vj = torch.matmul(wJjT, r).squeeze(-1)
    P = P // rig - fixedp
    ii = ii // rig - fixedp
    jj = jj // rig - fixedp
    H = (safe_scatter_add_mat(Hii, ii, ii, P, P) + safe_scatter_add_mat(Hij, ii, jj, P, P) +
         safe_scatter_add_mat(Hji, jj, ii, P, P) + safe_scatter_add_mat(Hjj, jj, jj, P, P))
    v = safe_scatter_add_vec(vi, ii, P) + safe_scatter_add_vec(vj, jj, P)
    dx = block_solve(H.view(B, P, P, D, D), v)
    return pose_retr(poses, dx, torch.arange(P, device=dx.device) + fixedp)
