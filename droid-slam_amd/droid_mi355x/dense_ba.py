"""Differentiable dense bundle adjustment for the training path: what
DroidNet.forward calls between update iterations (geom/ba.py:31-157 BA and
MoBA semantics: one damped Gauss-Newton step on the poses (SE3) and inverse
depths, damping H + (ep + lm H) I on the pose block BEFORE the Schur step as
geom/chol.py does, w = 0.001 valid weight, valid = Z > 0.2, Z < 0.1 clamped
to 1, disparities > 10 zeroed and clamped at 0) with gradients to target,
weight and eta - and through the Jacobians to poses and disparities.

Organised the way the device BA is (csrc/ba_kernels.hip), not the way the
reference's Python is:
  * residual and Jacobians per (edge, pixel) in closed form - the twist
    derivative of the projection written out (the per-pixel form of
    droid_kernels.cu:281-330), Ji = -Jj Adj(Gij) via SE3.adjT, Jz = dπ/dh;
  * one 12x12 block and 12-vector per edge from the stacked J = [Ji | Jj],
    scattered into the pose system with a single index_add over the edge's
    four (a, b) pose pairs;
  * the depth coupling kept PER DEPTH FRAME: E_k (6P x HW) holds the pose
    rows that touch frame k, so S = H_damped - sum_k E_k diag(1/C_k) E_k^T
    and its rhs are batched products over frames (no (6P x M HW) matrix);
  * the reduced system solved by _SPDSolve, whose backward reuses the
    Cholesky factor (implicit function theorem: lambda = S^-1 dL/dx,
    dL/dS = -lambda x^T); a failed factorisation gives a zero step and no
    gradient, as the reference's solver.
Runs on torch-ROCm (any device, float32 / float64) over droid_mi355x.lie.SE3;
pinned by tests/golden/geom_ba.npz (the reference's geom/ba.py run in
float64: poses, disparities, gradients w.r.t. target / weight / eta).
"""
import torch

from .lie import SE3

MIN_DEPTH = 0.2
RIG = (-0.1, 0.0, 0.0, 0.0, 0.0, 0.0, 1.0)    # the stereo edge's fixed relative pose


class _SPDSolve(torch.autograd.Function):
    """x = A^-1 b for batched SPD A (B,n,n), b (B,n)."""

    @staticmethod
    def forward(ctx, A, b):
        L, info = torch.linalg.cholesky_ex(A)
        ctx.failed = bool((info != 0).any())
        if ctx.failed:
            return torch.zeros_like(b)
        x = torch.cholesky_solve(b.unsqueeze(-1), L).squeeze(-1)
        ctx.save_for_backward(L, x)
        return x

    @staticmethod
    def backward(ctx, gx):
        if ctx.failed:
            return None, None
        L, x = ctx.saved_tensors
        lam = torch.cholesky_solve(gx.unsqueeze(-1), L).squeeze(-1)
        return -lam.unsqueeze(-1) * x.unsqueeze(-2), lam


def _linearise(target, weight, poses, disps, intrinsics, ii, jj):
    """-> J (B,E,HW,2,12) = [Ji | Jj], Jz (B,E,HW,2), residual r and weight w (B,E,HW,2)."""
    B, _, H, W = disps.shape
    E = ii.shape[0]
    dt, dv = disps.dtype, disps.device
    y, x = torch.meshgrid(torch.arange(H, device=dv, dtype=dt), torch.arange(W, device=dv, dtype=dt), indexing="ij")
    fi, fj = intrinsics[:, ii], intrinsics[:, jj]                        # (B,E,4)
    px = lambda f, k: f[..., k, None, None]
    ray = torch.stack([(x - px(fi, 2)) / px(fi, 0), (y - px(fi, 3)) / px(fi, 1), torch.ones_like(x).expand(B, E, H, W)], -1)
    h = disps[:, ii]                                                     # (B,E,H,W)
    g = (poses[:, jj] * poses[:, ii].inv()).data
    st = (ii == jj).to(dv)
    if bool(st.any()):
        g = torch.where(st[None, :, None], torch.tensor(RIG, device=dv, dtype=dt), g)
    Gij = SE3(g)
    t = g[..., None, None, :3]
    # the point in frame j (homogeneous coordinate = disparity h): R ray + t h
    X1 = Gij[:, :, None, None] * torch.cat([ray, h[..., None]], -1)
    X, Y, Z = X1[..., 0], X1[..., 1], X1[..., 2]
    d = 1.0 / torch.where(Z < 0.5 * MIN_DEPTH, torch.ones_like(Z), Z)
    fx, fy, cx, cy = (px(fj, k) for k in range(4))
    u = fx * X * d + cx
    v = fy * Y * d + cy
    valid = (Z > MIN_DEPTH).to(dt)
    o = torch.zeros_like(d)
    hd, d2 = h * d, d * d
    # d(u, v)/d(twist of frame j), twist [rho, phi], left retraction
    Ju = fx[..., None] * torch.stack([hd, o, -X * h * d2, -X * Y * d2, d * Z + X * X * d2, -Y * d], -1)
    Jv = fy[..., None] * torch.stack([o, hd, -Y * h * d2, -d * Z - Y * Y * d2, X * Y * d2, X * d], -1)
    Jj = torch.stack([Ju, Jv], -2)                                       # (B,E,H,W,2,6)
    Ji = -Gij[:, :, None, None, None].adjT(Jj)
    Jz = torch.stack([fx * (t[..., 0] * d - t[..., 2] * X * d2), fy * (t[..., 1] * d - t[..., 2] * Y * d2)], -1)
    r = target - torch.stack([u, v], -1)
    w = 0.001 * valid[..., None] * weight
    HW = H * W
    J = torch.cat([Ji, Jj], -1).reshape(B, E, HW, 2, 12)
    return J, Jz.reshape(B, E, HW, 2), r.reshape(B, E, HW, 2), w.reshape(B, E, HW, 2)


def _pose_system(J, r, w, pi, pj, P, ep, lm, every_block=False):
    """Damped pose block H (B,6P,6P) and gradient v (B,6P) from the per-edge
    12x12 blocks; edges' pose indices pi / pj (fixed poses: outside [0, P)).
    every_block: damp the diagonal of EVERY 6x6 block (i, j), empty ones
    included - geom/chol.py:block_solve adds (ep + lm H) * eye(6) to the
    (B,P,P,6,6) view (MoBA); schur_solve damps only the 6P diagonal (BA)."""
    B, E = J.shape[:2]
    dt = J.dtype
    blk = torch.einsum("behcm,behc,behcn->bemn", J, w, J)              # (B,E,12,12)
    vec = torch.einsum("behcm,behc,behc->bem", J, w, r)                 # (B,E,12)
    H = torch.zeros(B, P * P, 6, 6, device=J.device, dtype=dt)
    v = torch.zeros(B, P, 6, device=J.device, dtype=dt)
    for a, pa in enumerate((pi, pj)):
        ok_a = (pa >= 0) & (pa < P)
        v = v.index_add(1, pa[ok_a], vec[:, ok_a, 6 * a:6 * a + 6])
        for b, pb in enumerate((pi, pj)):
            ok = ok_a & (pb >= 0) & (pb < P)
            H = H.index_add(1, pa[ok] * P + pb[ok], blk[:, ok, 6 * a:6 * a + 6, 6 * b:6 * b + 6])
    H = H.view(B, P, P, 6, 6)
    if every_block:
        H = H + torch.diag_embed(ep + lm * torch.diagonal(H, dim1=-2, dim2=-1))
    H = H.permute(0, 1, 3, 2, 4).reshape(B, 6 * P, 6 * P)
    if not every_block:
        H = H + torch.diag_embed(ep + lm * torch.diagonal(H, dim1=-2, dim2=-1))   # H + (ep + lm H) I
    return H, v.reshape(B, 6 * P)


def _retract(poses, dx, fixedp, P):
    B, N = poses.shape[:2]
    tau = torch.zeros(B, N, 6, device=dx.device, dtype=dx.dtype)
    tau = torch.cat([tau[:, :fixedp], dx.view(B, P, 6), tau[:, fixedp + P:]], 1)
    return poses.retr(tau)


def BA(target, weight, eta, poses, disps, intrinsics, ii, jj, fixedp=1, rig=1, ep=0.1, lm=1e-4):
    """Full BA step (geom/ba.py:31-106 semantics): target / weight (B,E,H,W,2),
    eta (B,M,H,W) with M = #unique(ii), poses SE3 (B,N), disps (B,N,H,W),
    intrinsics (B,N,4), ii / jj (E) -> (poses, disps)."""
    B, N, H, W = disps.shape
    HW = H * W
    J, Jz, r, w = _linearise(target, weight, poses, disps, intrinsics, ii, jj)
    P = N // rig - fixedp
    pi, pj = ii // rig - fixedp, jj // rig - fixedp
    A, v = _pose_system(J, r, w, pi, pj, P, ep, lm)
    # depth terms, per depth frame k (= unique source frame)
    kx, kk = torch.unique(ii, return_inverse=True)
    M = kx.shape[0]
    wz = w * Jz
    C = torch.zeros(B, M, HW, device=J.device, dtype=J.dtype).index_add(1, kk, (wz * Jz).sum(-1))
    C = C + eta.reshape(B, M, HW) + 1e-7
    wv = torch.zeros_like(C).index_add(1, kk, (wz * r).sum(-1))
    Epix = torch.einsum("behcm,behc->bemh", J, wz)                      # (B,E,12,HW): [Ei; Ej] rows
    Ek = torch.zeros(B, M * P, 6, HW, device=J.device, dtype=J.dtype)
    for a, pa in enumerate((pi, pj)):
        ok = (pa >= 0) & (pa < P)
        Ek = Ek.index_add(1, kk[ok] * P + pa[ok], Epix[:, ok, 6 * a:6 * a + 6])
    Ek = Ek.view(B, M, 6 * P, HW)
    Q = 1.0 / C
    S = A - torch.einsum("bmah,bmh,bmch->bac", Ek, Q, Ek)
    rhs = v - torch.einsum("bmah,bmh->ba", Ek, Q * wv)
    dx = _SPDSolve.apply(S, rhs)
    dz = Q * (wv - torch.einsum("bmah,ba->bmh", Ek, dx))
    poses = _retract(poses, dx, fixedp, P)
    disps = disps.index_add(1, kx, dz.view(B, M, H, W))
    disps = torch.where(disps > 10, torch.zeros_like(disps), disps)
    return poses, disps.clamp(min=0.0)


def MoBA(target, weight, eta, poses, disps, intrinsics, ii, jj, fixedp=1, rig=1, ep=0.1, lm=1e-4):
    """Motion-only BA step (geom/ba.py:109-157 semantics) -> poses."""
    B, N, H, W = disps.shape
    J, _, r, w = _linearise(target, weight, poses, disps, intrinsics, ii, jj)
    P = N // rig - fixedp
    A, v = _pose_system(J, r, w, ii // rig - fixedp, jj // rig - fixedp, P, ep, lm, every_block=True)
    return _retract(poses, _SPDSolve.apply(A, v), fixedp, P)
