"""SE3 on torch tensors, differentiable (autograd through every op) - what the
differentiable BA (geom/ba.py, geom/projective_ops.py) uses of lietorch (the
un-vendored lietorch 0.2).  Data layout as lietorch:
[tx, ty, tz, qx, qy, qz, qw]; tangent vectors [rho (translation), phi
(rotation)]; retr(a) = Exp(a) * X (left retraction, lietorch's `retr`).
"""
import torch


def _qmul(a, b):
    av, aw = a[..., :3], a[..., 3:]
    bv, bw = b[..., :3], b[..., 3:]
    return torch.cat([aw * bv + bw * av + torch.cross(av, bv, dim=-1), aw * bw - (av * bv).sum(-1, keepdim=True)], -1)


def _qrot(q, x):
    """rotate 3-vectors x by unit quaternions q (xyzw)."""
    qv, qw = q[..., :3], q[..., 3:]
    uv = 2.0 * torch.cross(qv.expand_as(x), x, dim=-1)
    return x + qw * uv + torch.cross(qv.expand_as(x), uv, dim=-1)


def _qinv(q):
    return torch.cat([-q[..., :3], q[..., 3:]], -1)


class SE3:
    manifold_dim = 6
    embedded_dim = 7

    def __init__(self, data):
        self.data = data

    @staticmethod
    def Identity(*batch, device=None, dtype=torch.float32):
        d = torch.zeros(tuple(batch) + (7,), device=device, dtype=dtype)
        d[..., 6] = 1.0
        return SE3(d)

    @property
    def shape(self):
        return self.data.shape[:-1]

    def __getitem__(self, idx):
        return SE3(self.data[idx])

    def inv(self):
        t, q = self.data[..., :3], self.data[..., 3:]
        qi = _qinv(q)
        return SE3(torch.cat([-_qrot(qi, t), qi], -1))

    def __mul__(self, other):
        t, q = self.data[..., :3], self.data[..., 3:]
        if isinstance(other, SE3):   # group product
            t2, q2 = other.data[..., :3], other.data[..., 3:]
            return SE3(torch.cat([t + _qrot(q, t2), _qmul(q, q2)], -1))
        # action on homogeneous points [X, Y, Z, W]: R p + t W
        p, w = other[..., :3], other[..., 3:]
        return torch.cat([_qrot(q, p) + t * w, w], -1)

    def adjT(self, a):
        """dual adjoint Adj(g)^T on tangent row vectors a (..., 6)."""
        t, q = self.data[..., :3], self.data[..., 3:]
        qi = _qinv(q)
        at, ar = a[..., :3], a[..., 3:]
        return torch.cat([_qrot(qi, at), _qrot(qi, ar + torch.cross(at, t.expand_as(at), dim=-1))], -1)

    @staticmethod
    def exp(tau):
        """Exp: tangent (..., 6) = [rho, phi] -> SE3 (Sophus / lietorch closed form)."""
        rho, phi = tau[..., :3], tau[..., 3:]
        th2 = (phi * phi).sum(-1, keepdim=True)
        small = th2 < 1e-8
        # the closed forms are evaluated at a benign angle where the Taylor
        # branch is taken, so neither branch (nor its gradient) is ever 0/0
        th2s = torch.where(small, torch.ones_like(th2), th2)
        th = torch.sqrt(th2s)
        # quaternion of the rotation
        s_half = torch.where(small, 0.5 - th2 / 48.0, torch.sin(0.5 * th) / th)
        c_half = torch.where(small, 1.0 - th2 / 8.0, torch.cos(0.5 * th))
        q = torch.cat([s_half * phi, c_half], -1)
        # V = I + A [phi]x + B [phi]x^2
        A = torch.where(small, 0.5 - th2 / 24.0, (1.0 - torch.cos(th)) / th2s)
        Bc = torch.where(small, 1.0 / 6.0 - th2 / 120.0, (th - torch.sin(th)) / (th2s * th))
        px = torch.cross(phi, rho, dim=-1)
        pxx = torch.cross(phi, px, dim=-1)
        t = rho + A * px + Bc * pxx
        return SE3(torch.cat([t, q], -1))

    def retr(self, a):
        return SE3.exp(a) * self
