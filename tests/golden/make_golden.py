"""Generate golden input/output vectors by importing the REFERENCE's own Python.

Run in the build container only (the reference never travels to the GPU box):

    python tests/golden/make_golden.py

It imports /root/reference/droid_slam with import-only stubs for the
un-vendored / CUDA-only modules (`droid_backends`, `lietorch`) and a
restatement of `torch_scatter.scatter_mean` (third-party, not installed;
restated below as an index_add mean).  Every fixture is
computed in fp32 on CPU by the reference code itself:

  corr_pyramid.npz   CorrBlock(fmap1, fmap2).corr_pyramid   (modules/corr.py:24-38,63-71)
  alt_pyramid.npz    AltCorrBlock(fmaps).pyramid            (modules/corr.py:92-104)
  update_module.npz  UpdateModule.forward(...)              (droid_net.py:111-143, gru.py:19-32)
  convgru.npz        ConvGRU.forward(...)                   (modules/gru.py:19-32)
  cvx_upsample.npz   cvx_upsample(...)                      (droid_net.py:21-35)
  projective_ops.npz projective_transform(..., jacobian=True) (geom/projective_ops.py:96-125)
  proximity.npz      FactorGraph.add_proximity_factors(...)  (factor_graph.py:305-369)
  encoders.npz       BasicEncoder fnet / cnet                (modules/extractor.py, droid_net.py:149-150)
  motion_filter.npz  MotionFilter.track keyframe decisions   (motion_filter.py:45-82)
  geom_ba.npz        geom/ba.py BA / MoBA + their gradients   (geom/ba.py:31-158, geom/chol.py)
  dense_ba.npz       one undamped geom/ba.py BA step          (geom/ba.py:31-106, chol.py:47-75)

lietorch (un-vendored, v0.2) is needed by geom/projective_ops.py as a working
group: `LieStandIn.SE3` below restates the lietorch SE3 operations that file
uses (compose, inverse, action on homogeneous points, adjT) from lietorch's
published definitions, data layout [tx, ty, tz, qx, qy, qz, qw].  The fixture
therefore pins the reference's projective composition and Jacobian chain
(iproj / actp / proj, the stereo override, the depth clamps) against the
oracle's restatement of droid_kernels.cu; the SE3 primitives themselves stay
pinned only by scipy / finite differences.  The reference's
`device="cuda"` literal (projective_ops.py:105) is served by mapping that
device to the CPU while the fixture is computed (torch.as_tensor wrapper);
the reference file itself is imported unmodified.

Weights come from tests/golden/fill.py (RNG-free), inputs from a seeded numpy
generator; both are stored in the fixture so the tests never re-derive them.
"""
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/droid_slam"
sys.path.insert(0, HERE)
from fill import det_fill  # noqa: E402


def _install_stubs():
    for name in ["droid_backends", "lietorch", "torch_scatter"]:
        sys.modules[name] = types.ModuleType(name)
    lt = sys.modules["lietorch"]
    lt.SE3 = lt.Sim3 = lt.SO3 = type("Stub", (), {})

    def scatter_mean(src, index, dim=-1, dim_size=None):
        # torch_scatter.scatter_mean restated: mean of src slices sharing an index.
        dim = dim % src.dim()
        n = int(index.max()) + 1 if dim_size is None else dim_size
        shape = list(src.shape)
        shape[dim] = n
        out = torch.zeros(shape, dtype=src.dtype)
        out.index_add_(dim, index, src)
        cnt = torch.zeros(n, dtype=src.dtype)
        cnt.index_add_(0, index, torch.ones_like(index, dtype=src.dtype))
        view = [1] * src.dim()
        view[dim] = n
        return out / cnt.clamp(min=1).view(view)

    ts = sys.modules["torch_scatter"]
    ts.scatter_mean = scatter_mean
    ts.scatter_sum = None


class LieStandIn:
    """lietorch SE3 semantics (data [t, q_xyzw]) for geom/projective_ops.py."""

    @staticmethod
    def _qmul(a, b):
        av, aw = a[..., :3], a[..., 3:]
        bv, bw = b[..., :3], b[..., 3:]
        return torch.cat([aw * bv + bw * av + torch.cross(av, bv, dim=-1),
                          aw * bw - (av * bv).sum(-1, keepdim=True)], -1)

    @staticmethod
    def _rot(q, X):
        qv, qw = q[..., :3], q[..., 3:]
        uv = 2 * torch.cross(qv.expand_as(X), X, dim=-1)
        return X + qw * uv + torch.cross(qv.expand_as(X), uv, dim=-1)

    class SE3:
        def __init__(self, data):
            self.data = data

        def __getitem__(self, idx):
            return LieStandIn.SE3(self.data[idx])

        def inv(self):
            t, q = self.data[..., :3], self.data[..., 3:]
            qi = torch.cat([-q[..., :3], q[..., 3:]], -1)
            return LieStandIn.SE3(torch.cat([-LieStandIn._rot(qi, t), qi], -1))

        def __mul__(self, other):
            t, q = self.data[..., :3], self.data[..., 3:]
            if isinstance(other, LieStandIn.SE3):      # group product
                t2, q2 = other.data[..., :3], other.data[..., 3:]
                return LieStandIn.SE3(torch.cat([t + LieStandIn._rot(q, t2), LieStandIn._qmul(q, q2)], -1))
            X, w = other[..., :3], other[..., 3:]      # action on homogeneous points [X, w] -> [R X + t w, w]
            return torch.cat([LieStandIn._rot(q, X) + t * w, w], -1)

        def adjT(self, a):
            """Adj(T)^T a for a cotangent a = [a_t, a_r] (lietorch tangent order)."""
            t, q = self.data[..., :3], self.data[..., 3:]
            qi = torch.cat([-q[..., :3], q[..., 3:]], -1)
            at, ar = a[..., :3], a[..., 3:]
            tt = t.expand_as(at)
            return torch.cat([LieStandIn._rot(qi, at), LieStandIn._rot(qi, ar + torch.cross(at, tt, dim=-1))], -1)

        manifold_dim = 6

        @property
        def shape(self):
            return self.data.shape[:-1]

        def retr(self, a):
            """Exp(a) * self, Exp by the matrix exponential of the 4x4 twist
            [[phi]x, rho; 0, 0] (torch.linalg.matrix_exp, differentiable) - an
            evaluation independent of the closed form droid_mi355x.lie uses."""
            rho, phi = a[..., :3], a[..., 3:]
            o = torch.zeros_like(phi[..., 0])
            px, py, pz = phi.unbind(-1)
            hat = torch.stack([torch.stack([o, -pz, py, rho[..., 0]], -1), torch.stack([pz, o, -px, rho[..., 1]], -1),
                               torch.stack([-py, px, o, rho[..., 2]], -1), torch.stack([o, o, o, o], -1)], -2)
            T = torch.linalg.matrix_exp(hat)
            R, t = T[..., :3, :3], T[..., :3, 3]
            qw = 0.5 * torch.sqrt(torch.clamp(1.0 + R[..., 0, 0] + R[..., 1, 1] + R[..., 2, 2], min=1e-12))
            q = torch.stack([(R[..., 2, 1] - R[..., 1, 2]) / (4 * qw), (R[..., 0, 2] - R[..., 2, 0]) / (4 * qw),
                             (R[..., 1, 0] - R[..., 0, 1]) / (4 * qw), qw], -1)
            return LieStandIn.SE3(torch.cat([t, q], -1)) * self

    class Sim3:
        pass


def projective_fixture(rng):
    """geom/projective_ops.py:96-125 with jacobian=True on a small graph with
    temporal, loop and stereo (i == j) edges."""
    sys.modules["lietorch"].SE3 = LieStandIn.SE3
    sys.modules["lietorch"].Sim3 = LieStandIn.Sim3
    import importlib
    import geom.projective_ops as pops
    pops = importlib.reload(pops)   # bind the working SE3 (an earlier import saw the name-only stub)

    N, H, W = 5, 6, 8
    ang = 0.05 * rng.standard_normal((N, 3))
    th = np.linalg.norm(ang, axis=-1, keepdims=True)
    q = np.concatenate([np.sin(th / 2) * ang / th, np.cos(th / 2)], -1)
    t = 0.1 * rng.standard_normal((N, 3)) + np.array([0.0, 0.0, 0.05]) * np.arange(N)[:, None]
    poses = np.concatenate([t, q], -1).astype(np.float32)   # the reference pipeline is fp32 (:105 literal)
    disps = rng.uniform(0.2, 1.0, (N, H, W)).astype(np.float32)
    intr = (np.tile(np.array([6.0, 6.0, 4.0, 3.0]), (N, 1)) * (1 + 0.02 * rng.standard_normal((N, 4)))).astype(np.float32)
    ii = np.array([0, 1, 1, 2, 3, 4, 0, 2], dtype=np.int64)
    jj = np.array([1, 0, 2, 2, 1, 3, 4, 2], dtype=np.int64)     # (2, 2) is a stereo edge
    orig = torch.as_tensor

    def as_tensor_cpu(*a, **k):
        if k.get("device") == "cuda":
            k["device"] = "cpu"
        return orig(*a, **k)

    torch.as_tensor = as_tensor_cpu
    try:
        x1, valid, (Ji, Jj, Jz) = pops.projective_transform(
            LieStandIn.SE3(torch.from_numpy(poses)[None]), torch.from_numpy(disps)[None],
            torch.from_numpy(intr)[None], torch.from_numpy(ii), torch.from_numpy(jj), jacobian=True)
    finally:
        torch.as_tensor = orig
    # the BA kernel takes one intrinsics vector (droid.cpp:88-117): the same graph with intrinsics[0] everywhere
    intr1 = np.tile(intr[:1], (N, 1))
    torch.as_tensor = as_tensor_cpu
    try:
        x1s, valids, (Jis, Jjs, Jzs) = pops.projective_transform(
            LieStandIn.SE3(torch.from_numpy(poses)[None]), torch.from_numpy(disps)[None],
            torch.from_numpy(intr1)[None], torch.from_numpy(ii), torch.from_numpy(jj), jacobian=True)
    finally:
        torch.as_tensor = orig
    np.savez_compressed(os.path.join(HERE, "projective_ops.npz"), poses=poses, disps=disps, intrinsics=intr,
                        ii=ii, jj=jj, coords=x1[0].numpy(), valid=valid[0].numpy(), Ji=Ji[0].numpy(),
                        Jj=Jj[0].numpy(), Jz=Jz[0].numpy(), coords_shared=x1s[0].numpy(),
                        valid_shared=valids[0].numpy(), Ji_shared=Jis[0].numpy(), Jj_shared=Jjs[0].numpy(),
                        Jz_shared=Jzs[0].numpy())


def proximity_fixture(rng):
    """FactorGraph.add_proximity_factors (factor_graph.py:305-369) run by the
    reference itself on stand-in graph state: video.distance returns the stored
    distances, add_factors records the edge list it is handed.  Cases cover the
    static edges with t0 > t1 (the negative-index wrap), stereo, the
    max_factors cap, max_factors = -1, NaN and > 100 distances."""
    sys.modules.setdefault("matplotlib", types.ModuleType("matplotlib"))
    sys.modules.setdefault("matplotlib.pyplot", types.ModuleType("matplotlib.pyplot"))
    from factor_graph import FactorGraph
    from types import SimpleNamespace as NS
    cases = [dict(t=48, t0=0, t1=0, rad=2, nms=2, thresh=16.0, stereo=False, max_factors=100000, ne=60, nan=0),
             dict(t=40, t0=12, t1=6, rad=2, nms=2, thresh=16.0, stereo=True, max_factors=300, ne=40, nan=0),
             dict(t=64, t0=0, t1=0, rad=3, nms=3, thresh=12.0, stereo=False, max_factors=-1, ne=30, nan=0),
             dict(t=56, t0=4, t1=4, rad=2, nms=1, thresh=20.0, stereo=False, max_factors=100000, ne=50, nan=6),
             dict(t=72, t0=0, t1=0, rad=2, nms=2, thresh=16.0, stereo=False, max_factors=500, ne=80, nan=0)]
    out = {}
    for c, cs in enumerate(cases):
        t, t0, t1 = cs["t"], cs["t0"], cs["t1"]
        gi, gj = np.meshgrid(np.arange(t0, t), np.arange(t1, t), indexing="ij")
        # a camera lapping a 16-frame circuit: frames 16 apart see the same place
        ph = np.pi * (gi - gj) / 16.0
        d = (40.0 * np.abs(np.sin(ph)) + rng.uniform(0.0, 6.0, gi.shape) + 0.02 * np.abs(gi - gj)).astype(np.float32)
        d = d.reshape(-1)
        far = rng.choice(d.size, size=d.size // 20, replace=False)
        d[far] = rng.uniform(100.5, 200.0, far.size).astype(np.float32)
        if cs["nan"]:
            d[rng.choice(d.size, size=cs["nan"], replace=False)] = np.nan
        ne = cs["ne"]
        ei = rng.integers(0, t, ne)
        ej = np.clip(ei + rng.integers(-20, 21, ne), 0, t - 1)
        k1, k2 = ne // 2, 3 * ne // 4
        rec = {}
        fake = NS(video=NS(counter=NS(value=t), stereo=cs["stereo"],
                           distance=lambda ii, jj, beta=0.25, _d=d: torch.from_numpy(_d.copy())),
                  ii=torch.from_numpy(ei[:k1]), jj=torch.from_numpy(ej[:k1]),
                  ii_bad=torch.from_numpy(ei[k1:k2]), jj_bad=torch.from_numpy(ej[k1:k2]),
                  ii_inac=torch.from_numpy(ei[k2:]), jj_inac=torch.from_numpy(ej[k2:]),
                  max_factors=cs["max_factors"], device="cpu",
                  add_factors=lambda ii, jj, remove=False: rec.update(ii=ii.numpy().copy(), jj=jj.numpy().copy()))
        FactorGraph.add_proximity_factors(fake, t0=t0, t1=t1, rad=cs["rad"], nms=cs["nms"], beta=0.25,
                                          thresh=cs["thresh"], remove=False)
        out.update({"c%d_%s" % (c, k): np.asarray(v) for k, v in cs.items()})
        out.update({"c%d_d" % c: d, "c%d_ei" % c: ei, "c%d_ej" % c: ej, "c%d_k1" % c: k1, "c%d_k2" % c: k2,
                    "c%d_es_ii" % c: rec["ii"], "c%d_es_jj" % c: rec["jj"]})
    out["ncases"] = len(cases)
    np.savez_compressed(os.path.join(HERE, "proximity.npz"), **out)


def encoder_fixture(rng):
    """BasicEncoder (modules/extractor.py) as DroidNet builds it - fnet
    (128, 'instance') and cnet (256, 'none') - with the deterministic fill, on a
    normalised 2-image batch."""
    from modules.extractor import BasicEncoder
    x = rng.standard_normal((1, 2, 3, 64, 96)).astype(np.float32)
    out = {"x": x}
    for name, dim, norm in (("fnet", 128, "instance"), ("cnet", 256, "none")):
        enc = BasicEncoder(output_dim=dim, norm_fn=norm)
        det_fill(enc)
        out[name] = enc(torch.from_numpy(x)).numpy()
    # DroidNet's parameter names and shapes: the layout droid.pth is saved in
    import droid_net
    sd = droid_net.DroidNet().state_dict()
    out["droidnet_keys"] = np.array(list(sd.keys()))
    out["droidnet_shapes"] = np.array([",".join(map(str, v.shape)) for v in sd.values()])
    np.savez_compressed(os.path.join(HERE, "encoders.npz"), **out)


def motion_filter_fixture(rng):
    """MotionFilter.track (motion_filter.py:45-82) run by the reference on a
    stand-in video: a textured scene translating a little more every frame;
    fnet / cnet / update with the deterministic fill.  The reference's
    droid_backends.corr_index_forward (CUDA) is served by the oracle's
    restatement of correlation_kernels.cu (oracle/corr.py, checked against
    grid_sample); lietorch's SE3.Identity by its data [0,0,0,0,0,0,1]."""
    from types import SimpleNamespace as NS
    sys.path.insert(0, os.path.join(HERE, "..", ".."))
    from oracle import corr as ocorr
    sys.modules.setdefault("cv2", types.ModuleType("cv2"))
    db = sys.modules["droid_backends"]
    db.corr_index_forward = lambda vol, coords, r: [torch.from_numpy(
        ocorr.corr_index_forward(vol.numpy(), coords.numpy(), r))]
    lt = sys.modules["lietorch"]
    lt.SE3.Identity = staticmethod(lambda *a: NS(data=torch.as_tensor([[0, 0, 0, 0, 0, 0, 1.0]])))
    import importlib
    import motion_filter as mf
    mf = importlib.reload(mf)
    import droid_net
    net = droid_net.DroidNet()
    det_fill(net)
    # scene: smooth random texture, frame k translated by shift[k] pixels (x) and shift[k]/2 (y)
    H, W = 128, 192        # 16 x 24 maps: the volume's fourth pooling needs >= 16 rows
    base = rng.uniform(0, 255, (3, H // 4 + 16, W // 4 + 16)).astype(np.float32)
    tex = torch.nn.functional.interpolate(torch.from_numpy(base)[None], scale_factor=4, mode="bilinear",
                                          align_corners=False)[0].numpy()
    shifts = np.array([0, 1, 2, 4, 7, 11, 16, 22, 29, 37], dtype=np.int64)
    frames = np.stack([tex[:, 4 + s // 2: 4 + s // 2 + H, 8 + s: 8 + s + W] for s in shifts]).clip(0, 255).astype(np.uint8)
    intr = torch.as_tensor([50.0, 50.0, W / 2, H / 2])

    def run(thresh):
        appended, feats = [], []
        video = NS(counter=NS(value=0))

        def append(*item):
            appended.append(float(item[0]))
            if len(feats) < 3:
                feats.append((item[6].numpy().copy(), item[7].numpy().copy(), item[8].numpy().copy()))
            video.counter.value += 1
        video.append = append
        f = mf.MotionFilter(net, video, thresh=thresh, device="cpu")
        for k in range(len(frames)):
            f.track(float(k), torch.from_numpy(frames[k])[None], intrinsics=intr)   # (1, 3, H, W) uint8 BGR
        return appended, feats

    # the per-frame mean |delta| the check computes (a spy on its Tensor.norm call)
    orig_norm = torch.Tensor.norm
    seen = []

    def spy(self, *a, **k):
        r = orig_norm(self, *a, **k)
        if k.get("dim") == -1 and self.dim() == 5:
            seen.append(float(r.mean()))
        return r
    torch.Tensor.norm = spy
    out = {"frames": frames, "intrinsics": intr.numpy()}
    try:
        # thresh 0: every frame is a keyframe (motion against the previous frame);
        # thresh inf: none after the first (motion against frame 0).  With the
        # deterministic, untrained weights the motion values differ by ~1 %, so
        # the fixtures pin the values and both branches, not a borderline decision.
        for tag, th in (("all", 0.0), ("none", float("inf"))):
            seen.clear()
            appended, feats = run(th)
            out["motion_" + tag] = np.array(seen)
            out["appended_" + tag] = np.array(appended)
            if tag == "all":
                for q, (g, n_, i_) in enumerate(feats):
                    out["gmap%d" % q], out["net%d" % q], out["inp%d" % q] = g, n_, i_
    finally:
        torch.Tensor.norm = orig_norm
    np.savez_compressed(os.path.join(HERE, "motion_filter.npz"), **out)


def geom_ba_fixture(rng):
    """geom/ba.py BA and MoBA (the differentiable training-path BA, with
    geom/chol.py's implicit-gradient LLT) run by the reference on CPU in
    float64 with the SE3 stand-in, plus the gradients of a fixed linear
    functional of the result w.r.t. target, weight and eta."""
    sys.modules["lietorch"].SE3 = LieStandIn.SE3
    sys.modules["lietorch"].Sim3 = LieStandIn.Sim3

    def scatter_sum(src, index, dim=-1, dim_size=None):
        dim = dim % src.dim()
        n = int(index.max()) + 1 if dim_size is None else dim_size
        shape = list(src.shape)
        shape[dim] = n
        return torch.zeros(shape, dtype=src.dtype).index_add_(dim, index, src)
    sys.modules["torch_scatter"].scatter_sum = scatter_sum
    import importlib
    import geom.projective_ops as pops
    importlib.reload(pops)
    import geom.chol as gchol
    importlib.reload(gchol)
    import geom.ba as gba
    gba = importlib.reload(gba)

    def as_cpu(*a, **k):   # the stereo-edge literal, on the CPU in float64
        k.pop("device", None)
        return torch.tensor(*a, dtype=torch.float64) if not isinstance(a[0], torch.Tensor) else a[0].clone()
    orig = pops.torch.as_tensor
    P, ht, wd = 5, 8, 12
    poses = np.zeros((1, P, 7))
    poses[..., 6] = 1.0
    poses[0, :, 2] = 0.1 * np.arange(P)                       # forward motion
    poses[0, :, :3] += rng.normal(0, 0.02, (P, 3))
    q = rng.normal(0, 0.02, (P, 3))
    poses[0, :, 3:6] = q
    poses[0, :, 6] = np.sqrt(1 - (q ** 2).sum(-1))
    disps = rng.uniform(0.4, 1.0, (1, P, ht, wd))
    intr = np.tile([[10.0, 10.0, wd / 2, ht / 2]], (1, P, 1))
    ii = np.array([0, 1, 1, 2, 2, 3, 3, 4, 0, 4, 2], dtype=np.int64)
    jj = np.array([1, 0, 2, 1, 3, 2, 4, 3, 2, 2, 2], dtype=np.int64)   # last: a stereo (i == j) edge
    E = len(ii)
    tgt = rng.normal(0, 1.0, (1, E, ht, wd, 2))
    wgt = rng.uniform(0.1, 1.0, (1, E, ht, wd, 2))
    kx = np.unique(ii)
    eta = rng.uniform(1e-3, 1e-2, (1, len(kx), ht, wd))
    c_pose = rng.normal(0, 1.0, (1, P, 7))
    c_disp = rng.normal(0, 1.0, (1, P, ht, wd))
    out = dict(poses=poses, disps=disps, intrinsics=intr, ii=ii, jj=jj, eta=eta, c_pose=c_pose, c_disp=c_disp)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64))
    pops.torch.as_tensor = as_cpu   # the reference's device="cuda" literal (projective_ops.py:105) -> CPU
    try:
        with torch.enable_grad():
            Gs = LieStandIn.SE3(T(poses))
            x0 = pops.projective_transform(Gs, T(disps), T(intr), torch.from_numpy(ii), torch.from_numpy(jj))[0]
            target = (x0.detach() + 0.5 * T(tgt)).requires_grad_()   # residuals of a few pixels
            weight = T(wgt).requires_grad_()
            etat = T(eta).requires_grad_()
            p1, d1 = gba.BA(target, weight, etat, Gs, T(disps), T(intr), torch.from_numpy(ii), torch.from_numpy(jj),
                            fixedp=1)
            loss = (p1.data * T(c_pose)).sum() + (d1 * T(c_disp)).sum()
            gt, gw, ge = torch.autograd.grad(loss, [target, weight, etat])
            out.update(target=target.detach().numpy(), weight=weight.detach().numpy(), ba_poses=p1.data.detach().numpy(),
                       ba_disps=d1.detach().numpy(), grad_target=gt.numpy(), grad_weight=gw.numpy(), grad_eta=ge.numpy())
            target2 = target.detach().clone().requires_grad_()
            p2 = gba.MoBA(target2, weight.detach(), etat.detach(), Gs, T(disps), T(intr), torch.from_numpy(ii),
                          torch.from_numpy(jj), fixedp=1)
            g2, = torch.autograd.grad((p2.data * T(c_pose)).sum(), [target2])
            out.update(moba_poses=p2.data.detach().numpy(), moba_grad_target=g2.numpy())
    finally:
        pops.torch.as_tensor = orig
    np.savez_compressed(os.path.join(HERE, "geom_ba.npz"), **out)


def dense_ba_fixture(rng):
    """geom/ba.py BA (one Gauss-Newton step: linearisation, assembly, Schur
    complement, LLT, back-substitution, retraction) with geom/chol.py's
    schur_solve called with ep = lm = 0 - the reference's own functions, only
    the damping defaults changed, because ba_cuda damps A - S after the Schur
    complement (droid_kernels.cu:1117-1219) while schur_solve damps H before it;
    undamped, both compute the same step.  A mono graph with every point in
    front of both cameras beyond both depth cut-offs (geom 0.2, CUDA 0.25), so
    it pins droid_backends.ba / oracle/ba.py's step on the reference's Python."""
    sys.modules["lietorch"].SE3 = LieStandIn.SE3

    def scatter_sum(src, index, dim=-1, dim_size=None):   # torch_scatter.scatter_sum restated
        dim = dim % src.dim()
        n = int(index.max()) + 1 if dim_size is None else dim_size
        shape = list(src.shape)
        shape[dim] = n
        return torch.zeros(shape, dtype=src.dtype).index_add_(dim, index, src)
    sys.modules["torch_scatter"].scatter_sum = scatter_sum
    import functools
    import importlib
    import geom.projective_ops as pops
    importlib.reload(pops)
    import geom.chol as gchol
    importlib.reload(gchol)
    import geom.ba as gba
    gba = importlib.reload(gba)
    gba.schur_solve = functools.partial(gchol.schur_solve, ep=0.0, lm=0.0)
    P, ht, wd = 6, 16, 24
    poses = np.zeros((1, P, 7))
    poses[0, :, 2] = 0.08 * np.arange(P)
    poses[0, :, :3] += rng.normal(0, 0.01, (P, 3))
    q = rng.normal(0, 0.01, (P, 3))
    poses[0, :, 3:6] = q
    poses[0, :, 6] = np.sqrt(1 - (q ** 2).sum(-1))
    disps = rng.uniform(0.4, 1.0, (1, P, ht, wd))
    intr = np.tile([[20.0, 20.0, wd / 2, ht / 2]], (1, P, 1))
    pairs = [(i, j) for i in range(P) for j in range(P) if 1 <= abs(i - j) <= 2]
    ii = np.array([a for a, _ in pairs], dtype=np.int64)
    jj = np.array([b for _, b in pairs], dtype=np.int64)
    E = len(ii)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64))

    def as_cpu(*a, **k):   # the stereo-edge literal (projective_ops.py:105), on the CPU in float64
        k.pop("device", None)
        return torch.tensor(*a, dtype=torch.float64) if not isinstance(a[0], torch.Tensor) else a[0].clone()
    orig = pops.torch.as_tensor
    pops.torch.as_tensor = as_cpu
    try:
        Gs = LieStandIn.SE3(T(poses))
        x0, valid = pops.projective_transform(Gs, T(disps), T(intr), torch.from_numpy(ii), torch.from_numpy(jj))[:2]
        assert bool((valid > 0).all())
        target = x0 + T(rng.normal(0, 0.5, (1, E, ht, wd, 2)))
        weight = T(rng.uniform(0.1, 1.0, (1, E, ht, wd, 2)))
        eta = T(rng.uniform(1e-3, 1e-2, (1, P, ht, wd)))
        p1, d1 = gba.BA(target, weight, eta, Gs, T(disps), T(intr), torch.from_numpy(ii), torch.from_numpy(jj),
                        fixedp=1)
    finally:
        pops.torch.as_tensor = orig
    np.savez_compressed(os.path.join(HERE, "dense_ba.npz"), poses=poses, disps=disps, intrinsics=intr, ii=ii, jj=jj,
                        target=target.numpy(), weight=weight.numpy(), eta=eta.numpy(),
                        ba_poses=p1.data.numpy(), ba_disps=d1.numpy())


def ate_fixture():
    """The reference's own ATE known-answer pair (thirdparty/tartanair_tools/
    evaluation/pose_{gt,est}.txt, data) and ATEEvaluator.evaluate's outputs on
    it (evaluator_base.py:33-55), with and without scale."""
    import contextlib
    import io
    d = os.path.join(os.path.dirname(REF), "thirdparty", "tartanair_tools")
    sys.path.insert(0, d)
    try:
        from evaluation.evaluator_base import ATEEvaluator
    finally:
        sys.path.remove(d)
    gt = np.loadtxt(os.path.join(d, "evaluation", "pose_gt.txt"))
    est = np.loadtxt(os.path.join(d, "evaluation", "pose_est.txt"))
    out = dict(pose_gt=gt, pose_est=est)
    for scale in (True, False):
        with contextlib.redirect_stdout(io.StringIO()) as log:
            err, _, _ = ATEEvaluator().evaluate(gt, est, scale)
        s = [float(l.split(":")[1]) for l in log.getvalue().splitlines() if "ATE scale" in l][0]
        out["ate_scale" if scale else "ate_noscale"] = np.float64(err)
        out["s_scale" if scale else "s_noscale"] = np.float64(s)
    np.savez_compressed(os.path.join(HERE, "tartanair_poses.npz"), **out)


def main():
    _install_stubs()
    sys.path.insert(0, REF)
    from modules.corr import CorrBlock, AltCorrBlock
    from modules.gru import ConvGRU
    import droid_net

    torch.set_grad_enabled(False)
    rng = np.random.default_rng(2024)

    # --- CorrBlock pyramid (all-pairs volume + avg-pool levels) ---------------
    f1 = rng.standard_normal((1, 2, 128, 16, 16)).astype(np.float32)
    f2 = rng.standard_normal((1, 2, 128, 16, 16)).astype(np.float32)
    cb = CorrBlock(torch.from_numpy(f1), torch.from_numpy(f2), num_levels=4, radius=3)
    np.savez_compressed(os.path.join(HERE, "corr_pyramid.npz"), fmap1=f1, fmap2=f2,
                        **{f"level{i}": cb.corr_pyramid[i].numpy() for i in range(4)})

    # --- AltCorrBlock feature pyramid -----------------------------------------
    fm = rng.standard_normal((1, 3, 128, 16, 16)).astype(np.float32)
    ab = AltCorrBlock(torch.from_numpy(fm), num_levels=4, radius=3)
    np.savez_compressed(os.path.join(HERE, "alt_pyramid.npz"), fmaps=fm,
                        **{f"level{i}": ab.pyramid[i].numpy() for i in range(4)})

    # --- ConvGRU (small planes) ------------------------------------------------
    gru = ConvGRU(16, 24)
    det_fill(gru)
    h = np.tanh(rng.standard_normal((2, 16, 6, 8))).astype(np.float32)
    x1 = rng.standard_normal((2, 10, 6, 8)).astype(np.float32)
    x2 = rng.standard_normal((2, 14, 6, 8)).astype(np.float32)
    out = gru(torch.from_numpy(h), torch.from_numpy(x1), torch.from_numpy(x2))
    np.savez_compressed(os.path.join(HERE, "convgru.npz"), h=h, x1=x1, x2=x2, out=out.numpy())

    # --- UpdateModule (full planes, tiny spatial size) -------------------------
    um = droid_net.UpdateModule()
    det_fill(um)
    E, H, W = 5, 6, 8
    net = np.tanh(rng.standard_normal((1, E, 128, H, W))).astype(np.float32)
    inp = np.maximum(rng.standard_normal((1, E, 128, H, W)), 0).astype(np.float32)
    corr = rng.standard_normal((1, E, 196, H, W)).astype(np.float32)
    flow = np.clip(4.0 * rng.standard_normal((1, E, 4, H, W)), -64, 64).astype(np.float32)
    ii = np.array([0, 0, 1, 2, 2], dtype=np.int64)
    jj = np.array([1, 2, 0, 1, 3], dtype=np.int64)
    net_o, delta, weight, eta, upmask = um(
        torch.from_numpy(net), torch.from_numpy(inp), torch.from_numpy(corr),
        torch.from_numpy(flow), torch.from_numpy(ii), torch.from_numpy(jj))
    np.savez_compressed(os.path.join(HERE, "update_module.npz"), net=net, inp=inp, corr=corr,
                        flow=flow, ii=ii, jj=jj, net_out=net_o.numpy(), delta=delta.numpy(),
                        weight=weight.numpy(), eta=eta.numpy(), upmask=upmask.numpy())

    # --- convex upsampling (used by DepthVideo.upsample) -----------------------
    data = rng.standard_normal((2, 6, 8, 1)).astype(np.float32)
    mask = rng.standard_normal((2, 576, 6, 8)).astype(np.float32)
    up = droid_net.cvx_upsample(torch.from_numpy(data), torch.from_numpy(mask))
    np.savez_compressed(os.path.join(HERE, "cvx_upsample.npz"), data=data, mask=mask, up=up.numpy())

    # --- projective transform + Jacobians (BA linearisation) -----------------
    projective_fixture(np.random.default_rng(2025))

    # --- proximity edges (global-backend edge rebuild) --------------------------
    proximity_fixture(np.random.default_rng(2026))

    # --- MotionFilter: feature encoders and the keyframe check -----------------
    encoder_fixture(np.random.default_rng(2027))
    motion_filter_fixture(np.random.default_rng(2028))

    # --- differentiable BA (training path) --------------------------------------
    geom_ba_fixture(np.random.default_rng(2029))

    # --- the dense BA step, undamped, from geom/ba.py (pins droid_backends.ba) --
    dense_ba_fixture(np.random.default_rng(2030))

    # --- ATE known answer (the trajectory-level "ATE vs ref" evaluator) ---------
    ate_fixture()
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
