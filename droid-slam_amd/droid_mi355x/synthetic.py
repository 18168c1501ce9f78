"""Synthetic frame graphs and states for the BASELINE configs.

Seeds: numpy.random.default_rng(1000 + config_id).  Intrinsics at 1/8
resolution [32, 32, 32, 24] (TartanAir 0.8*[320,320,320,240]/8); world->cam
poses [t, q_xyzw] along a smooth forward trajectory (0.05 m/KF along z, yaw
sigma 0.01 rad/KF, T0 = identity); GT disparities a smooth random field in
[0.2, 1.0]; BA targets = reproject(GT) + N(0, 0.5 px); the optimised state is
the GT perturbed by sigma_t 0.01 m, sigma_R 0.005 rad, disps*(1 + 0.05 N(0,1));
weights ~ U(0,1); eta = 0.2*U(1e-3, 1e-2) + 1e-7.  Pure numpy (no device),
shared by tests, bench.py and the CPU baseline.
"""
import numpy as np

INTRINSICS = np.array([32.0, 32.0, 32.0, 24.0], dtype=np.float32)


def _quat_from_rotvec(r):
    th = np.linalg.norm(r, axis=-1, keepdims=True)
    half = 0.5 * th
    with np.errstate(invalid="ignore", divide="ignore"):
        s = np.where(th > 1e-12, np.sin(half) / np.where(th > 1e-12, th, 1.0), 0.5)
    return np.concatenate([s * r, np.cos(half)], axis=-1)


def _qmul(a, b):
    av, aw = a[..., :3], a[..., 3:]
    bv, bw = b[..., :3], b[..., 3:]
    return np.concatenate([aw * bv + bw * av + np.cross(av, bv), aw * bw - np.sum(av * bv, -1, keepdims=True)], -1)


def trajectory(n, rng):
    """world->cam poses of a forward-moving camera with small yaw drift."""
    yaw = np.cumsum(np.concatenate([[0.0], rng.normal(0, 0.01, n - 1)]))
    z = 0.05 * np.arange(n)
    poses = np.zeros((n, 7))
    for k in range(n):
        q = _quat_from_rotvec(np.array([0.0, yaw[k], 0.0]))          # cam<-world rotation
        c = np.array([0.0, 0.0, z[k]])                                 # camera centre in world
        qc = q.copy()
        # t = -R c
        qv, qw = qc[:3], qc[3]
        uv = 2 * np.cross(qv, c)
        Rc = c + qw * uv + np.cross(qv, uv)
        poses[k, :3] = -Rc
        poses[k, 3:] = q
    return poses


def smooth_disps(n, h, w, rng):
    """smooth random field in [0.2, 1.0]."""
    yy, xx = np.meshgrid(np.linspace(0, 1, h), np.linspace(0, 1, w), indexing="ij")
    out = np.zeros((n, h, w))
    for k in range(n):
        f = np.zeros((h, w))
        for _ in range(3):
            a, b, ph = rng.uniform(0.5, 3.0), rng.uniform(0.5, 3.0), rng.uniform(0, 2 * np.pi)
            f += np.sin(2 * np.pi * (a * xx + b * yy) + ph)
        f = (f - f.min()) / max(f.max() - f.min(), 1e-9)
        out[k] = 0.2 + 0.8 * f
    return out


def perturb(poses, disps, rng):
    p = poses.copy()
    p[:, :3] += rng.normal(0, 0.01, (len(p), 3))
    dq = _quat_from_rotvec(rng.normal(0, 0.005, (len(p), 3)))
    p[:, 3:] = _qmul(dq, p[:, 3:])
    d = disps * (1 + 0.05 * rng.normal(0, 1, disps.shape))
    return p, np.clip(d, 0.05, None)


def trajectory_laps(n, lap, rng):
    """world->cam poses of a camera driving `n / lap` laps of a circle (0.05 m
    per KF, heading along the tangent, a few cm / mrad of lap-to-lap jitter):
    keyframe i revisits the place of i - lap, as loop closures need."""
    R = 0.05 * lap / (2 * np.pi)
    th = 2 * np.pi * np.arange(n) / lap
    poses = np.zeros((n, 7))
    for k in range(n):
        r = R + 0.02 * rng.normal()
        c = np.array([r * (1 - np.cos(th[k])), 0.01 * rng.normal(), r * np.sin(th[k])])   # camera centre
        q = _quat_from_rotvec(np.array([0.0, -(th[k] + 0.01 * rng.normal()), 0.0]))     # cam<-world
        qv, qw = q[:3], q[3]
        uv = 2 * np.cross(qv, c)
        poses[k, :3] = -(c + qw * uv + np.cross(qv, uv))
        poses[k, 3:] = q
    return poses


def c3_edges(num_kf=256, num_edges=2048, rng=None, max_out=None):
    """±1..±3 temporal neighbours plus random bidirectional loop edges |i-j| > 3
    (no out-degree cap unless max_out is given)."""
    rng = rng or np.random.default_rng(1003)
    max_out = max_out or num_kf
    es = [(i, j) for i in range(num_kf) for j in range(num_kf) if i != j and abs(i - j) <= 3]
    have = set(es)
    out = {}
    for i, _ in es:
        out[i] = out.get(i, 0) + 1
    while len(es) + 2 <= num_edges:
        i, j = rng.integers(0, num_kf, 2)
        if abs(i - j) <= 3 or (i, j) in have or out.get(i, 0) >= max_out or out.get(j, 0) >= max_out:
            continue
        for a, b in ((i, j), (j, i)):
            es.append((int(a), int(b)))
            have.add((a, b))
            out[a] = out.get(a, 0) + 1
    e = np.asarray(es, dtype=np.int64)
    return e[:, 0], e[:, 1]


def c4_edges(num_kf=128, loops=100, rng=None):
    """Stereo config: one (i, i) stereo edge per keyframe
    (factor_graph.py:335-337; it correlates against the right image), +-1..+-3
    temporal neighbours and ~`loops` random bidirectional loop edges |i-j| > 3."""
    rng = rng or np.random.default_rng(1004)
    es = [(i, i) for i in range(num_kf)]
    es += [(i, j) for i in range(num_kf) for j in range(num_kf) if i != j and abs(i - j) <= 3]
    have = set(es)
    target = len(es) + loops
    while len(es) + 2 <= target:
        i, j = (int(x) for x in rng.integers(0, num_kf, 2))
        if abs(i - j) <= 3 or (i, j) in have:
            continue
        for a, b in ((i, j), (j, i)):
            es.append((a, b))
            have.add((a, b))
    e = np.asarray(es, dtype=np.int64)
    return e[:, 0], e[:, 1]


def c5_edges(num_kf=2048, lap=256, loop_pairs=None, rng=None):
    """Sharded config: 2048 KFs driving 8 laps of a circuit
    (trajectory_laps), ±1..±3 temporal neighbours plus bidirectional revisit
    loops i <-> i - m*lap + d (m >= 1, |d| <= 2) - the proximity edges
    frame_distance finds when a trajectory returns to a place - up to ~8 edges
    per KF (16k edges at 2048 KF)."""
    rng = rng or np.random.default_rng(1005)
    es = [(i, j) for i in range(num_kf) for j in range(max(0, i - 3), min(num_kf, i + 4)) if i != j]
    if loop_pairs is None:
        loop_pairs = max(0, (8 * num_kf - len(es)) // 2)
    have = set(es)
    added = 0
    while added < loop_pairs and num_kf > lap:
        i = int(rng.integers(lap, num_kf))
        m = int(rng.integers(1, i // lap + 1))
        j = i - m * lap + int(rng.integers(-2, 3))
        if j < 0 or j >= num_kf or abs(i - j) <= 3 or (i, j) in have:
            continue
        for a, b in ((i, j), (j, i)):
            es.append((a, b))
            have.add((a, b))
        added += 1
    e = np.asarray(es, dtype=np.int64)
    return e[:, 0], e[:, 1]


def dense_edges(num_kf=48, out_degree=42, rng=None):
    """High-degree graph (the backend's max_factors = 16 t regime and beyond,
    droid_backend.py:31): every frame links to `out_degree` others, always
    including its ±1..±3 neighbours."""
    rng = rng or np.random.default_rng(1006)
    es = []
    for i in range(num_kf):
        near = [j for j in range(max(0, i - 3), min(num_kf, i + 4)) if j != i]
        far = [j for j in range(num_kf) if j != i and j not in near]
        pick = rng.choice(far, size=min(len(far), out_degree - len(near)), replace=False)
        es += [(i, j) for j in near] + [(i, int(j)) for j in sorted(pick)]
    e = np.asarray(es, dtype=np.int64)
    return e[:, 0], e[:, 1]


def c2_edges():
    """Frontend window: 16-KF buffer, optimise [8,16); |i-j|<=3 in [4,16) plus
    inactive-style edges from [8,16) into [5,8) -> 96 edges."""
    es = [(i, j) for i in range(4, 16) for j in range(4, 16) if i != j and abs(i - j) <= 3]
    extra = [(i, j) for i in range(8, 16) for j in range(5, 8) if abs(i - j) > 3]
    for i, j in extra:
        if len(es) >= 96:
            break
        es.append((i, j))
        if len(es) < 96:
            es.append((j, i))
    e = np.asarray(es[:96], dtype=np.int64)
    return e[:, 0], e[:, 1]


def reproject_np(poses, disps, intr, ii, jj):
    """pixel ii -> frame jj with the BA kernel's conventions (float64)."""
    import sys, os  # local import keeps this module numpy-only
    E = len(ii)
    _, H, W = disps.shape
    fx, fy, cx, cy = intr
    v, u = np.meshgrid(np.arange(H, dtype=np.float64), np.arange(W, dtype=np.float64), indexing="ij")
    out = np.zeros((E, 2, H, W))
    for e, (i, j) in enumerate(zip(ii, jj)):
        qi, qj = poses[i, 3:], poses[j, 3:]
        qij = _qmul(qj, np.concatenate([-qi[:3], qi[3:]]))
        def rot(q, X):
            qv, qw = q[:3], q[3]
            uv = 2 * np.cross(qv, X)
            return X + qw * uv + np.cross(qv, uv)
        if i == j:
            tij, qij = np.array([-0.1, 0.0, 0.0]), np.array([0.0, 0.0, 0.0, 1.0])
        else:
            tij = poses[j, :3] - rot(qij, poses[i, :3])
        X = np.stack([(u - cx) / fx, (v - cy) / fy, np.ones_like(u)], -1)
        Y = rot(qij, X.reshape(-1, 3)).reshape(H, W, 3) + disps[i][..., None] * tij
        Z = np.where(Y[..., 2] < 0.1, 1.0, Y[..., 2])
        out[e, 0] = fx * Y[..., 0] / Z + cx
        out[e, 1] = fy * Y[..., 1] / Z + cy
    return out


def ba_problem(config="C2", H=48, W=64, seed=None, edges=None, num_frames=None, t0=None, t1=None,
               sens_fraction=0.0):
    """Inputs of one droid_backends.ba() call for a config (numpy, float32)."""
    cid = {"C2": 2, "C3": 3, "C4": 4, "C5": 5}.get(config, 9)
    rng = np.random.default_rng(1000 + cid if seed is None else seed)
    if edges is not None:
        ii, jj = edges
    elif config == "C2":
        ii, jj = c2_edges()
    elif config == "C3":
        ii, jj = c3_edges(rng=np.random.default_rng(1003))
    elif config == "C4":
        ii, jj = c4_edges(rng=np.random.default_rng(1004))
    elif config == "C5":
        ii, jj = c5_edges()
    else:
        raise ValueError(config)
    N = num_frames or int(max(ii.max(), jj.max())) + 1
    if t0 is None:
        t0 = 8 if config == "C2" else 1
    if t1 is None:
        t1 = int(max(ii.max(), jj.max())) + 1
    gt_poses = trajectory_laps(N, 256, rng) if config == "C5" else trajectory(N, rng)
    gt_disps = smooth_disps(N, H, W, rng)
    targets = reproject_np(gt_poses, gt_disps, INTRINSICS.astype(np.float64), ii, jj)
    targets += rng.normal(0, 0.5, targets.shape)
    poses, disps = perturb(gt_poses, gt_disps, rng)
    poses[0] = gt_poses[0]
    weights = rng.uniform(0, 1, targets.shape)
    kx = np.unique(np.concatenate([np.arange(t0, t1), ii]))
    eta = 0.2 * rng.uniform(1e-3, 1e-2, (len(kx), H, W)) + 1e-7
    disps_sens = np.zeros_like(disps)
    if sens_fraction > 0:
        m = rng.uniform(0, 1, disps.shape) < sens_fraction
        disps_sens = np.where(m, gt_disps * (1 + 0.01 * rng.normal(0, 1, disps.shape)), 0.0)
    f32 = lambda a: np.ascontiguousarray(a, dtype=np.float32)
    return dict(poses=f32(poses), disps=f32(disps), intrinsics=f32(INTRINSICS), disps_sens=f32(disps_sens),
                targets=f32(targets), weights=f32(weights), eta=f32(eta), ii=ii.astype(np.int64),
                jj=jj.astype(np.int64), t0=int(t0), t1=int(t1))
