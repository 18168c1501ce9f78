"""Geometry restatements (numpy, fp64 by default).

projective_transform : droid_slam/geom/projective_ops.py:96-125 (+iproj :18-37,
                       proj :39-65, actp :67-94) with lietorch SE3 semantics.
frame_distance       : src/droid_kernels.cu:518-657
projmap              : src/droid_kernels.cu:427-516
iproj                : src/droid_kernels.cu:779-850
depth_filter         : src/droid_kernels.cu:661-775
"""
import numpy as np

from .se3 import act_se3, act_so3, pose_inv, pose_mul, rel_se3

MIN_DEPTH_POPS = 0.2      # projective_ops.py:6
MIN_DEPTH_KERNEL = 0.25   # droid_kernels.cu:26
STEREO_POSE = np.array([-0.1, 0.0, 0.0, 0.0, 0.0, 0.0, 1.0])  # projective_ops.py:105


def coords_grid(ht, wd, dtype=np.float64):
    """projective_ops.py:11-16: (..., [x, y])."""
    y, x = np.meshgrid(np.arange(ht, dtype=dtype), np.arange(wd, dtype=dtype), indexing="ij")
    return np.stack([x, y], axis=-1)


def projective_transform(poses, disps, intrinsics, ii, jj, dtype=np.float64):
    """Map pixels of frame ii into frame jj (projective_ops.py:96-125).

    poses (N,7), disps (N,H,W), intrinsics (N,4) -> coords (E,H,W,2), valid (E,H,W,1)
    Gij = poses[jj] * poses[ii]^-1, stereo edges (ii == jj) forced to
    [-0.1,0,0, 0,0,0,1] (:105); proj clamps Z < 0.1 -> 1 (:44); valid = Z > 0.2 (:112).
    """
    poses = np.asarray(poses, dtype)
    disps = np.asarray(disps, dtype)
    intr = np.asarray(intrinsics, dtype)
    ii = np.asarray(ii)
    jj = np.asarray(jj)
    _, H, W = disps.shape
    fx, fy, cx, cy = [intr[ii, k][:, None, None] for k in range(4)]
    y, x = np.meshgrid(np.arange(H, dtype=dtype), np.arange(W, dtype=dtype), indexing="ij")
    X0 = np.stack([(x - cx) / fx, (y - cy) / fy, np.ones_like(disps[ii]), disps[ii]], axis=-1)
    Gij = pose_mul(poses[jj], pose_inv(poses[ii]))
    Gij[ii == jj] = STEREO_POSE
    G = Gij[:, None, None, :]
    X1 = act_se3(np.broadcast_to(G[..., :3], X0[..., :3].shape),
                 np.broadcast_to(G[..., 3:], X0[..., :3].shape[:-1] + (4,)), X0)
    fx, fy, cx, cy = [intr[jj, k][:, None, None] for k in range(4)]
    Z = np.where(X1[..., 2] < 0.5 * MIN_DEPTH_POPS, 1.0, X1[..., 2])
    d = 1.0 / Z
    coords = np.stack([fx * (X1[..., 0] * d) + cx, fy * (X1[..., 1] * d) + cy], axis=-1)
    valid = ((X1[..., 2] > MIN_DEPTH_POPS) & (X0[..., 2] > MIN_DEPTH_POPS)).astype(dtype)[..., None]
    return coords, valid


def _pixel_rays(H, W, intr, dtype):
    fx, fy, cx, cy = [dtype(v) for v in intr]
    v, u = np.meshgrid(np.arange(H, dtype=dtype), np.arange(W, dtype=dtype), indexing="ij")
    return u, v, (u - cx) / fx, (v - cy) / fy


def frame_distance(poses, disps, intrinsics, ii, jj, beta, dtype=np.float64):
    """frame_distance_kernel droid_kernels.cu:518-657 (+ host :1438-1460)."""
    poses = np.asarray(poses, dtype)
    disps = np.asarray(disps, dtype)
    fx, fy, cx, cy = [dtype(v) for v in intrinsics]
    _, H, W = disps.shape
    u, v, xr, yr = _pixel_rays(H, W, intrinsics, dtype)
    out = np.zeros(len(ii), dtype)
    for e, (i, j) in enumerate(zip(np.asarray(ii), np.asarray(jj))):
        tij, qij = rel_se3(poses[i, :3], poses[i, 3:], poses[j, :3], poses[j, 3:])
        Xi = np.stack([xr, yr, np.ones_like(xr), disps[i]], axis=-1)
        Xj = act_se3(tij, qij, Xi)
        d = np.sqrt((fx * Xj[..., 0] / Xj[..., 2] + cx - u) ** 2 + (fy * Xj[..., 1] / Xj[..., 2] + cy - v) ** 2)
        ok = Xj[..., 2] > MIN_DEPTH_KERNEL
        accum = beta * np.sum(np.where(ok, d, 0.0))
        valid = beta * np.sum(ok)
        Xt = Xi[..., :3] + Xi[..., 3:4] * tij
        d = np.sqrt((fx * Xt[..., 0] / Xt[..., 2] + cx - u) ** 2 + (fy * Xt[..., 1] / Xt[..., 2] + cy - v) ** 2)
        ok = Xt[..., 2] > MIN_DEPTH_KERNEL
        accum += (1 - beta) * np.sum(np.where(ok, d, 0.0))
        valid += (1 - beta) * np.sum(ok)
        total = H * W * 1.0
        out[e] = 1000.0 if valid / (total + 1e-8) < 0.75 else accum / valid
    return out


def projmap(poses, disps, intrinsics, ii, jj, dtype=np.float64):
    """projmap_kernel droid_kernels.cu:427-516 -> coords (E,H,W,3) [x,y,0], valid (E,H,W,1)."""
    poses = np.asarray(poses, dtype)
    disps = np.asarray(disps, dtype)
    fx, fy, cx, cy = [dtype(v) for v in intrinsics]
    _, H, W = disps.shape
    u, v, xr, yr = _pixel_rays(H, W, intrinsics, dtype)
    E = len(ii)
    coords = np.zeros((E, H, W, 3), dtype)
    valid = np.zeros((E, H, W, 1), dtype)
    for e, (i, j) in enumerate(zip(np.asarray(ii), np.asarray(jj))):
        tij, qij = rel_se3(poses[i, :3], poses[i, 3:], poses[j, :3], poses[j, 3:])
        Xj = act_se3(tij, qij, np.stack([xr, yr, np.ones_like(xr), disps[i]], axis=-1))
        front = Xj[..., 2] > 0.01
        with np.errstate(divide="ignore", invalid="ignore"):
            coords[e, ..., 0] = np.where(front, fx * (Xj[..., 0] / Xj[..., 2]) + cx, u)
            coords[e, ..., 1] = np.where(front, fy * (Xj[..., 1] / Xj[..., 2]) + cy, v)
        valid[e, ..., 0] = (Xj[..., 2] > MIN_DEPTH_KERNEL).astype(dtype)
    return coords, valid


def iproj(poses, disps, intrinsics, dtype=np.float64):
    """iproj_kernel droid_kernels.cu:779-850: points = (R [x,y,1] + t d) / d."""
    poses = np.asarray(poses, dtype)
    disps = np.asarray(disps, dtype)
    N, H, W = disps.shape
    _, _, xr, yr = _pixel_rays(H, W, intrinsics, dtype)
    out = np.zeros((N, H, W, 3), dtype)
    for n in range(N):
        X = act_se3(poses[n, :3], poses[n, 3:], np.stack([xr, yr, np.ones_like(xr), disps[n]], axis=-1))
        out[n] = X[..., :3] / X[..., 3:4]
    return out


def depth_filter(poses, disps, intrinsics, ix, thresh, dtype=np.float64):
    """depth_filter_kernel droid_kernels.cu:661-775 (+ host :1491-1515).

    Neighbours of frame ix: ix-1, ix-2, ix-3 and ix+3, ix+4, ix+5 (neigh_id
    mapping at :695).  counter[b,i,j] counts neighbours whose reprojected
    disparity agrees with one of the 4 surrounding pixels within thresh[b].
    """
    poses = np.asarray(poses, dtype)
    disps = np.asarray(disps, dtype)
    fx, fy, cx, cy = [dtype(v) for v in intrinsics]
    num, H, W = disps.shape
    _, _, xr, yr = _pixel_rays(H, W, intrinsics, dtype)
    counter = np.zeros((len(ix), H, W), dtype)
    for b, i in enumerate(np.asarray(ix)):
        t = dtype(thresh[b])
        for neigh in range(6):
            j = i - neigh - 1 if neigh < 3 else i + neigh
            if j < 0 or j >= num:
                continue
            tij, qij = rel_se3(poses[i, :3], poses[i, 3:], poses[j, :3], poses[j, 3:])
            Xj = act_se3(tij, qij, np.stack([xr, yr, np.ones_like(xr), disps[i]], axis=-1))
            with np.errstate(divide="ignore", invalid="ignore"):
                uj = fx * (Xj[..., 0] / Xj[..., 2]) + cx
                vj = fy * (Xj[..., 1] / Xj[..., 2]) + cy
                dj = Xj[..., 3] / Xj[..., 2]
            u0 = np.floor(uj)
            v0 = np.floor(vj)
            inb = (u0 >= 0) & (v0 >= 0) & (u0 < W - 1) & (v0 < H - 1)
            u0i = np.clip(np.nan_to_num(u0), 0, W - 2).astype(np.int64)
            v0i = np.clip(np.nan_to_num(v0), 0, H - 2).astype(np.int64)
            dd = [disps[j][v0i + a, u0i + c] for a, c in ((0, 0), (0, 1), (1, 0), (1, 1))]
            with np.errstate(divide="ignore", invalid="ignore"):
                hit = np.zeros_like(inb)
                for dk in dd:
                    hit |= np.abs(1.0 / dj - 1.0 / dk) < t
            counter[b] += (inb & hit).astype(dtype)
    return counter
