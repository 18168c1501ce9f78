"""Keyframe state buffers (mirror of droid_slam/depth_video.py).

Same buffers and methods as the reference DepthVideo (depth_video.py:12-193)
for the parts the update path touches: poses/disps/disps_sens/intrinsics,
fmaps/nets/inps, `reproject`, `distance`, `ba`, `normalize`, `upsample`.
Geometry is lietorch-free: `reproject` calls the fused HIP projective-transform
kernel.  Buffers live in HBM; torch.multiprocessing sharing (the reference's
visualiser process) is out of scope.
"""
import threading

import numpy as np
import torch

import droid_backends

from .update import cvx_upsample


class _Counter:
    """Stand-in for multiprocessing.Value('i') with its lock."""

    def __init__(self):
        self.value = 0
        self._lock = threading.RLock()

    def get_lock(self):
        return self._lock


class DepthVideo:
    def __init__(self, image_size=(480, 640), buffer=1024, stereo=False, device="cuda:0"):
        self.counter = _Counter()
        self.ready = _Counter()
        self.ht = ht = image_size[0]
        self.wd = wd = image_size[1]
        self.device = torch.device(device)
        dev = self.device
        self.tstamp = torch.zeros(buffer, device=dev, dtype=torch.float)
        self.images = torch.zeros(buffer, 3, ht, wd, device=dev, dtype=torch.uint8)
        self.dirty = torch.zeros(buffer, device=dev, dtype=torch.bool)
        self.red = torch.zeros(buffer, device=dev, dtype=torch.bool)
        self.poses = torch.zeros(buffer, 7, device=dev, dtype=torch.float)
        self.disps = torch.ones(buffer, ht // 8, wd // 8, device=dev, dtype=torch.float)
        self.disps_sens = torch.zeros(buffer, ht // 8, wd // 8, device=dev, dtype=torch.float)
        self.disps_up = torch.zeros(buffer, ht, wd, device=dev, dtype=torch.float)
        self.intrinsics = torch.zeros(buffer, 4, device=dev, dtype=torch.float)
        self.stereo = stereo
        c = 2 if stereo else 1
        self.fmaps = torch.zeros(buffer, c, 128, ht // 8, wd // 8, dtype=torch.half, device=dev)
        self.nets = torch.zeros(buffer, 128, ht // 8, wd // 8, dtype=torch.half, device=dev)
        self.inps = torch.zeros(buffer, 128, ht // 8, wd // 8, dtype=torch.half, device=dev)
        self.poses[:] = torch.as_tensor([0, 0, 0, 0, 0, 0, 1], dtype=torch.float, device=dev)

    def get_lock(self):
        return self.counter.get_lock()

    def __item_setter(self, index, item):
        if isinstance(index, int) and index >= self.counter.value:
            self.counter.value = index + 1
        elif isinstance(index, torch.Tensor) and index.max().item() > self.counter.value:
            self.counter.value = index.max().item() + 1
        self.tstamp[index] = item[0]
        self.images[index] = item[1]
        if item[2] is not None:
            self.poses[index] = item[2]
        if item[3] is not None:
            self.disps[index] = item[3]
        if item[4] is not None:
            depth = item[4][3::8, 3::8]
            self.disps_sens[index] = torch.where(depth > 0, 1.0 / depth, depth)
        if item[5] is not None:
            self.intrinsics[index] = item[5]
        if len(item) > 6:
            self.fmaps[index] = item[6]
        if len(item) > 7:
            self.nets[index] = item[7]
        if len(item) > 8:
            self.inps[index] = item[8]

    def __setitem__(self, index, item):
        with self.get_lock():
            self.__item_setter(index, item)

    def __getitem__(self, index):
        with self.get_lock():
            if isinstance(index, int) and index < 0:
                index = self.counter.value + index
            return (self.poses[index], self.disps[index], self.intrinsics[index],
                    self.fmaps[index], self.nets[index], self.inps[index])

    def append(self, *item):
        with self.get_lock():
            self.__item_setter(self.counter.value, item)

    @staticmethod
    def format_indicies(ii, jj, device="cuda"):
        if not isinstance(ii, torch.Tensor):
            ii = torch.as_tensor(ii)
        if not isinstance(jj, torch.Tensor):
            jj = torch.as_tensor(jj)
        return (ii.to(device=device, dtype=torch.long).reshape(-1),
                jj.to(device=device, dtype=torch.long).reshape(-1))

    def upsample(self, ix, mask):
        disps_up = cvx_upsample(self.disps[ix].unsqueeze(-1), mask)
        self.disps_up[ix] = disps_up.squeeze()

    def normalize(self):
        with self.get_lock():
            n = self.counter.value
            s = self.disps[:n].mean()
            self.disps[:n] /= s
            self.poses[:n, :3] *= s
            self.dirty[:n] = True

    def reproject(self, ii, jj, target=None):
        """project pixels of ii into jj (depth_video.py:139-147) -> coords
        (1,E,H,W,2), valid (1,E,H,W,1) [, motion features (1,E,4,H,W) if target]."""
        ii, jj = DepthVideo.format_indicies(ii, jj, self.device)
        out = droid_backends.projective_transform(self.poses, self.disps, self.intrinsics, ii, jj,
                                                  target=None if target is None else target.reshape(
                                                      -1, self.ht // 8, self.wd // 8, 2).contiguous())
        return tuple(o.unsqueeze(0) for o in out)

    def distance(self, ii=None, jj=None, beta=0.3, bidirectional=True):
        """frame distance metric (depth_video.py:149-179)."""
        return_matrix = False
        N = self.counter.value
        if ii is None:
            return_matrix = True
            ii, jj = torch.meshgrid(torch.arange(N), torch.arange(N), indexing="ij")
        ii, jj = DepthVideo.format_indicies(ii, jj, self.device)
        if bidirectional:
            poses = self.poses[:N].clone()
            d1 = droid_backends.frame_distance(poses, self.disps, self.intrinsics[0].contiguous(), ii, jj, beta)
            d2 = droid_backends.frame_distance(poses, self.disps, self.intrinsics[0].contiguous(), jj, ii, beta)
            d = 0.5 * (d1 + d2)
        else:
            d = droid_backends.frame_distance(self.poses, self.disps, self.intrinsics[0].contiguous(), ii, jj, beta)
        if return_matrix:
            return d.reshape(N, N)
        return d

    def ba(self, target, weight, eta, ii, jj, t0=1, t1=None, itrs=2, lm=1e-4, ep=0.1, motion_only=False,
           ii_host=None, jj_host=None, comm=None, edge_tag=None):
        """dense bundle adjustment (depth_video.py:181-193).

        comm (edge-sharded multi-GPU): dict(group=process group, own=(lo, hi),
        t1=global t1, version=edge-set version).  Each rank passes only the
        edges whose source frame it owns; the reduced camera system is summed
        with one all-reduce per Gauss-Newton iteration and solved identically
        on every rank.  edge_tag names which of the caller's edge sets this
        is (e.g. with / without the inactive edges) for the global-list cache."""
        with self.get_lock():
            if ii_host is None:
                ii_host = ii.cpu().numpy()
            if jj_host is None:
                jj_host = jj.cpu().numpy()
            if comm is not None and comm.get("t1") is not None and t1 is None:
                t1 = comm["t1"]
            if t1 is None:
                t1 = int(max(np.max(ii_host), np.max(jj_host))) + 1
            intr = self.intrinsics[0].contiguous()
            if comm is None:
                out = droid_backends.ba(self.poses, self.disps, intr, self.disps_sens, target, weight, eta, ii, jj,
                                        t0, t1, itrs, lm, ep, motion_only, ii_host=ii_host, jj_host=jj_host)
            else:
                out = ba_sharded(self.poses, self.disps, intr, self.disps_sens, target, weight, eta, ii_host,
                                 jj_host, t0, t1, itrs, lm, ep, motion_only, comm, edge_tag)
            self.disps.clamp_(min=0.001)
            return out


def ba_sharded(poses, disps, intrinsics, disps_sens, target, weight, eta, ii_host, jj_host, t0, t1, itrs, lm, ep,
               motion_only, comm, edge_tag=None):
    """One rank of the edge-sharded BA: local linearisation + Schur terms,
    all_reduce(SUM) of the reduced system's input tiles (RCCL over xGMI), then
    the same damped fp64 Cholesky on every rank; dz only for owned frames.

    The pose order and the factor's tile structure come from the GLOBAL edge
    list (global_edges), so the tiles line up across ranks and only the
    structurally nonzero 64x64 tiles of A - S and the rhs row cross the links
    (9.6 MB at C3, 66 MB at C5 instead of the dense 603 MB).

    Failures are agreed on, not per rank: the solves' status words are
    all-reduced (MAX) on the device after the last GN iteration, and every rank
    raises at its next BA call (or droid_backends.check_status()) if any rank's
    dataflow Cholesky timed out - no rank is left waiting in a collective."""
    import torch.distributed as dist
    group = comm.get("group")
    N, H, W = disps.shape
    eta_rows = eta.numel() // (H * W)
    last = comm.pop("_last_plan", None)
    if last is not None:
        last.check_status()          # the previous call's agreed status (every rank raises alike)
    gedges = global_edges(ii_host, jj_host, comm, (int(t0), int(t1), bool(motion_only), edge_tag))
    plan = droid_backends.get_plan(ii_host, jj_host, N, H, W, int(t0), int(t1), eta_rows, motion_only,
                                   poses.device, own=tuple(comm["own"]), gedges=gedges)
    dx = torch.empty((plan.P, 6), dtype=torch.float32, device=poses.device)
    dz = None if motion_only else torch.empty((plan.K, H * W), dtype=torch.float32, device=poses.device)
    flat = plan.system.view(-1)
    plan.clear_status()
    timing = comm.get("_ar_events")   # bench: HIP events around each all-reduce, or None
    for _ in range(itrs):
        plan.build_system(poses, disps, intrinsics, disps_sens, target, weight, eta)
        if timing is not None:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
        if timing is not None:
            ev[1].record()
            timing.append(ev + (flat.numel() * flat.element_size(),))
        plan.solve_update(poses, disps, intrinsics, disps_sens, target, weight, eta, lm, ep, dx, dz)
    # status values are 0..3 per word, so MAX keeps the timeout bit (value >= 2) of any rank
    status = plan.status_words().clone()
    dist.all_reduce(status, op=dist.ReduceOp.MAX, group=group)
    plan._record_status(status)
    comm["_last_plan"] = plan
    return [dx, dz]


def global_edges(ii_host, jj_host, comm, call_key):
    """The union of every rank's BA edges, in rank order.

    Whether to (re)gather must be decided identically on every rank, or one
    rank blocks in the gather while the others enter the next all-reduce.  The
    cache is therefore keyed by replicated values only: comm["version"] (bumped
    by every FactorGraph edge edit, which the ranks issue in lockstep) and the
    call's (t0, t1, motion_only, edge tag).  Without a "version" in comm the
    list is gathered on every call.  On a cache hit the local edges must be
    part of the cached list (a rank that edited alone is a caller bug: raise)."""
    import torch.distributed as dist
    group = comm.get("group")
    ii_host = np.asarray(ii_host, np.int64)
    jj_host = np.asarray(jj_host, np.int64)
    version = comm.get("version")
    key = None if version is None else (version,) + tuple(call_key)
    cache = comm.setdefault("_gedges", {})
    hit = cache.get(key) if key is not None else None
    if hit is None:
        parts = [None] * dist.get_world_size(group)
        dist.all_gather_object(parts, (ii_host, jj_host), group=group)
        hit = (np.concatenate([p[0] for p in parts]), np.concatenate([p[1] for p in parts]))
        if key is not None:
            if len(cache) >= 4:
                cache.pop(next(iter(cache)))
            cache[key] = hit
    elif len(ii_host):
        n = int(max(hit[0].max(), hit[1].max(), ii_host.max(), jj_host.max())) + 1
        have = np.unique(hit[0] * n + hit[1])
        if not np.isin(ii_host * n + jj_host, have).all():
            raise RuntimeError("ba (sharded): this rank's edges are not in the global edge list of edge-set "
                               "version %r - edge edits must be issued on every rank" % (version,))
    return hit
