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

    # the item tuple the frontend writes (depth_video.py:46-77): (tstamp, image,
    # pose, disp, depth, intrinsics[, fmap, net, inp]); pose / disp / depth /
    # intrinsics may be None (kept), the trailing features may be absent
    _ITEM_FIELDS = ("tstamp", "images", "poses", "disps", None, "intrinsics", "fmaps", "nets", "inps")
    _OPTIONAL = frozenset(("poses", "disps", "intrinsics"))

    def _grow_counter(self, index):
        """the frame count follows the highest slot written (an int slot at or
        past the end, or an index tensor whose largest entry exceeds it)."""
        if isinstance(index, int):
            top = index if index >= self.counter.value else None
        elif isinstance(index, torch.Tensor):
            hi = int(index.max().item())
            top = hi if hi > self.counter.value else None
        else:
            top = None
        if top is not None:
            self.counter.value = top + 1

    def _write(self, index, item):
        self._grow_counter(index)
        for k, value in enumerate(item[:len(self._ITEM_FIELDS)]):
            name = self._ITEM_FIELDS[k]
            if name is None:      # a full-resolution depth map -> sensor disparity at 1/8 resolution
                if value is not None:
                    d8 = value[3::8, 3::8]
                    self.disps_sens[index] = torch.where(d8 > 0, 1.0 / d8, d8)
            elif value is not None or name not in self._OPTIONAL:
                getattr(self, name)[index] = value

    def __setitem__(self, index, item):
        with self.get_lock():
            self._write(index, item)

    def __getitem__(self, index):
        with self.get_lock():
            slot = self.counter.value + index if isinstance(index, int) and index < 0 else index
            return tuple(getattr(self, name)[slot] for name in ("poses", "disps", "intrinsics", "fmaps", "nets",
                                                                  "inps"))

    def append(self, *item):
        with self.get_lock():
            self._write(self.counter.value, item)

    @staticmethod
    def format_indicies(ii, jj, device="cuda"):
        """edge index lists (any sequence or tensor) -> flat int64 tensors on device."""
        def flat(x):
            return torch.as_tensor(x).to(device=device, dtype=torch.long).reshape(-1)
        return flat(ii), flat(jj)

    def upsample(self, ix, mask):
        """convex upsampling of the 1/8 disparities of frames ix (depth_video.py:123-127)."""
        self.disps_up[ix] = cvx_upsample(self.disps[ix].unsqueeze(-1), mask).squeeze()

    def normalize(self):
        """rescale so the mean disparity of the stored frames is 1 (poses' translations
        scaled alike), depth_video.py:129-136."""
        with self.get_lock():
            live = slice(0, self.counter.value)
            scale = self.disps[live].mean()
            self.disps[live].div_(scale)
            self.poses[live, :3].mul_(scale)
            self.dirty[live] = True

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

    Failures are agreed on, not per rank: after each GN iteration's Cholesky
    the status words are OR-reduced (per bit, 64 bytes) on the device BEFORE the
    back-substitution and retraction, so if any rank's dataflow solve timed out
    every rank skips that step (the replicated poses never diverge), and every
    rank raises at its next BA call (or droid_backends.check_status()) - no
    rank is left waiting in a collective."""
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
    status = plan.status_words()     # a view of the device status words [this solve, sticky]
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
        sev = comm.get("_solve_events")   # bench: HIP events around the replicated solve, or None
        if sev is not None:
            se = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            se[0].record()
        plan.solve_system(lm, ep, dx)
        if sev is not None:
            se[1].record()
            sev.append(se)
        # the status words agreed before the step is applied: a bitwise OR over
        # the ranks (one int per bit, all-reduced MAX, repacked - ADVICE r5: a
        # MAX of the packed words kept the skip bit but could drop another
        # rank's non-SPD bit).  A rank whose dataflow solve timed out makes EVERY
        # rank skip this step's back-substitution and retraction, so the
        # replicated poses stay equal
        or_reduce_status(status, group)
        plan.apply_update(poses, disps, intrinsics, disps_sens, target, weight, eta, dx, dz)
    plan._record_status()     # the agreed words (identical on every rank)
    comm["_last_plan"] = plan
    return [dx, dz]


_STATUS_BITS = 8   # the status word's bits (0 non-SPD, 1 skipped, 2 corrupt state; spare to 7)


def or_reduce_status(status, group=None):
    """In place: the bitwise OR of the int status words over the ranks of
    `group` - one int per bit, all-reduced with MAX, repacked (a MAX of the
    packed words keeps the highest word, dropping the other ranks' lower bits)."""
    import torch.distributed as dist
    # made on the device (a host tensor's .to() would be a pageable H2D copy per
    # GN iteration, which waits for the stream)
    shifts = torch.arange(_STATUS_BITS, device=status.device, dtype=status.dtype)
    bits = (status.unsqueeze(-1) >> shifts) & 1
    dist.all_reduce(bits, op=dist.ReduceOp.MAX, group=group)
    status.copy_((bits << shifts).sum(-1, dtype=status.dtype))
    return status


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
    local = (ii_host.tobytes(), jj_host.tobytes())
    if hit is None:
        parts = [None] * dist.get_world_size(group)
        dist.all_gather_object(parts, (ii_host, jj_host), group=group)
        hit = (np.concatenate([p[0] for p in parts]), np.concatenate([p[1] for p in parts]), {local})
        if key is not None:
            if len(cache) >= 4:
                cache.pop(next(iter(cache)))
            cache[key] = hit
    elif len(ii_host) and local not in hit[2]:
        # validated once per (cached list, local edge list): later hits skip the set test
        n = int(max(hit[0].max(), hit[1].max(), ii_host.max(), jj_host.max())) + 1
        have = np.unique(hit[0] * n + hit[1])
        if not np.isin(ii_host * n + jj_host, have).all():
            raise RuntimeError("ba (sharded): this rank's edges are not in the global edge list of edge-set "
                               "version %r - edge edits must be issued on every rank" % (version,))
        hit[2].add(local)
    return hit[0], hit[1]
