"""Lockstep replay of the frontend's sequence on the device FactorGraph and on
the oracle graph (test infrastructure, not a test module).

The sequence is droid_frontend.py's: __initialize (:75-106) - neighbourhood
edges, 8 update(1, use_inactive=True), proximity edges, 8 more, the next
frame's pose/disparity guess, rm_factors(ii < warmup - 4, store=True) - then
per new keyframe __update (:35-73): rm_factors(age > max_age, store=True),
add_proximity_factors(t1 - 5, max(t1 - window, 0), remove=True), 4
update(use_inactive=True), the keyframe test distance([t1-3], [t1-2]) <
keyframe_thresh -> rm_keyframe(t1 - 2), else 2 more updates, then the next
frame's guess.  Defaults are demo.py's (warmup 8, beta 0.3, frontend_nms 1,
keyframe_thresh 4.0, frontend_window 25, frontend_thresh 16.0,
frontend_radius 2; max_factors 48, max_age 25).

The two sides only differ in arithmetic (fp16 convs / fp32 BA linearisation
on the device, fp32 convs + fp64 BA in the oracle).  The discrete decisions
(which proximity edges, whether a keyframe is dropped) are taken from the
ORACLE and applied to both sides, so the trajectories stay comparable; each
side's own decision is recorded and the mismatches reported.
"""
import os
import sys
import time

import numpy as np
import torch

from oracle import ate as oate
from oracle import frontend as ofe


class DeviceSide:
    """droid_mi355x FactorGraph + DepthVideo behind the oracle Graph's surface."""

    def __init__(self, video, graph):
        self.video, self.g = video, graph

    @property
    def counter(self):
        return self.video.counter.value

    def append(self, k, fmap, net, inp, intr):
        v = self.video
        v.fmaps[k] = torch.from_numpy(fmap).to(v.fmaps.device)
        v.nets[k] = torch.from_numpy(net).to(v.nets.device)
        v.inps[k] = torch.from_numpy(inp).to(v.inps.device)
        v.intrinsics[k] = torch.from_numpy(intr).to(v.intrinsics.device)
        v.counter.value = k + 1

    def set_counter(self, n):
        self.video.counter.value = n

    def poses(self):
        return self.video.poses.cpu().numpy().astype(np.float64)

    def disps(self):
        return self.video.disps.cpu().numpy().astype(np.float64)

    def guess_next(self, t1, mean_from):
        """droid_frontend.py:69-70 / :93-94"""
        v = self.video
        v.poses[t1] = v.poses[t1 - 1].clone()
        v.disps[t1] = v.disps[mean_from:t1].mean()

    def distance(self, i, j, beta):
        return float(self.video.distance([i], [j], beta=beta, bidirectional=True).item())

    def proximity_edge_list(self, t0, t1, rad, nms, beta, thresh):
        return self.g.proximity_factor_list(t0, t1, rad=rad, nms=nms, beta=beta, thresh=thresh)


class OracleSide:
    def __init__(self, graph):
        self.g = graph
        self.video = graph.video

    @property
    def counter(self):
        return self.video.counter

    def append(self, k, fmap, net, inp, intr):
        v = self.video
        v.fmaps[k], v.nets[k], v.inps[k], v.intrinsics[k] = fmap, net, inp, intr
        v.counter = k + 1

    def set_counter(self, n):
        self.video.counter = n

    def poses(self):
        return self.video.poses.copy()

    def disps(self):
        return self.video.disps.copy()

    def guess_next(self, t1, mean_from):
        v = self.video
        v.poses[t1] = v.poses[t1 - 1]
        v.disps[t1] = v.disps[mean_from:t1].mean()

    def distance(self, i, j, beta):
        return float(self.video.distance(np.array([i]), np.array([j]), beta=beta)[0])

    def proximity_edge_list(self, t0, t1, rad, nms, beta, thresh):
        d = self.g.proximity_distances(t0, t1, beta)
        return self.g.proximity_edge_list(d, t0, t1, rad, nms, thresh)


def replay(dev, ref, stream, num_frames, warmup=8, beta=0.3, nms=1, keyframe_thresh=4.0, window=25, thresh=16.0,
           radius=2, max_age=25, log=None):
    """Run the frontend over `num_frames` frames of `stream(k) -> (fmap, net,
    inp, intrinsics)` on both sides.  dev may be None (oracle only, for
    timing).  Returns a report dict."""
    sides = [s for s in (dev, ref) if s is not None]
    rep = dict(steps=[], edge_mismatch=0, keyframe_mismatch=0, removed_keyframes=0, updates=0)

    def compare(tag):
        n = ref.counter
        rec = dict(tag=tag, frames=n, edges=len(ref.g.ii))
        if dev is not None:
            pd, pr = dev.poses()[:n], ref.poses()[:n]
            rec["dpose"] = float(np.abs(pd - pr).max())
            rec["ddisp"] = float(np.abs(dev.disps()[:n] - ref.disps()[:n]).max())
            assert len(dev.g._ii) == len(ref.g.ii) and np.array_equal(dev.g._ii, ref.g.ii), "edge lists diverged"
        rep["steps"].append(rec)
        if log:
            log(rec)

    debug = os.environ.get("DROID_GRAPH_DEBUG", "0") == "1"

    def update(tag, **kw):
        for s in sides:
            s.g.update(**kw)
            if debug:   # diagnostics: attribute a device fault to its side and update
                torch.cuda.synchronize()
                print("[replay] update %d (%s) %s done" % (rep["updates"], tag, type(s).__name__), file=sys.stderr,
                      flush=True)
        rep["updates"] += 1
        compare(tag)

    def proximity(t0, t1, rad, nms_, beta_, remove):
        es = ref.proximity_edge_list(t0, t1, rad, nms_, beta_, thresh)
        if dev is not None:
            es_dev = dev.proximity_edge_list(t0, t1, rad, nms_, beta_, thresh)
            if not np.array_equal(es_dev, es):
                rep["edge_mismatch"] += 1
        for s in sides:
            s.g.add_factors(es[:, 0], es[:, 1], remove)

    t_start = time.time()
    for k in range(warmup):
        for s in sides:
            s.append(k, *stream(k))
    # __initialize
    t1 = warmup
    for s in sides:
        s.g.add_neighborhood_factors(0, t1, r=3)
    for _ in range(8):
        update("init", t0=1, use_inactive=True)
    proximity(0, 0, 2, 2, 0.25, False)
    for _ in range(8):
        update("init+prox", t0=1, use_inactive=True)
    for s in sides:
        s.guess_next(t1, t1 - 4)
        s.g.rm_factors(s.g._ii < warmup - 4 if s is dev else s.g.ii < warmup - 4, store=True)
    # __update per new frame
    for k in range(warmup, num_frames):
        for s in sides:
            s.append(s.counter, *stream(k))
        t1 += 1
        for s in sides:
            age = s.g.age.cpu().numpy() if s is dev else s.g.age
            s.g.rm_factors(age > max_age, store=True)
        proximity(t1 - 5, max(t1 - window, 0), radius, nms, beta, True)
        for _ in range(4):
            update("kf%d" % k, use_inactive=True)
        d_ref = ref.distance(t1 - 3, t1 - 2, beta)
        rep.setdefault("keyframe_distances", []).append(d_ref)
        drop = d_ref < keyframe_thresh
        if dev is not None and (dev.distance(t1 - 3, t1 - 2, beta) < keyframe_thresh) != drop:
            rep["keyframe_mismatch"] += 1
        if drop:
            rep["removed_keyframes"] += 1
            for s in sides:
                s.g.rm_keyframe(t1 - 2)
                s.set_counter(s.counter - 1)
            t1 -= 1
        else:
            for _ in range(2):
                update("kf%d+" % k, use_inactive=True)
        for s in sides:
            s.guess_next(t1, t1 - 1)
    rep["seconds"] = time.time() - t_start
    n = ref.counter
    rep["keyframes"] = n
    if dev is not None:
        rep["max_dpose"] = max(r["dpose"] for r in rep["steps"])
        rep["max_ddisp"] = max(r["ddisp"] for r in rep["steps"])
        cd, cr = oate.camera_centres(dev.poses()[:n]), oate.camera_centres(ref.poses()[:n])
        traj = lambda c: np.concatenate([c, np.tile([0, 0, 0, 1.0], (len(c), 1))], 1)
        rep["ate_vs_ref"] = oate.ate(traj(cr), traj(cd), False)[0]
        rep["ate_vs_ref_scaled"] = oate.ate(traj(cr), traj(cd), True)[0]
        rep["trajectory_extent"] = float(np.linalg.norm(cr - cr[0], axis=1).max())
    return rep


def synthetic_stream(H, W, seed=1100):
    """frame k -> (fmap (1,128,H,W), net, inp (128,H,W)) fp16-valued, intrinsics."""
    from droid_mi355x import synthetic

    def frame(k):
        rng = np.random.default_rng(seed + k)
        fmap = rng.normal(size=(1, 128, H, W)).astype(np.float16)
        net = np.tanh(rng.normal(size=(128, H, W))).astype(np.float16)
        inp = np.maximum(rng.normal(size=(128, H, W)), 0).astype(np.float16)
        intr = (synthetic.INTRINSICS * np.float32(W / 64.0)).astype(np.float32)
        return fmap, net, inp, intr
    return frame


def oracle_side(params, H, W, buffer, device=None):
    v = ofe.Video(np.tile([0, 0, 0, 0, 0, 0, 1.0], (buffer, 1)), np.ones((buffer, H, W)), np.zeros((buffer, H, W)),
                  np.zeros((buffer, 4)), np.zeros((buffer, 1, 128, H, W)), np.zeros((buffer, 128, H, W)),
                  np.zeros((buffer, 128, H, W)), 0)
    return OracleSide(ofe.Graph(v, params, max_factors=48, device=device))
