"""The frame graph's bookkeeping and the frontend's sequence, restated on the
CPU over the oracle's update() (TEST INFRASTRUCTURE ONLY, see
oracle/__init__.py): the checker for trajectory-level parity - many update()
calls with edge edits in between, as a real run makes them.

  Video          DepthVideo state + distance()        depth_video.py:22-38, 149-179
  Graph          FactorGraph edge edits + update()    factor_graph.py:43-242, 292-369
  frontend_*     DroidFrontend.__initialize/__update  droid_frontend.py:35-106

Conventions kept from the reference: edges are appended in call order; the
inactive store keeps (ii, jj, target, weight) of removed edges (store=True);
rm_keyframe shifts frame ix+1 into ix and renumbers every edge index >= ix
(its edges die); the max_factors cap removes by POSITION through argsort(age)
(factor_graph.py:105-106, kept literally; ties broken stably - torch.argsort
leaves that order unspecified).  The state the reference carries in fp16
(per-edge net, the update operator's outputs) is rounded to fp16.
"""
import numpy as np

from . import factor_graph as ofg
from . import geometry as og


class Video:
    """poses (N,7) fp64, disps / disps_sens (N,H,W) fp64, intrinsics (N,4),
    fmaps (N,rig,128,H,W), nets / inps (N,128,H,W) fp32 (values of the
    reference's fp16 buffers); counter = frames in use."""

    def __init__(self, poses, disps, disps_sens, intrinsics, fmaps, nets, inps, counter):
        self.poses = np.array(poses, np.float64)
        self.disps = np.array(disps, np.float64)
        self.disps_sens = np.array(disps_sens, np.float64)
        self.intrinsics = np.array(intrinsics, np.float64)
        self.fmaps = np.array(fmaps, np.float32)
        self.nets = np.array(nets, np.float32)
        self.inps = np.array(inps, np.float32)
        self.counter = int(counter)
        self.stereo = self.fmaps.shape[1] > 1

    def distance(self, ii, jj, beta=0.3, bidirectional=True):
        """depth_video.py:149-179 (frame_distance in both directions, averaged)."""
        n = self.counter
        p = self.poses[:n]
        d1 = og.frame_distance(p, self.disps, self.intrinsics[0], ii, jj, beta, dtype=np.float32)
        if not bidirectional:
            return d1
        d2 = og.frame_distance(p, self.disps, self.intrinsics[0], jj, ii, beta, dtype=np.float32)
        return 0.5 * (d1 + d2)

    def reproject(self, ii, jj):
        coords, _ = og.projective_transform(self.poses, self.disps, self.intrinsics, ii, jj, dtype=np.float32)
        return coords.astype(np.float64)


class Graph:
    """factor_graph.py's FactorGraph on the oracle.  params: UpdateModule
    state dict (numpy)."""

    def __init__(self, video, params, max_factors=-1, device=None):
        self.video = video
        self.params = params
        self.device = device      # torch device of the fp32 update operator (None: CPU)
        self.max_factors = max_factors
        N, H, W = video.disps.shape
        self.ht, self.wd = H, W
        z = lambda: np.zeros(0, np.int64)
        self.ii, self.jj, self.age = z(), z(), z()
        self.ii_inac, self.jj_inac, self.ii_bad, self.jj_bad = z(), z(), z(), z()
        self.net = np.zeros((0, 128, H, W), np.float32)
        self.inp = np.zeros((0, 128, H, W), np.float32)
        self.target = np.zeros((0, H, W, 2))
        self.weight = np.zeros((0, H, W, 2))
        self.target_inac = np.zeros((0, H, W, 2))
        self.weight_inac = np.zeros((0, H, W, 2))
        self.damping = 1e-6 * np.ones_like(video.disps)       # :29
        self.has_corr = False

    @property
    def _ii(self):
        return self.ii

    def add_factors(self, ii, jj, remove=False):
        """:85-133"""
        ii = np.asarray(ii, np.int64).reshape(-1)
        jj = np.asarray(jj, np.int64).reshape(-1)
        have = set(zip(self.ii.tolist(), self.jj.tolist())) | set(zip(self.ii_inac.tolist(), self.jj_inac.tolist()))
        keep = np.array([(a, b) not in have for a, b in zip(ii.tolist(), jj.tolist())], bool)
        ii, jj = ii[keep], jj[keep]
        if len(ii) == 0:
            return
        if self.max_factors > 0 and len(self.ii) + len(ii) > self.max_factors and self.has_corr and remove:
            order = np.argsort(self.age, kind="stable")
            self.rm_factors(order >= self.max_factors - len(ii), store=True)
        v = self.video
        self.net = np.concatenate([self.net, v.nets[ii]])
        self.inp = np.concatenate([self.inp, v.inps[ii]])
        self.has_corr = True
        target = v.reproject(ii, jj)
        self.ii = np.concatenate([self.ii, ii])
        self.jj = np.concatenate([self.jj, jj])
        self.age = np.concatenate([self.age, np.zeros(len(ii), np.int64)])
        self.target = np.concatenate([self.target, target])
        self.weight = np.concatenate([self.weight, np.zeros_like(target)])

    def rm_factors(self, mask, store=False):
        """:136-160"""
        mask = np.asarray(mask, bool).reshape(-1)
        if store:
            self.ii_inac = np.concatenate([self.ii_inac, self.ii[mask]])
            self.jj_inac = np.concatenate([self.jj_inac, self.jj[mask]])
            self.target_inac = np.concatenate([self.target_inac, self.target[mask]])
            self.weight_inac = np.concatenate([self.weight_inac, self.weight[mask]])
        k = ~mask
        self.ii, self.jj, self.age = self.ii[k], self.jj[k], self.age[k]
        self.net, self.inp = self.net[k], self.inp[k]
        self.target, self.weight = self.target[k], self.weight[k]

    def rm_keyframe(self, ix):
        """:164-193"""
        v = self.video
        for buf in (v.poses, v.disps, v.disps_sens, v.intrinsics, v.nets, v.inps, v.fmaps):
            buf[ix] = buf[ix + 1]
        m = (self.ii_inac == ix) | (self.jj_inac == ix)
        self.ii_inac = np.where(self.ii_inac >= ix, self.ii_inac - 1, self.ii_inac)
        self.jj_inac = np.where(self.jj_inac >= ix, self.jj_inac - 1, self.jj_inac)
        if m.any():
            self.ii_inac, self.jj_inac = self.ii_inac[~m], self.jj_inac[~m]
            self.target_inac, self.weight_inac = self.target_inac[~m], self.weight_inac[~m]
        m = (self.ii == ix) | (self.jj == ix)
        self.ii = np.where(self.ii >= ix, self.ii - 1, self.ii)
        self.jj = np.where(self.jj >= ix, self.jj - 1, self.jj)
        self.rm_factors(m, store=False)

    def add_neighborhood_factors(self, t0, t1, r=3):
        """:292-302"""
        ii, jj = np.meshgrid(np.arange(t0, t1), np.arange(t0, t1), indexing="ij")
        ii, jj = ii.reshape(-1), jj.reshape(-1)
        c = 1 if self.video.stereo else 0
        keep = (np.abs(ii - jj) > c) & (np.abs(ii - jj) <= r)
        self.add_factors(ii[keep], jj[keep])

    def proximity_distances(self, t0=0, t1=0, beta=0.25):
        t = self.video.counter
        ii, jj = np.meshgrid(np.arange(t0, t), np.arange(t1, t), indexing="ij")
        return self.video.distance(ii.reshape(-1), jj.reshape(-1), beta=beta)

    def proximity_edge_list(self, d, t0=0, t1=0, rad=2, nms=2, thresh=16.0):
        """:305-368 after video.distance (oracle/factor_graph.proximity_edges)."""
        return ofg.proximity_edges(d, t0, t1, self.video.counter, rad, nms, thresh,
                                   np.concatenate([self.ii, self.ii_bad, self.ii_inac]),
                                   np.concatenate([self.jj, self.jj_bad, self.jj_inac]), self.video.stereo,
                                   self.max_factors)

    def add_proximity_factors(self, t0=0, t1=0, rad=2, nms=2, beta=0.25, thresh=16.0, remove=False):
        es = self.proximity_edge_list(self.proximity_distances(t0, t1, beta), t0, t1, rad, nms, thresh)
        self.add_factors(es[:, 0], es[:, 1], remove)

    def update(self, t0=None, t1=None, itrs=2, use_inactive=False, EP=1e-7, motion_only=False):
        """:197-242 through oracle/factor_graph.update (fp16 outputs)."""
        v = self.video
        n = v.poses.shape[0]
        out = ofg.update(self.params, v.poses, v.disps, v.disps_sens, v.intrinsics, v.fmaps, self.ii, self.jj,
                         self.net, self.inp, self.target, self.weight, self.damping, t0=t0, t1=t1, itrs=itrs,
                         use_inactive=use_inactive, EP=EP, motion_only=motion_only,
                         inactive=(self.ii_inac, self.jj_inac, self.target_inac, self.weight_inac),
                         torch_corr=True, f16_outputs=True, device=self.device)
        self.net = out["net"].astype(np.float16).astype(np.float32)
        self.target, self.weight, self.damping = out["target"], out["weight"], out["damping"]
        v.poses[:n] = out["poses"]
        v.disps[:n] = out["disps"]
        self.age = self.age + 1
        return out
