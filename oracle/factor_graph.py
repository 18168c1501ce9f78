"""One FactorGraph.update() composed from the oracle restatements (CPU,
fp32 / fp64) - the whole-iteration checker for droid_mi355x.FactorGraph.update.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Follows /root/reference/droid_slam/factor_graph.py:196-242 step by step:
  :201-204  coords1 = reproject(ii, jj); motn = [coords1 - coords0,
            target - coords1] -> (E,4,H,W), clamped to +-64
  :206      corr = CorrBlock(coords1): the 4-level r=3 lookup of the volume
            <fmap1[ii]/4, fmap2[jj]/4> (stereo edges read the right image,
            factor_graph.py:112-114)
  :208-209  net, delta, weight, damping, upmask = update_op(...)
  :211-213  t0 = max(1, ii.min() + 1) when None
  :215-219  target = coords1 + delta; weight; damping[unique(ii)] = damping
  :221-227  use_inactive: stored edges with ii, jj >= t0 - 3 join the BA
  :229-235  damping = 0.2 * damping[unique(ii)] + EP; targets / weights
            permuted to (E,2,H,W); video.ba(..., itrs, lm=1e-4, ep=0.1)
  depth_video.py:181-193  t1 = max(ii, jj) + 1; disps.clamp_(min=0.001)
"""
import numpy as np
import torch

from . import ba as oba
from . import corr as oc
from . import geometry as og
from . import update_module as oum


def update(params, poses, disps, disps_sens, intrinsics, fmaps, ii, jj, net, inp, target, weight, damping,
           t0=None, t1=None, itrs=2, use_inactive=False, EP=1e-7, motion_only=False, inactive=None, lm=1e-4,
           ep=0.1, torch_corr=False, f16_outputs=False, device=None):
    """params: UpdateModule state dict (numpy); poses (N,7), disps/disps_sens
    (N,H,W), intrinsics (N,4), fmaps (N,rig,128,H,W); ii/jj (E); net/inp
    (E,128,H,W); target/weight (E,H,W,2); damping (N,H,W); inactive =
    (ii, jj, target, weight) of the stored edges.  Inputs are not mutated.
    update_lowmem (factor_graph.py:245-290) is one call per step with t0=1,
    t1=counter, lm=1e-5, ep=1e-2 (its alt correlation equals the volume's up
    to fp16 rounding, corr.py:91-139).

    torch_corr: the pyramid + lookup as torch fp32 matmul / avg_pool2d /
    grid_sample (oracle/corr.py *_torch, equal to the loop restatement,
    tests/test_oracle_golden.py) - the same values, fast enough for replays of
    whole frontend sequences.  f16_outputs: round the update operator's
    outputs (net, delta, weight, eta) to fp16, as the reference's autocast
    region stores them (factor_graph.py:209-220) - for multi-update replays
    whose state the reference carries in fp16.  device: a torch device for
    the torch_corr lookup and the fp32 update operator (the plain-torch
    reference of the same ops; TF32 must be off); the BA stays fp64 numpy.

    Returns dict(net, target, weight, damping, coords1, ba_in=(targets, weights,
    eta, ii, jj, t0, t1), poses, disps)."""
    p = {k: torch.from_numpy(np.asarray(v, np.float32)) for k, v in params.items()}
    ii = np.asarray(ii, np.int64)
    jj = np.asarray(jj, np.int64)
    N, H, W = disps.shape
    E = len(ii)
    coords1, _ = og.projective_transform(poses, disps, intrinsics, ii, jj)
    grid = og.coords_grid(H, W)
    motn = np.concatenate([coords1 - grid, target - coords1], -1).transpose(0, 3, 1, 2).clip(-64.0, 64.0)
    rig = fmaps.shape[1]
    f1 = fmaps[ii, 0].astype(np.float32)
    f2 = fmaps[jj, np.where((ii == jj) & (rig > 1), 1, 0)].astype(np.float32)
    dv = torch.device("cpu") if device is None else torch.device(device)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dv)
    if dv.type != "cpu":
        p = {k: v.to(dv) for k, v in p.items()}
    if torch_corr:
        pyr = oc.corr_pyramid_torch(T(f1[None]), T(f2[None]))
        corr = oc.lookup_pyramid_torch(pyr, T(coords1.astype(np.float32)), 3)[None]
        del pyr
    else:
        pyr = oc.corr_pyramid(f1[None], f2[None])
        corr = T(oc.lookup_pyramid(pyr, coords1[None].astype(np.float32), 3))
    with torch.no_grad():
        net1, delta, weight1, eta, _ = oum.update_module(
            p, T(np.asarray(net, np.float32))[None], T(np.asarray(inp, np.float32))[None],
            corr, T(motn[None].astype(np.float32)), T(ii), T(jj))
    if f16_outputs:
        net1, delta, weight1, eta = (x.half().float() for x in (net1, delta, weight1, eta))
    net1, delta, weight1, eta = (x.cpu() for x in (net1, delta, weight1, eta))
    if t0 is None:
        t0 = max(1, int(ii.min()) + 1)
    target = coords1 + delta[0].double().numpy()
    weight = weight1[0].double().numpy()
    damping = np.array(damping, dtype=np.float64)
    damping[np.unique(ii)] = eta[0].double().numpy()
    if use_inactive and inactive is not None:
        i_in, j_in, t_in, w_in = inactive
        m = (i_in >= t0 - 3) & (j_in >= t0 - 3)
        ii_ba = np.concatenate([i_in[m], ii])
        jj_ba = np.concatenate([j_in[m], jj])
        tgt = np.concatenate([t_in[m], target])
        wgt = np.concatenate([w_in[m], weight])
    else:
        ii_ba, jj_ba, tgt, wgt = ii, jj, target, weight
    eta_ba = 0.2 * damping[np.unique(ii_ba)] + EP
    tgt = tgt.transpose(0, 3, 1, 2)
    wgt = wgt.transpose(0, 3, 1, 2)
    if t1 is None:
        t1 = int(max(ii_ba.max(), jj_ba.max())) + 1
    out = oba.ba(poses, disps, intrinsics[0], disps_sens, tgt, wgt, eta_ba, ii_ba, jj_ba, t0, t1, itrs, lm, ep,
                 motion_only)
    return dict(net=net1[0].double().numpy(), target=target, weight=weight, damping=damping, coords1=coords1,
                ba_in=(tgt, wgt, eta_ba, ii_ba, jj_ba, t0, t1), poses=out["poses"],
                disps=np.maximum(out["disps"], 0.001))


def proximity_edges(d, t0, t1, t, rad, nms, thresh, ii_all, jj_all, stereo, max_factors):
    """FactorGraph.add_proximity_factors (reference factor_graph.py:305-369)
    after video.distance, restated line by line: d = the float32 distances of
    the meshgrid [t0, t) x [t1, t) (row-major), ii_all/jj_all = ii|ii_bad|ii_inac,
    jj|jj_bad|jj_inac.  Returns the edge list es (k, 2) int64 in the
    reference's order (static edges, then accepted pairs (i, j), (j, i)).
    argsort is stable here; torch.argsort's order among equal distances is
    unspecified (the fixtures use distinct distances)."""
    d = np.array(d, dtype=np.float32).reshape(-1).copy()
    ncol = t - t1
    ii, jj = np.meshgrid(np.arange(t0, t), np.arange(t1, t), indexing="ij")
    ii, jj = ii.reshape(-1), jj.reshape(-1)
    d[ii - rad < jj] = np.inf                                     # :316
    with np.errstate(invalid="ignore"):
        d[d > 100] = np.inf                                       # :317

    def suppress(i, j):                                           # :321-330, :361-366
        for di in range(-nms, nms + 1):
            for dj in range(-nms, nms + 1):
                if abs(di) + abs(dj) <= max(min(abs(i - j) - 2, nms), 0):
                    i1, j1 = i + di, j + dj
                    if t0 <= i1 < t and t1 <= j1 < t:
                        d[(i1 - t0) * ncol + (j1 - t1)] = np.inf

    for i, j in zip(np.asarray(ii_all).tolist(), np.asarray(jj_all).tolist()):
        suppress(i, j)
    es = []
    for i in range(t0, t):                                        # :333-341 (negative indices wrap)
        if stereo:
            es.append((i, i))
            d[(i - t0) * ncol + (i - t1)] = np.inf
        for j in range(max(i - rad - 1, 0), i):
            es.append((i, j))
            es.append((j, i))
            d[(i - t0) * ncol + (j - t1)] = np.inf
    for k in np.argsort(d, kind="stable"):                        # :343-366 (NaN sorts last)
        if d[k] > thresh:
            continue
        if len(es) > max_factors:
            break
        i, j = int(ii[k]), int(jj[k])
        es.append((i, j))
        es.append((j, i))
        suppress(i, j)
    return np.asarray(es, dtype=np.int64).reshape(-1, 2)
