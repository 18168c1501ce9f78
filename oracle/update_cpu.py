"""CPU baseline of one FactorGraph.update() (factor_graph.py:196-242), built from
the oracle restatements - the "reference's pure-PyTorch CPU path" that
BASELINE.md asks for does not exist in the reference (droid_backends is
CUDA-only, geom/ba.py needs lietorch), so this restatement stands in for it.

Used only by bench.py's cpu_baseline leg.  Timed on a bounded sample:
  per-edge stages (reproject + motion features, CorrBlock volume + 4-level
  lookup, UpdateModule fp32) on `sample_edges` edges, scaled to all edges;
  BA (ba_cuda semantics, fp64) for ONE Gauss-Newton iteration on the full
  graph, scaled by the iteration count.
"""
import time

import numpy as np
import torch

from . import ba as oba
from . import corr as oc
from . import geometry as og
from . import update_module as oum


def time_update(prob, fmaps, nets, inps, params, sample_edges=8, iterations=2, threads=None):
    if threads:
        torch.set_num_threads(threads)
    ii, jj = prob["ii"], prob["jj"]
    E = len(ii)
    S = min(sample_edges, E)
    N, H, W = prob["disps"].shape
    intr = np.tile(prob["intrinsics"][None], (N, 1))
    p = {k: torch.from_numpy(v) for k, v in params.items()}

    t = time.perf_counter()
    si, sj = ii[:S], jj[:S]
    coords1, _ = og.projective_transform(prob["poses"], prob["disps"], intr, si, sj, dtype=np.float32)
    grid = og.coords_grid(H, W, np.float32)
    target = coords1  # first update: target == reprojection
    motn = np.concatenate([coords1 - grid, target - coords1], -1).transpose(0, 3, 1, 2).clip(-64, 64)
    f1 = fmaps[si][None].astype(np.float32)
    f2 = fmaps[sj][None].astype(np.float32)
    pyr = [v.astype(np.float32) for v in oc.corr_pyramid(f1, f2)]
    corr = oc.lookup_pyramid(pyr, coords1[None].astype(np.float32), 3)
    with torch.no_grad():
        oum.update_module(p, torch.from_numpy(nets[si][None].astype(np.float32)),
                          torch.from_numpy(inps[si][None].astype(np.float32)), torch.from_numpy(corr),
                          torch.from_numpy(motn[None].astype(np.float32)), torch.from_numpy(si),
                          torch.from_numpy(sj))
    t_edges = time.perf_counter() - t

    t = time.perf_counter()
    oba.ba(**{k: prob[k] for k in ("poses", "disps", "intrinsics", "disps_sens", "targets", "weights", "eta",
                                   "ii", "jj", "t0", "t1")}, iterations=1, lm=1e-4, ep=0.1, motion_only=False)
    t_ba = time.perf_counter() - t
    total = t_edges * (E / S) + t_ba * iterations
    return dict(seconds_per_update=total, t_edge_sample=t_edges, sample_edges=S, t_ba_iter=t_ba,
                threads=torch.get_num_threads())
