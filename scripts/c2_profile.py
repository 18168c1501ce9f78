"""Where the C2 frontend's time goes (scripts only): host issue vs GPU time of
one update(use_inactive=True), and the pieces of a per-keyframe edge change
(rm_factors, add_factors with the new edges' corr volume, the first update on
the new edge set with its BA plan build), each timed with a device sync.

usage: python scripts/c2_profile.py"""
import argparse
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "droid-slam_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import droid_backends  # noqa: E402

args = argparse.Namespace(config="C2", frames=16, edges=2048, ht=384, wd=512, corr="volume", lowmem=False,
                          reference_op=False, force_dist=False, reference_layout=False)
dev = torch.device("cuda:0")
video, graph, _, e_local = bench.build_state(args, 0, 1, dev)


def timed(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    return 1000 * (t1 - t0), 1000 * (time.perf_counter() - t0)


with torch.no_grad():
    for _ in range(3):
        graph.update(use_inactive=True)
    st = [timed(lambda: graph.update(use_inactive=True)) for _ in range(10)]
    print("steady update: host issue %.3f ms, wall %.3f ms" % tuple(np.median(np.array(st), 0)))
    rows = []
    for c in range(5):
        sel = (graph._ii == 15) & (graph._jj == 12) | (graph._ii == 12) & (graph._jj == 15)
        r = timed(lambda: graph.rm_factors(sel, store=False))
        a = timed(lambda: graph.add_factors(np.array([15, 12]), np.array([12, 15])))
        droid_backends._PLAN_CACHE.clear()
        u1 = timed(lambda: graph.update(use_inactive=True))
        u2 = timed(lambda: graph.update(use_inactive=True))
        rows.append([r[1], a[0], a[1], u1[0], u1[1], u2[1]])
    m = np.median(np.array(rows), 0)
    print("edge change: rm_factors %.3f ms, add_factors host %.3f / wall %.3f ms, first update host %.3f / wall %.3f ms, "
          "second update %.3f ms" % tuple(m))
