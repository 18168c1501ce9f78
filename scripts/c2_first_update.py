"""Host-time breakdown of the first update() after a frontend edge change
(scripts only): wraps the pieces of FactorGraph.update with perf_counter
timers (no device sync inside), then runs rm + add + update twice.

usage: python scripts/c2_first_update.py"""
import argparse
import os
import sys
import time
from collections import defaultdict

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
T = defaultdict(float)


def wrap(obj, name, label):
    f = getattr(obj, name)

    def g(*a, **k):
        t0 = time.perf_counter()
        r = f(*a, **k)
        T[label] += 1000 * (time.perf_counter() - t0)
        return r
    setattr(obj, name, g)


wrap(graph, "_ba_inputs", "_ba_inputs")
wrap(graph, "_dev", "_dev")
wrap(graph.update_op, "forward", "update_op")
wrap(graph.video, "ba", "video.ba")
wrap(droid_backends, "head_finish", "head_finish")
wrap(droid_backends, "eta_damping", "eta_damping")
wrap(droid_backends, "projective_transform", "projective_transform")
wrap(droid_backends, "BaPlan", "BaPlan()")
with torch.no_grad():
    for _ in range(3):
        graph.update(use_inactive=True)
    torch.cuda.synchronize()
    for c in range(3):
        sel = (graph._ii == 15) & (graph._jj == 12) | (graph._ii == 12) & (graph._jj == 15)
        graph.rm_factors(sel, store=False)
        graph.add_factors(np.array([15, 12]), np.array([12, 15]))
        droid_backends._PLAN_CACHE.clear()
        torch.cuda.synchronize()
        for tag in ("first", "second"):
            T.clear()
            t0 = time.perf_counter()
            graph.update(use_inactive=True)
            host = 1000 * (time.perf_counter() - t0)
            torch.cuda.synchronize()
            print("%s update: host %.3f ms: " % (tag, host) + ", ".join("%s %.3f" % kv for kv in sorted(T.items())))
