"""Host issue time of one FactorGraph.update() (Python + ctypes launches, no
sync) vs its GPU time, per config: if the host part approaches the GPU part,
small graphs (the frontend, or each rank of an 8-way sharded C3) become launch
bound.  usage: python scripts/host_overhead.py [C2|C3] [--edges E --frames N]"""
import argparse
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "droid-slam_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("config", nargs="?", default="C3")
ap.add_argument("--edges", type=int, default=2048)
ap.add_argument("--frames", type=int, default=256)
a = ap.parse_args()
args = argparse.Namespace(config=a.config, frames=16 if a.config == "C2" else a.frames, edges=a.edges, ht=384, wd=512,
                          corr="volume", lowmem=False, reference_op=False, force_dist=False, reference_layout=False)
dev = torch.device("cuda:0")
video, graph, _, e_local = bench.build_state(args, 0, 1, dev)
kw = dict(use_inactive=True) if a.config == "C2" else {}
with torch.no_grad():
    for _ in range(3):
        graph.update(**kw)
    torch.cuda.synchronize()
    host, tot = [], []
    for _ in range(10):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        graph.update(**kw)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        host.append(1000 * (t1 - t0))
        tot.append(1000 * (t2 - t0))
print("%s edges=%d: host issue %.3f ms, issue+drain %.3f ms (median of 10)" % (a.config, e_local, np.median(host),
                                                                              np.median(tot)))
