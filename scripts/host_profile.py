"""cProfile of the host side of FactorGraph.update() (Python + ctypes launch
issue) on a bench state, after warm-up: where the issue time of a small graph
goes.  usage: python scripts/host_profile.py [C2|C3] [N_UPDATES]"""
import argparse
import cProfile
import os
import pstats
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "droid-slam_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 50
args = argparse.Namespace(config=cfg, frames=16 if cfg == "C2" else 256, edges=2048, ht=384, wd=512,
                          corr="volume", lowmem=False, reference_op=False)
dev = torch.device("cuda:0")
video, graph, _, _ = bench.build_state(args, 0, 1, dev)
kw = dict(use_inactive=True) if cfg == "C2" else {}
with torch.no_grad():
    for _ in range(5):
        graph.update(**kw)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(n):
        graph.update(**kw)
    pr.disable()
    torch.cuda.synchronize()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(35)
st.sort_stats("cumulative").print_stats(30)
