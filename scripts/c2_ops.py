"""Which torch ops run inside one C2 update(use_inactive=True) (scripts only):
torch.profiler op table (CPU-side op counts and their device kernels), to find
the small copies / fills / elementwise kernels around the HIP kernels.

usage: python scripts/c2_ops.py [C2|C3]"""
import argparse
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "droid-slam_amd")]
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

import bench  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
args = argparse.Namespace(config=cfg, frames=16 if cfg == "C2" else 256, edges=2048, ht=384, wd=512, corr="volume",
                          lowmem=False, reference_op=False, force_dist=False, reference_layout=False)
dev = torch.device("cuda:0")
video, graph, _, e_local = bench.build_state(args, 0, 1, dev)
kw = dict(use_inactive=True) if cfg == "C2" else {}
with torch.no_grad():
    for _ in range(3):
        graph.update(**kw)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        for _ in range(5):
            graph.update(**kw)
        torch.cuda.synchronize()
print(prof.key_averages(group_by_input_shape=True).table(sort_by="count", row_limit=60, max_name_column_width=40,
                                                          max_shapes_column_width=60))
