"""Time droid_backends.ba on a config (default C3) with HIP events."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "droid-slam_amd"))
import numpy as np
import torch

import droid_backends
from droid_mi355x import synthetic

cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
prob = synthetic.ba_problem(cfg)
dev = torch.device("cuda:0")
t = {k: torch.from_numpy(prob[k]).to(dev) for k in ("poses", "disps", "intrinsics", "disps_sens", "targets",
                                                     "weights", "eta", "ii", "jj")}
p0, d0 = t["poses"].clone(), t["disps"].clone()
times = []
for r in range(reps + 1):
    t["poses"].copy_(p0)
    t["disps"].copy_(d0)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    h0 = time.perf_counter()
    s.record()
    droid_backends.ba(t["poses"], t["disps"], t["intrinsics"], t["disps_sens"], t["targets"], t["weights"], t["eta"],
                      t["ii"], t["jj"], prob["t0"], prob["t1"], 2, 1e-4, 0.1, False,
                      ii_host=prob["ii"], jj_host=prob["jj"])
    e.record()
    h1 = time.perf_counter()
    torch.cuda.synchronize()
    if r > 0:
        times.append((s.elapsed_time(e), 1000 * (h1 - h0)))
print("%s ba(itrs=2): gpu %.3f ms, host-issue %.3f ms (median of %d)" %
      (cfg, np.median([a for a, _ in times]), np.median([b for _, b in times]), reps))
