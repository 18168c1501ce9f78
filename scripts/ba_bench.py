"""Time droid_backends.ba (itrs=2) per config with HIP events, and the host
cost of building its plan (the analyse step: kx, Schur rows, assembly lists,
pose order, tile structure, task list) - what an edge-set change costs.

usage: python scripts/ba_bench.py [C2 C3 C5 ...] [--reps N] [--hw H W]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "droid-slam_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import droid_backends  # noqa: E402
from droid_mi355x import synthetic  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("configs", nargs="*", default=["C3"])
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--hw", type=int, nargs=2, default=[48, 64])
args = ap.parse_args()
dev = torch.device("cuda:0")
for cfg in args.configs:
    prob = synthetic.ba_problem(cfg, H=args.hw[0], W=args.hw[1])
    t = {k: torch.from_numpy(prob[k]).to(dev) for k in ("poses", "disps", "intrinsics", "disps_sens", "targets",
                                                         "weights", "eta", "ii", "jj")}
    N, H, W = prob["disps"].shape
    h0 = time.perf_counter()
    plan = droid_backends.BaPlan(prob["ii"], prob["jj"], N, H, W, prob["t0"], prob["t1"], prob["eta"].shape[0],
                                 False, dev)
    torch.cuda.synchronize()
    plan_ms = 1000 * (time.perf_counter() - h0)
    p0, d0 = t["poses"].clone(), t["disps"].clone()
    times = []
    for r in range(args.reps + 1):
        t["poses"].copy_(p0)
        t["disps"].copy_(d0)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        h0 = time.perf_counter()
        s.record()
        plan.run(t["poses"], t["disps"], t["intrinsics"], t["disps_sens"], t["targets"], t["weights"], t["eta"],
                 2, 1e-5, 1e-2)
        e.record()
        h1 = time.perf_counter()
        torch.cuda.synchronize()
        plan.check_status()
        if r > 0:
            times.append((s.elapsed_time(e), 1000 * (h1 - h0)))
    print("%s E=%d P=%d order=%s wide=%d tasks=%d tiles(input)=%d: plan build %.1f ms (host), "
          "ba(itrs=2) gpu %.3f ms, host-issue %.3f ms (median of %d)"
          % (cfg, len(prob["ii"]), plan.P, plan.order, plan.num_wide, plan.ntasks, plan.system.shape[0], plan_ms,
             np.median([a for a, _ in times]), np.median([b for _, b in times]), args.reps), flush=True)
