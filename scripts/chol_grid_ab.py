"""BA(itrs=2) time by the dataflow Cholesky's worker count (DROID_CHOL_GRID, read
per launch by the A/B build: run with DROID_HIP_LIB=droid-slam_amd/lib/ab/...),
grid sizes alternated in one process so clock drift spreads over all of them.

usage: python scripts/chol_grid_ab.py [C3 C5 ...] [--grids 0 256 ...] [--reps N]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "droid-slam_amd"))
import torch  # noqa: E402

import droid_backends  # noqa: E402
from droid_mi355x import synthetic  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("configs", nargs="*", default=["C3"])
ap.add_argument("--grids", type=int, nargs="+", default=[0, 256])
ap.add_argument("--reps", type=int, default=6)
ap.add_argument("--rounds", type=int, default=3)
args = ap.parse_args()
dev = torch.device("cuda:0")
for cfg in args.configs:
    prob = synthetic.ba_problem(cfg, H=48, W=64)
    t = {k: torch.from_numpy(prob[k]).to(dev) for k in ("poses", "disps", "intrinsics", "disps_sens", "targets",
                                                         "weights", "eta", "ii", "jj")}
    N, H, W = prob["disps"].shape
    plan = droid_backends.BaPlan(prob["ii"], prob["jj"], N, H, W, prob["t0"], prob["t1"], prob["eta"].shape[0],
                                 False, dev)
    p0, d0 = t["poses"].clone(), t["disps"].clone()
    res = {g: [] for g in args.grids}
    out = {}
    for rnd in range(args.rounds):
        for g in args.grids:
            os.environ["DROID_CHOL_GRID"] = str(g)
            for r in range(args.reps + 1):
                t["poses"].copy_(p0)
                t["disps"].copy_(d0)
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                plan.run(t["poses"], t["disps"], t["intrinsics"], t["disps_sens"], t["targets"], t["weights"],
                         t["eta"], 2, 1e-5, 1e-2)
                e.record()
                torch.cuda.synchronize()
                plan.check_status()
                if r > 0:
                    res[g].append(s.elapsed_time(e))
            if g not in out:
                out[g] = t["poses"].clone()
    ref = out[args.grids[0]]
    for g in args.grids:
        v = sorted(res[g])
        print("%s grid %4s: BA(itrs=2) min %.3f median %.3f ms  max|dposes| vs grid %s: %.2e" % (
            cfg, g if g else "dflt", v[0], v[len(v) // 2], args.grids[0] or "dflt",
            float((out[g] - ref).abs().max())), flush=True)
