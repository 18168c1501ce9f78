"""Timeline of the dataflow Cholesky (profiling build: make -C
droid-slam_amd/csrc prof) on one BA iteration of a config: per potrf task
(the critical chain) the phase durations in us, the hand-off gap to the next
potrf, and the other task types' durations.

usage: python scripts/chol_timeline.py [C3|C5]"""
import ctypes
import os
import sys

_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "droid-slam_amd", "lib", "prof", "libdroid_hip.so")
os.environ.setdefault("DROID_HIP_LIB", _LIB)
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "droid-slam_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import droid_backends  # noqa: E402
from droid_backends._lib import lib  # noqa: E402
from droid_mi355x import synthetic  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
dev = torch.device("cuda:0")
prob = synthetic.ba_problem(cfg)
t = {k: torch.from_numpy(prob[k]).to(dev) for k in ("poses", "disps", "intrinsics", "disps_sens", "targets",
                                                     "weights", "eta")}
N, H, W = prob["disps"].shape
plan = droid_backends.BaPlan(prob["ii"], prob["jj"], N, H, W, prob["t0"], prob["t1"], prob["eta"].shape[0], False, dev)
prof = torch.zeros((plan.ntasks, 8), dtype=torch.int64, device=dev)
for it in range(3):
    if it == 2:
        assert lib.droid_chol_set_profile(ctypes.c_void_p(prof.data_ptr())) == 0
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    plan.run(t["poses"], t["disps"], t["intrinsics"], t["disps_sens"], t["targets"], t["weights"], t["eta"], 1,
             1e-5, 1e-2)
    e.record()
    torch.cuda.synchronize()
    print("ba(itrs=1) %.3f ms" % s.elapsed_time(e))
lib.droid_chol_set_profile(ctypes.c_void_p(0))
p = prof.cpu().numpy().astype(np.float64) / 100.0   # us
t0 = p[p[:, 0] > 0, 0].min()
print("%s: n=%d tasks=%d, Cholesky span %.1f us" % (cfg, plan.P * 6, plan.ntasks, p[:, 7].max() - t0))
pot = np.nonzero(p[:, 3] > 0)[0]
pot = pot[np.argsort(p[pot, 0])]
# stamps: 0 ticket, 1 deps met, 2 last update applied, 3 panels done, 6 A(k+1,k) ready,
# 5 trsm(k+1,k) done (pivot tiles published right after), 4 L_kk^-1 done, 7 task end
names = ["wait deps", "last update", "panels", "diag inv + trsm(k+1,k)", "stores+publish+Linv", "Linv store"]
rows = []
for a, k in enumerate(pot):
    r = p[k]
    b5 = r[5] if r[5] > 0 else r[3]
    ph = [r[1] - r[0], r[2] - r[1], r[3] - r[2], b5 - r[3], r[4] - b5, r[7] - r[4]]
    step = (p[pot[a + 1], 2] - r[2]) if a + 1 < len(pot) else np.nan
    rows.append(ph + [r[7] - r[0], step])
rows = np.array(rows)
print("potrf tasks (%d): median us: " % len(pot) + ", ".join("%s %.2f" % (nm, v) for nm, v in zip(
    names + ["total", "chain step (panels start -> next panels start)"], np.nanmedian(rows, 0))))
below = p[pot, 5] > 0
wa = (p[pot, 6] - p[pot, 3])[below]
print("wait for A(k+1,k)'s other updates after the panels: median %.2f us, p90 %.2f, %d of %d > 0.5 us" % (
    np.median(wa), np.percentile(wa, 90), int((wa > 0.5).sum()), len(wa)))
other = np.setdiff1d(np.nonzero(p[:, 7] > 0)[0], pot)
dur = p[other, 7] - p[other, 1]
print("other tasks (%d): median work %.2f us, median wait %.2f us" % (len(other), np.median(dur), np.median(p[other, 1] - p[other, 0])))
# where the chain waits: potrf(k+1)'s other updates done (its stamp 1) vs potrf(k)'s trsm(k+1,k) (stamp 5)
late = np.array([p[pot[a + 1], 1] - p[pot[a], 5] for a in range(len(pot) - 1)])
print("other updates of A(k+1,k+1) done after potrf(k) published: %d of %d steps, median %.2f us (p90 %.2f); "
      "last-update phase when not late: median %.2f us" % ((late > 0).sum(), len(late), np.median(late),
                                                            np.percentile(late, 90),
                                                            np.median(rows[1:, 1][late <= 0]) if (late <= 0).any() else np.nan))
for a in range(min(6, len(pot))):
    print("  potrf #%d: " % a + " ".join("%.2f" % v for v in rows[a]))
