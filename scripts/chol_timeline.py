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
prof = torch.zeros((plan.ntasks, 24), dtype=torch.int64, device=dev)
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
nt = plan.ntasks
tasks = np.zeros(8 * nt, np.int32)
assert lib.droid_chol_plan_tasks(plan._h, tasks.ctypes.data_as(ctypes.c_void_p)) == 0
tasks = tasks.reshape(nt, 8)
typ = tasks[:, 0]
key = {(int(t[0]), int(t[1]), int(t[2]), int(t[3])): q for q, t in enumerate(tasks)}
pot = np.nonzero(typ == 0)[0]
pot = pot[np.argsort(p[pot, 0])]
# potrf stamps: 0 ticket (or chained start), 1 deps met, 2 last update's block column 0 applied (panels
# start), 3 panels done, 6 tile (k+1,k) in LDS and the D_p formed, 5 (k+1,k) solved + published, 7 end;
# 8 + 2p / 9 + 2p: wave 0's panel p start / end; 16 / 17 wave 1's D_p start / end; 18 tile solved; 19 stores issued
# (phase 4 - stamps 3 -> 6 - is the D_p, the L_kk stores and the barrier after which tile (k+1,k)
# is in LDS; phase 5 the tall_solve of (k+1,k), its stores and publish; until round 6 the labels
# read "wait A(k+1,k)" / "D + trsm(k+1,k) + publish")
names = ["wait deps", "L(k,klast) + col 0", "panels", "D_p + L_kk stores + barrier", "trsm(k+1,k) + publish", "end"]
rows = []
for a, k in enumerate(pot):
    r = p[k]
    ph = [r[1] - r[0], r[2] - r[1], r[3] - r[2], r[6] - r[3], r[5] - r[6], r[7] - r[5]]
    step = (p[pot[a + 1], 2] - r[2]) if a + 1 < len(pot) else np.nan
    rows.append(ph + [r[7] - r[0], step])
rows = np.array(rows)
print("potrf tasks (%d): median us: " % len(pot) + ", ".join("%s %.2f" % (nm, v) for nm, v in zip(
    names + ["total", "chain step (panels start -> next panels start)"], np.nanmedian(rows, 0))))
fac_end = p[pot, 5].max()
print("factor: first ticket -> last (k+1,k) publish %.1f us" % (fac_end - t0))
for ty, nm in ((1, "trsm"), (2, "update")):
    q = np.nonzero(typ == ty)[0]
    if len(q):
        print("%s tasks (%d): median us: wait deps %.2f, loads %.2f, compute %.2f, store+publish %.2f" % (
            nm, len(q), *np.median(np.stack([p[q, 1] - p[q, 0], p[q, 2] - p[q, 1], p[q, 3] - p[q, 2],
                                             p[q, 7] - p[q, 3]]), 1)))
# the second chain into potrf(k)'s tail: potrf(k-1) L_kk flag -> trsm(k+1,k-1) -> update(k+1,k,k-1) -> potrf(k) stamp 6
ch = []
for k in range(2, len(pot) - 1):
    tr = key.get((1, k + 1, k - 1, k - 1))
    up = key.get((2, k + 1, k, k - 1), tr)   # fused into the trsm task (its stamp 4: the update's inputs loaded)
    pk, pk1 = key[(0, k - 1, k - 1, k - 1)], key[(0, k, k, k)]
    if tr is None or up is None:
        continue
    base = p[pk, 3]
    up1 = p[up, 1] if up != tr else p[tr, 4]
    ch.append([p[tr, 1] - base, p[tr, 3] - base, up1 - base, p[up, 7] - base, p[pk1, 3] - base, p[pk1, 6] - base])
if ch:
    print("second chain, us after potrf(k-1)'s panels end (median): trsm(k+1,k-1) deps met %.2f / solved %.2f, "
          "update(k+1,k,k-1) inputs in %.2f / end %.2f; potrf(k) panels end %.2f, A(k+1,k) in LDS %.2f"
          % tuple(np.median(np.array(ch), 0)))
bc = np.nonzero(typ == 3)[0]
if len(bc):
    print("back solve: %d bcol tasks, last potrf publish -> last bcol end %.1f us; per bcol median: parent wait -> end %.2f us"
          % (len(bc), p[bc, 7].max() - fac_end, np.median((p[bc, 7] - np.where(p[bc, 3] > 0, p[bc, 3], p[bc, 2])))))
if len(bc) and os.environ.get("TL_BCOL"):
    o = bc[np.argsort(-tasks[bc, 1])]
    print("bcol c: ticket, deps met, rows done, parent x in, end (us after the last (k+1,k) publish)")
    for q in o:
        print("  bcol %3d: " % tasks[q, 1] + " ".join("%8.2f" % (p[q, s] - fac_end if p[q, s] > 0 else np.nan)
                                                  for s in (0, 1, 2, 3, 7)))
tl = []
for k in pot:   # the tail: wave 1's D_p (16 -> 17), the barrier (6), the tile solve (18), stores issued (19)
    r = p[k]
    if r[16] > 0 and r[19] > 0:
        tl.append([r[16] - r[3], r[17] - r[16], r[6] - r[17], r[18] - r[6], r[19] - r[18], r[5] - r[19]])
if tl:
    print("tail, median us: panels end -> D start %.2f, D_p %.2f, D end -> barrier %.2f, tall_solve %.2f, "
          "tile store issue %.2f, -> stamp 5 %.2f" % tuple(np.median(np.array(tl), 0)))
pp = []
for k in pot:   # wave 0's panels (stamps 8 + 2p / 9 + 2p) and the gaps between them (period overrun + lookahead)
    r = p[k]
    if r[8] > 0 and r[15] > 0:
        pp.append([r[9] - r[8], r[11] - r[10], r[13] - r[12], r[15] - r[14], r[10] - r[9], r[12] - r[11], r[14] - r[13]])
if pp:
    print("panels (wave 0), median us: p0 %.2f p1 %.2f p2 %.2f p3 %.2f; gaps p0->p1 %.2f p1->p2 %.2f p2->p3 %.2f"
          % tuple(np.median(np.array(pp), 0)))
if len(bc) and os.environ.get("TL_BCOL"):
    o = bc[np.argsort(-tasks[bc, 1])]
    print("bcol c: ticket, deps met, rows done, parent x in, end (us after the last (k+1,k) publish)")
    for q in o:
        print("  bcol %3d: " % tasks[q, 1] + " ".join("%8.2f" % (p[q, s] - fac_end if p[q, s] > 0 else np.nan)
                                                  for s in (0, 1, 2, 3, 7)))
tl = []
for k in pot:   # the tail: wave 1's D_p (16 -> 17), the barrier (6), the tile solve (18), stores issued (19)
    r = p[k]
    if r[16] > 0 and r[19] > 0:
        tl.append([r[16] - r[3], r[17] - r[16], r[6] - r[17], r[18] - r[6], r[19] - r[18], r[5] - r[19]])
if tl:
    print("tail, median us: panels end -> D start %.2f, D_p %.2f, D end -> barrier %.2f, tall_solve %.2f, "
          "tile store issue %.2f, -> stamp 5 %.2f" % tuple(np.median(np.array(tl), 0)))
pp = []
for k in pot:   # wave 0's panels (stamps 8 + 2p / 9 + 2p) and the gaps between them (period overrun + lookahead)
    r = p[k]
    if r[8] > 0 and r[15] > 0:
        pp.append([r[9] - r[8], r[11] - r[10], r[13] - r[12], r[15] - r[14], r[10] - r[9], r[12] - r[11], r[14] - r[13]])
if pp:
    print("panels (wave 0), median us: p0 %.2f p1 %.2f p2 %.2f p3 %.2f; gaps p0->p1 %.2f p1->p2 %.2f p2->p3 %.2f"
          % tuple(np.median(np.array(pp), 0)))
for a in range(min(6, len(pot))):
    print("  potrf #%d: " % a + " ".join("%.2f" % v for v in rows[a]))
