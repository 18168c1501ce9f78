"""Per-task timeline of the dataflow Cholesky (DROID_CHOL_TPROF): where the
critical path of an n x n solve spends its time."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "droid-slam_amd"))
import numpy as np
import torch
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1530
tprof = torch.zeros(65536 + 16 * 64, dtype=torch.int64, device="cuda:0")
torch.cuda.synchronize()
os.environ["DROID_CHOL_TPROF"] = str(tprof.data_ptr())
import droid_backends
rng = np.random.default_rng(n)
A = rng.normal(size=(n, n)) / np.sqrt(n)
A = A @ A.T + np.eye(n)
b = rng.normal(size=n)
Ad, bd = torch.tensor(A, device="cuda:0"), torch.tensor(b, device="cuda:0")
for it in range(4):
    tprof.zero_()
    dx, failed = droid_backends.dense_spd_solve(Ad, bd, 0.0, 0.0)
    torch.cuda.synchronize()
err = np.abs(dx.cpu().numpy() - np.linalg.solve(A, b)).max()
P = tprof[65536:].view(-1, 16).cpu().numpy()
T = tprof[:65536].view(-1, 4).cpu().numpy()
T = T[T[:, 3] > 0]
names = {0: "potrf", 1: "trsm", 2: "update", 3: "bsolve", 4: "bupd"}
t0 = T[:, 1].min()
T = T.astype(np.float64)
T[:, 1:] = (T[:, 1:] - t0) * 0.01  # 100 MHz ticks -> us
code = T[:, 0].astype(np.int64)
typ = (code >> 12) & 15
ti, tj, tk_ = (code >> 16) & 0xffff, (code >> 32) & 0xffff, (code >> 48) & 0xffff
print("n=%d tasks=%d span=%.1f us err=%.2g failed=%s" % (n, len(T), T[:, 3].max(), err, failed))
for t in sorted(set(typ)):
    m = typ == t
    print("%-7s n=%5d  wait(deps) mean %.2f us  work mean %.2f us  max %.2f" %
          (names.get(t, t), m.sum(), (T[m, 2] - T[m, 1]).mean(), (T[m, 3] - T[m, 2]).mean(), (T[m, 3] - T[m, 2]).max()))
# potrf chain
pot = np.where(typ == 0)[0]
print("critical chain per k: potrf(k) [got deps end] -> trsm(k+1,k) -> update(k+1,k+1,k)")
def find(t, i, j, k):
    m = np.where((typ == t) & (ti == i) & (tj == j) & (tk_ == k))[0]
    return m[0] if len(m) else None
for q in pot:
    k = tk_[q]
    s = "  k=%2d potrf %8.2f %8.2f %8.2f" % (k, T[q, 1], T[q, 2], T[q, 3])
    a = find(1, k + 1, k, k)
    if a is not None:
        s += " | trsm %8.2f %8.2f %8.2f" % tuple(T[a, 1:4])
    u = find(2, k + 1, k + 1, k)
    if u is not None:
        s += " | upd %8.2f %8.2f %8.2f" % tuple(T[u, 1:4])
    print(s)
np.save("gpurun_out/chol_timeline_%d.npy" % n, T)

print("potrf phase times (us, mean over k): stamp deltas")
P = P[:24].astype(np.float64)
valid = P[:, 0] > 0
D = np.diff(P[valid][:, :15], axis=1) * 0.01
print(" ".join("%.2f" % v for v in D.mean(0)))
