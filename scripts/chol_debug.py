import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "droid-slam_amd"))
import numpy as np
import torch
import droid_backends
sizes = [int(a) for a in sys.argv[1:]] or [6]
for n in sizes:
    rng = np.random.default_rng(n)
    Q, _ = np.linalg.qr(rng.normal(size=(n, n)))
    A = (Q * np.geomspace(1, 1e3, n)) @ Q.T
    b = rng.normal(size=n)
    for rep in range(3):
        t = time.time()
        dx, failed = droid_backends.dense_spd_solve(torch.tensor(A, device="cuda:0"), torch.tensor(b, device="cuda:0"), 0.0, 0.0)
        torch.cuda.synchronize()
        print("n %d rep %d: %.3fs failed=%s err=%.3g" % (n, rep, time.time() - t, failed,
              np.abs(dx.cpu().numpy() - np.linalg.solve(A, b)).max()), flush=True)
