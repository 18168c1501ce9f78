"""rocSOLVER (via torch.linalg) dense fp64 Cholesky + solve timings for the
reduced-camera-system sizes, for comparison with the hand-written kernels."""
import torch
import time
dev = torch.device("cuda:0")
for n in (48, 762, 1530, 3066):
    A = torch.randn(n, n, dtype=torch.float64, device=dev)
    A = A @ A.T + n * torch.eye(n, dtype=torch.float64, device=dev)
    b = torch.randn(n, 1, dtype=torch.float64, device=dev)
    for _ in range(3):
        L, info = torch.linalg.cholesky_ex(A)
        x = torch.cholesky_solve(b, L)
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        L, info = torch.linalg.cholesky_ex(A)
        x = torch.cholesky_solve(b, L)
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    print("n=%5d  potrf+potrs %.3f ms" % (n, min(ts)), flush=True)
