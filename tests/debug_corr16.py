"""Diagnostic: locate fp16 lookup mismatches of the generic kernel vs the oracle."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "droid-slam_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
import torch
import droid_backends
from oracle import corr as oc
rng = np.random.default_rng(11)
B, H, W, H2, W2 = 3, 12, 16, 12, 16
vol = rng.normal(size=(B, H, W, H2, W2)).astype(np.float16)
base = np.stack(np.meshgrid(np.arange(W) * W2 / W, np.arange(H) * H2 / H), 0)[None]
c = base + rng.normal(0, 3.0, (B, 2, H, W))
c[:, :, 0, 0] = -50.0; c[:, 0, 0, 1] = W2 - 0.5; c[:, 1, 1, 0] = -0.25
coords = c.astype(np.float32)
out, = droid_backends.corr_index_forward(torch.from_numpy(vol).cuda(), torch.from_numpy(coords).cuda(), 3)
got = out.cpu().numpy()
ref = oc.corr_index_forward(vol, coords, 3)
bad = np.argwhere(got.view(np.uint16) != ref.view(np.uint16))
print("mismatches", len(bad))
for n, i, j, y, x in bad[:10]:
    x0, y0 = coords[n, 0, y, x], coords[n, 1, y, x]
    fx, fy = np.floor(x0), np.floor(y0)
    dx, dy = np.float32(x0 - fx), np.float32(y0 - fy)
    t = lambda a, b: vol[n, y, x, int(fy) - 3 + b, int(fx) - 3 + a] if (0 <= int(fx)-3+a < W2 and 0 <= int(fy)-3+b < H2) else np.float16(0)
    taps = [t(i, j), t(i, j + 1), t(i + 1, j), t(i + 1, j + 1)]
    ws = [(1 - dx) * (1 - dy), (1 - dx) * dy, dx * (1 - dy), dx * dy]
    print(n, i, j, y, x, "x0,y0", x0, y0, "dx,dy", dx, dy, "taps", taps, "w16", [np.float16(w) for w in ws],
          "got", got[n, i, j, y, x], "ref", ref[n, i, j, y, x])
