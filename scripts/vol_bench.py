"""Time droid_corr_volume_pyramid (add_factors' per-edge volume build) at the C3
shape: 2048 edges of 48x64 over 256 frames, tiled layout, HIP events.  Prints
ms, written GB/s and a hash of a 64-edge build (compare kernels across runs:
DROID_VOL_VARIANT=1 / 2 / 3 selects the kernel)."""
import hashlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "droid-slam_amd"))
import droid_backends  # noqa: E402

dev = torch.device("cuda:0")
NF, H, W, E = 256, 48, 64, int(os.environ.get("VOL_EDGES", "2048"))
g = torch.Generator(device=dev).manual_seed(7)
f = (torch.randn((NF, H, W, 128), generator=g, device=dev) / 4).half()
rng = np.random.default_rng(3)
f1 = torch.from_numpy(rng.integers(0, NF, E).astype(np.int32)).to(dev)
f2 = torch.from_numpy(rng.integers(0, NF, E).astype(np.int32)).to(dev)
h = hashlib.sha1()
for tiled in (True, False):
    lv = droid_backends.corr_volume_pyramid(f, f1[:64], f2[:64], tiled)
    for x in lv:
        h.update(x.cpu().numpy().tobytes())
    del lv
print("hash64", h.hexdigest())
bytes_ = E * sum((H * W) * (((H >> l) + 7) // 8 * 8) * (W >> l) * 2 for l in range(4))
for rep in range(3):
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    lv = droid_backends.corr_volume_pyramid(f, f1, f2, True)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e)
    print("variant %s rep %d: %.2f ms, %.2f GB written, %.0f GB/s" % (
        "v" + os.environ.get("DROID_VOL_VARIANT", "4"), rep, ms, bytes_ / 1e9, bytes_ / ms / 1e6), flush=True)
    del lv
