"""Median launch time of corr_alt_ce0 on the C3 bench coordinates (2048 edges,
48x64) for the library in $DROID_HIP_LIB (scripts/alt_ablate.sh variants)."""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."),
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "droid-slam_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import droid_backends  # noqa: E402
from droid_mi355x import synthetic  # noqa: E402
from droid_mi355x.corr import AltCorrBlock  # noqa: E402
from oracle import geometry as og  # noqa: E402

H, W, n = 48, 64, 256
rng = np.random.default_rng(1003)
ii, jj = synthetic.c3_edges(256, 2048, rng=np.random.default_rng(1003))
gt = synthetic.trajectory(n, rng)
poses, disps = synthetic.perturb(gt, synthetic.smooth_disps(n, H, W, rng), rng)
coords, _ = og.projective_transform(poses, disps, np.tile(synthetic.INTRINSICS, (n, 1)), ii, jj)
dev = torch.device("cuda:0")
fm = torch.randn((1, n, 128, H, W), device=dev).half()
pyr = [lv.view((-1,) + tuple(lv.shape[2:])) for lv in AltCorrBlock(fm).pyramid]
c = torch.from_numpy(coords.astype(np.float32)).to(dev).contiguous()
w = (torch.randn((128, 224), device=dev) / 14).half()
w[:, 196:] = 0
b = torch.zeros(128, device=dev)
f1 = torch.as_tensor(ii, dtype=torch.int32, device=dev)
f2 = torch.as_tensor(jj, dtype=torch.int32, device=dev)
ts = []
for it in range(8):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    droid_backends.corr_alt_ce0(pyr, f1, f2, c, w, b)
    e.record()
    torch.cuda.synchronize()
    ts.append(s.elapsed_time(e))
print("%s: median %.3f ms (min %.3f)" % (os.environ.get("DROID_HIP_LIB", "default"), float(np.median(ts[2:])), min(ts)))
