"""Does the tile order's grouping of edges by source frame matter for the
factored z|r gate conv?  Times droid_conv_gru_pre_f16 (EPI_GRU_ZR, 256x256
band tile) at C3 shapes (2048 edges, 256 frames, 48x64) with HIP events for
three pre_idx layouts: edges grouped by frame (8 consecutive edges share one
per-frame term), the C3 graph's own order, and a random permutation.

usage: python scripts/pre_order_probe.py [--reps N]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "droid-slam_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import droid_backends  # noqa: E402
from droid_mi355x import synthetic  # noqa: E402
from droid_mi355x.fused import EPI_GRU_ZR, pack_conv  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=20)
args = ap.parse_args()
dev = torch.device("cuda:0")
E, U, H, W = 2048, 256, 48, 64
g = torch.Generator(device="cpu").manual_seed(0)
r16 = lambda *s: (torch.randn(*s, generator=g) * 0.5).half().to(dev)
net, cf, ff = r16(E, H, W, 128), r16(E, H, W, 128), r16(E, H, W, 64)
wp = pack_conv((torch.randn(256, 320, 3, 3, generator=g) * 0.02).to(dev), [128, 128, 64])
bias = (torch.randn(256, generator=g) * 0.1).to(dev)
bb = (torch.randn(E, 256, generator=g) * 0.1).to(dev)
pre = r16(U, H, W, 384)
z, rn = torch.empty_like(net), torch.empty_like(net)
ii, _ = synthetic.c3_edges()
orders = {
    "grouped by frame": np.repeat(np.arange(U), E // U),
    "C3 graph order": np.unique(ii, return_inverse=True)[1],
    "random": np.random.default_rng(1).permutation(np.repeat(np.arange(U), E // U)),
}
for name, idx in orders.items():
    pidx = torch.as_tensor(idx.astype(np.int64), device=dev)
    run = lambda: droid_backends.conv_gru_pre_f16([(net, 0, 128), (cf, 0, 128), (ff, 0, 64)], wp, 256, bias, bb,
                                                  EPI_GRU_ZR, pre, pidx, 0, h=net, zout=z, rnet=rn)
    for _ in range(3):
        run()
    ts = []
    for _ in range(args.reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); run(); b.record(); torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    print("%-18s ZR conv %.3f ms (median of %d)" % (name, float(np.median(ts)), args.reps), flush=True)
