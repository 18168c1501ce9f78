"""Bound on serving the z|r epilogue's h from LDS: the
factored ConvGRU z|r gate conv at the C3 shape (2048 edges of 48x64, 256
source frames) on the A/B library, with and without its global re-read of h
(DROID_ZR_NO_H=1 drops it - r*h becomes r, a timing bound only, not a result).
HIP events, alternating, median of 9 each."""
import os
import sys

import numpy as np
import torch

os.environ.setdefault("DROID_HIP_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                                    "droid-slam_amd", "lib", "ab", "libdroid_hip.so"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "droid-slam_amd"))
import droid_backends  # noqa: E402
from droid_backends import EPI_GRU_ZR  # noqa: E402
from droid_mi355x.fused import pack_conv  # noqa: E402

dev = torch.device("cuda:0")
B, H, W, F_ = 2048, 48, 64, 256
g = torch.Generator(device=dev).manual_seed(3)
mk = lambda n, c: torch.randn((n, H, W, c), generator=g, device=dev).half()
h = torch.tanh(mk(B, 128).float()).half()
cf, ff = mk(B, 128), mk(B, 64)
pre = mk(F_, 384)
idx = torch.arange(B, device=dev) * F_ // B
wzr = pack_conv(torch.randn((256, 320, 3, 3), generator=g, device=dev) / 40, [128, 128, 64])
bzr = torch.randn(256, generator=g, device=dev)
bbzr = torch.randn((B, 256), generator=g, device=dev)
z, rn = (torch.empty((B, H, W, 128), dtype=torch.float16, device=dev) for _ in range(2))
assert droid_backends.conv_gate_tile(EPI_GRU_ZR, B, H, W) == 0   # the 8-wave 256x256 band tile (the C3 default)


def run(no_h):
    os.environ["DROID_ZR_NO_H"] = "1" if no_h else "0"
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    droid_backends.conv_gru_pre_f16([(h, 0, 128), (cf, 0, 128), (ff, 0, 64)], wzr, 256, bzr, bbzr, EPI_GRU_ZR, pre,
                                    idx, 0, h=h, zout=z, rnet=rn)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e)


for _ in range(3):
    run(False), run(True)
ts = {False: [], True: []}
for _ in range(9):
    for m in (False, True):
        ts[m].append(run(m))
a, b = np.median(ts[False]), np.median(ts[True])
print("z|r C3, 8-wave tile: with the h re-read %.3f ms, without %.3f ms (%.1f %%); per-launch h bytes %.2f GB"
      % (a, b, 100 * (b - a) / a, B * H * W * 128 * 2 / 1e9))
