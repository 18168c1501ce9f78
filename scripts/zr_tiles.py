"""A/B of the factored ConvGRU z|r gate conv (droid_conv_gru_pre_f16, C3 shape:
2048 edges of 48x64, 256 source frames) on the 8-wave 256x256 band tile
(droid_conv_set_tile(0)) and the software-pipelined 4-wave tile (2): HIP
events, alternating, median of 7 per tile; the outputs must be bitwise equal
(same products in the same order)."""
import os
import sys

import numpy as np
import torch

# the 4-wave tile ships in the A/B build (make ab)
os.environ.setdefault("DROID_HIP_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                                    "droid-slam_amd", "lib", "ab", "libdroid_hip.so"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "droid-slam_amd"))
import droid_backends  # noqa: E402
from droid_backends import EPI_GRU_ZR  # noqa: E402
from droid_mi355x.fused import pack_conv  # noqa: E402

dev = torch.device("cuda:0")
B, H, W, F_ = int(os.environ.get("GATE_EDGES", "2048")), 48, 64, 256
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


def zr():
    droid_backends.conv_gru_pre_f16([(h, 0, 128), (cf, 0, 128), (ff, 0, 64)], wzr, 256, bzr, bbzr, EPI_GRU_ZR, pre,
                                    idx, 0, h=h, zout=z, rnet=rn)


def timed(fn):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e)


flop = 2 * 256 * 320 * 9 * B * H * W
modes = (0, 2)
ts = {m: [] for m in modes}
outs = {}
for m in modes:
    droid_backends.conv_set_tile(m)
    print("tile %d -> kernel %d" % (m, droid_backends.conv_gate_tile(EPI_GRU_ZR, B, H, W)), flush=True)
    zr()
    torch.cuda.synchronize()
    outs[m] = (z.clone(), rn.clone())
for _ in range(7):
    for m in modes:
        droid_backends.conv_set_tile(m)
        ts[m].append(timed(zr))
droid_backends.conv_set_tile(-1)
for m in modes:
    ms = float(np.median(ts[m]))
    print("tile %d z|r %.3f ms (min %.3f)  %.0f TFLOP/s" % (m, ms, min(ts[m]), flop / ms / 1e9), flush=True)
same = all(torch.equal(a, b) for a, b in zip(outs[0], outs[2]))
print("bitwise equal:", same, " max|dz| %.3g" % float((outs[0][0].float() - outs[2][0].float()).abs().max()))
