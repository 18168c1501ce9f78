"""Time the ConvGRU gate convs (droid_conv_gru_pre_f16, factored per-frame inp
term) and a plain 3x3 128->128 band conv at the C3 shape (2048 edges of 48x64,
256 source frames) on each W=64 tile policy (droid_conv_set_tile: 0 = 8-wave
band tiles, 1 = the two-workgroups-per-CU tile).  HIP events, median of 5."""
import os
# its knobs are testing hooks (include/droid_backends_testing.h): the A/B library by default
os.environ.setdefault("DROID_HIP_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                                    "droid-slam_amd", "lib", "ab", "libdroid_hip.so"))
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "droid-slam_amd"))
import droid_backends  # noqa: E402
from droid_backends import EPI_GRU_Q, EPI_GRU_ZR  # noqa: E402
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
wq = pack_conv(torch.randn((128, 320, 3, 3), generator=g, device=dev) / 40, [128, 128, 64])
w1 = pack_conv(torch.randn((128, 128, 3, 3), generator=g, device=dev) / 30, [128])
bzr, bq, b1 = (torch.randn(n, generator=g, device=dev) for n in (256, 128, 128))
bbzr, bbq = torch.randn((B, 256), generator=g, device=dev), torch.randn((B, 128), generator=g, device=dev)
z, rn, hn, o1 = (torch.empty((B, H, W, 128), dtype=torch.float16, device=dev) for _ in range(4))


def zr():
    droid_backends.conv_gru_pre_f16([(h, 0, 128), (cf, 0, 128), (ff, 0, 64)], wzr, 256, bzr, bbzr, EPI_GRU_ZR, pre,
                                    idx, 0, h=h, zout=z, rnet=rn)


def q():
    droid_backends.conv_gru_pre_f16([(rn, 0, 128), (cf, 0, 128), (ff, 0, 64)], wq, 128, bq, bbq, EPI_GRU_Q, pre,
                                    idx, 256, h=h, z=z, out=hn)


def c128():
    droid_backends.conv_nhwc_f16([(cf, 0, 128)], w1, 128, 3, bias=b1, act=1, out=o1)


def timed(fn, reps=5):
    fn()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    return float(np.median(ts))


flop = {"z|r": 2 * 256 * 320 * 9, "q": 2 * 128 * 320 * 9, "128->128": 2 * 128 * 128 * 9}
res = {}
for mode in (0, 1):
    droid_backends.conv_set_tile(mode)
    for name, fn in (("z|r", zr), ("q", q), ("128->128", c128)):
        ms = timed(fn)
        res[(mode, name)] = ms
        print("tile %d %-9s %.3f ms  %.0f TFLOP/s" % (mode, name, ms, flop[name] * B * H * W / ms / 1e9), flush=True)
droid_backends.conv_set_tile(-1)
outs = {}
for mode in (0, 1):
    droid_backends.conv_set_tile(mode)
    zr(); q()
    torch.cuda.synchronize()
    outs[mode] = (z.clone(), rn.clone(), hn.clone())
droid_backends.conv_set_tile(-1)
print("max |tile0 - tile1|: z %.3g  rh %.3g  h' %.3g" % tuple(float((a.float() - b.float()).abs().max())
                                                           for a, b in zip(outs[0], outs[1])))
