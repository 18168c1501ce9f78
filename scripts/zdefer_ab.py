"""A/B of DROID_ZDEFER (z|r stores z's gate argument, q applies the sigmoid):
time the two gate convs at the C3 shape (2048 edges of 48x64, 256 source
frames, default tile policy) and hash the new hidden state h' - the two
builds must give the same bytes.  DROID_HIP_LIB selects the build
(droid-slam_amd/lib/v_zd0/libdroid_hip.so = DROID_ZDEFER=0)."""
import hashlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "droid-slam_amd"))
import droid_backends  # noqa: E402
from droid_backends import EPI_GRU_Q, EPI_GRU_ZR  # noqa: E402
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
wq = pack_conv(torch.randn((128, 320, 3, 3), generator=g, device=dev) / 40, [128, 128, 64])
bzr, bq = torch.randn(256, generator=g, device=dev), torch.randn(128, generator=g, device=dev)
bbzr, bbq = torch.randn((B, 256), generator=g, device=dev), torch.randn((B, 128), generator=g, device=dev)
z, rn, hn = (torch.empty((B, H, W, 128), dtype=torch.float16, device=dev) for _ in range(3))


def zr():
    droid_backends.conv_gru_pre_f16([(h, 0, 128), (cf, 0, 128), (ff, 0, 64)], wzr, 256, bzr, bbzr, EPI_GRU_ZR, pre,
                                    idx, 0, h=h, zout=z, rnet=rn)


def q():
    droid_backends.conv_gru_pre_f16([(rn, 0, 128), (cf, 0, 128), (ff, 0, 64)], wq, 128, bq, bbq, EPI_GRU_Q, pre,
                                    idx, 256, h=h, z=z, out=hn)


def timed(fn, reps=9):
    fn()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    return float(np.median(ts)), float(np.min(ts))


zr(); q()
torch.cuda.synchronize()
hh = hashlib.sha1(hn.view(torch.int16).cpu().numpy().tobytes()).hexdigest()
hr = hashlib.sha1(rn.view(torch.int16).cpu().numpy().tobytes()).hexdigest()
tz, tq = timed(zr), timed(q)
print("%s: z|r %.3f ms (min %.3f)  q %.3f ms (min %.3f)  sum %.3f  h' %s  r*h %s" % (
    os.path.basename(os.path.dirname(os.environ.get("DROID_HIP_LIB", "lib/x"))), tz[0], tz[1], tq[0], tq[1],
    tz[0] + tq[0], hh[:16], hr[:16]), flush=True)
