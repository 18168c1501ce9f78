"""A/B of the 64-channel band tile's stage shape (A/B build:
droid_conv_set_pair) on flow_encoder[2] at the C3 shape - 3x3 128 -> 64 + ReLU
over 2048 edges of 48x64 (conv_band_kernel<384, 64, .., ILV>): two-tap stages
(1, the product's) vs one-tap stages (0), interleaved rounds in one process;
the outputs must be bitwise equal.
Run with DROID_HIP_LIB=droid-slam_amd/lib/ab/libdroid_hip.so."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "droid-slam_amd"))
import droid_backends  # noqa: E402
from droid_backends._lib import lib  # noqa: E402
from droid_mi355x.fused import pack_conv  # noqa: E402

lib.droid_conv_set_pair.argtypes = [ctypes.c_int]
lib.droid_conv_set_pair.restype = ctypes.c_int
dev = torch.device("cuda:0")
E, H, W, cin, cout = int(os.environ.get("E", "2048")), 48, 64, 128, 64
g = torch.Generator(device=dev).manual_seed(11)
x = torch.relu(torch.randn((E, H, W, cin), generator=g, device=dev)).half()
w = torch.randn((cout, cin, 3, 3), generator=g, device=dev) / (cin * 9) ** 0.5
b = torch.randn(cout, generator=g, device=dev) * 0.1
wp = pack_conv(w, [cin])
outs = {v: torch.empty((E, H, W, cout), dtype=torch.float16, device=dev) for v in (0, 1)}
for v in (0, 1):
    lib.droid_conv_set_pair(v)
    droid_backends.conv_nhwc_f16([(x, 0, cin)], wp, cout, 3, bias=b, act=1, out=outs[v])
torch.cuda.synchronize()
print("two-tap vs one-tap stages bitwise equal:", torch.equal(outs[0], outs[1]))
ts = {0: [], 1: []}
for r in range(10):
    for v in ((0, 1) if r % 2 == 0 else (1, 0)):
        lib.droid_conv_set_pair(v)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(5):
            droid_backends.conv_nhwc_f16([(x, 0, cin)], wp, cout, 3, bias=b, act=1, out=outs[v])
        e.record()
        torch.cuda.synchronize()
        ts[v].append(s.elapsed_time(e) / 5)
flops = 2.0 * cin * cout * 9 * E * H * W
for v in (0, 1):
    t = sorted(ts[v])
    print("pair=%d: median %.3f ms (min %.3f) = %.0f TFLOP/s" % (v, t[len(t) // 2], t[0], flops / t[len(t) // 2] / 1e9))
lib.droid_conv_set_pair(1)
