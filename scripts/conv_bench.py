"""Per-conv timing of the fused update operator at E edges (48x64), HIP events."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "droid-slam_amd"))
import torch

import droid_backends
from droid_mi355x.fused import pack_conv

E = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
ONLY = sys.argv[2] if len(sys.argv) > 2 else None
H, W = 48, 64
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
t = lambda c, n=E: (torch.randn((n, H, W, c), generator=g, device=dev) * 0.5).half()
net, inp, cf, ff, c200, m8 = t(128), t(128), t(128), t(64), t(200), t(8)
dw = t(256)
cases = {
    "ce0 1x1 200->128": ([(c200, 0, 200)], 128, 1, {}),
    "ce2 3x3 128->128": ([(net, 0, 128)], 128, 3, {}),
    "fe0 7x7 8->128": ([(m8, 0, 8)], 128, 7, {}),
    "fe2 3x3 128->64": ([(net, 0, 128)], 64, 3, {}),
    "zr 3x3 448->256": ([(net, 0, 128), (inp, 0, 128), (cf, 0, 128), (ff, 0, 64)], 256, 3, {}),
    "q 3x3 448->128": ([(net, 0, 128), (inp, 0, 128), (cf, 0, 128), (ff, 0, 64)], 128, 3, {}),
    "dw0 3x3 128->256": ([(net, 0, 128)], 256, 3, {}),
    "head 3x3 256->4": ([(dw, 0, 256)], 4, 3, {}),
}
flops_total = 0
for name, (srcs, cout, ks, kw) in cases.items():
    if ONLY and not name.startswith(ONLY):
        continue
    cin = sum(c for _, _, c in srcs)
    w = torch.randn((cout, cin, ks, ks), generator=g, device=dev) * 0.02
    wp = pack_conv(w, [c for _, _, c in srcs])
    bias = torch.zeros(cout, device=dev)
    out = torch.empty((E, H, W, cout), dtype=torch.float16, device=dev)
    for _ in range(2):
        droid_backends.conv_nhwc_f16(srcs, wp, cout, ks, bias=bias, act=1, out=out)
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        droid_backends.conv_nhwc_f16(srcs, wp, cout, ks, bias=bias, act=1, out=out)
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    ms = min(ts)
    real = 2.0 * E * H * W * cout * cin * ks * ks
    print("%-20s %8.3f ms  %7.0f TFLOP/s (useful)" % (name, ms, real / ms / 1e9), flush=True)

if not ONLY or ONLY == "dwhead":
    from droid_mi355x.fused import pack_head_taps
    w0 = torch.randn((256, 128, 3, 3), generator=g, device=dev) * 0.02
    hw = pack_head_taps(torch.randn((4, 256, 3, 3), generator=g, device=dev) * 0.02)
    wp, b0 = pack_conv(w0, [128]), torch.zeros(256, device=dev)
    head = torch.zeros((E, H, W, 4), device=dev)
    ts = []
    for it in range(7):
        head.zero_()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        droid_backends.conv_dw_head_f16([(net, 0, 128)], wp, b0, hw, head)
        e.record()
        torch.cuda.synchronize()
        if it >= 2:
            ts.append(s.elapsed_time(e))
    ms = min(ts)
    real = 2.0 * E * H * W * (256 * 128 * 9 + 4 * 256 * 9)
    print("%-20s %8.3f ms  %7.0f TFLOP/s (useful)" % ("dw0+head fused", ms, real / ms / 1e9), flush=True)
