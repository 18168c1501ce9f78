"""Direct band conv vs Winograd tile on the update operator's 3x3 convs at C3
(E edges of 48x64), HIP events around each launch (min of 7).  Run one
library build per process: `DROID_HIP_LIB=... python scripts/wino_bench.py [E]`."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "droid-slam_amd"))
import torch

import droid_backends
from droid_backends import EPI_GRU_Q, EPI_GRU_ZR
from droid_mi355x.fused import pack_conv, pack_conv_wino

E = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
H, W = 48, 64
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
t = lambda c, n=E: (torch.randn((n, H, W, c), generator=g, device=dev) * 0.5).half()
net, cf, ff = t(128), t(128), t(64)
U = E // 8
pre = t(384, U)
pidx = (torch.arange(E, device=dev) // 8).long()
srcs = [(net, 0, 128), (cf, 0, 128), (ff, 0, 64)]
wzr = torch.randn((256, 320, 3, 3), generator=g, device=dev) * 0.02
wq = torch.randn((128, 320, 3, 3), generator=g, device=dev) * 0.02
w1 = torch.randn((128, 128, 3, 3), generator=g, device=dev) * 0.02
bzr, bq, b1 = torch.zeros(256, device=dev), torch.zeros(128, device=dev), torch.zeros(128, device=dev)
gbzr, gbq = torch.zeros((E, 256), device=dev), torch.zeros((E, 128), device=dev)
z, rn, hn, o1 = t(128), t(128), t(128), t(128)
P = {"zr": pack_conv(wzr, [128, 128, 64]), "q": pack_conv(wq, [128, 128, 64]), "a": pack_conv(w1, [128]),
     "zrw": pack_conv_wino(wzr, [128, 128, 64]), "qw": pack_conv_wino(wq, [128, 128, 64]),
     "aw": pack_conv_wino(w1, [128])}
cases = {
    "zr direct": lambda: droid_backends.conv_gru_pre_f16(srcs, P["zr"], 256, bzr, gbzr, EPI_GRU_ZR, pre, pidx, 0,
                                                          h=net, zout=z, rnet=rn),
    "zr wino": lambda: droid_backends.conv_wino_f16(srcs, P["zrw"], 256, bzr, gbzr, epi=EPI_GRU_ZR, pre=pre,
                                                    pre_idx=pidx, pre_coff=0, h=net, zout=z, rnet=rn),
    "q direct": lambda: droid_backends.conv_gru_pre_f16(srcs, P["q"], 128, bq, gbq, EPI_GRU_Q, pre, pidx, 256,
                                                         h=net, z=z, out=hn),
    "q wino": lambda: droid_backends.conv_wino_f16(srcs, P["qw"], 128, bq, gbq, epi=EPI_GRU_Q, pre=pre,
                                                   pre_idx=pidx, pre_coff=256, h=net, z=z, out=hn),
    "128 direct": lambda: droid_backends.conv_nhwc_f16([(net, 0, 128)], P["a"], 128, 3, bias=b1, act=1, out=o1),
    "128 wino": lambda: droid_backends.conv_wino_f16([(net, 0, 128)], P["aw"], 128, bias=b1, act=1, out=o1),
}
from droid_mi355x.fused import pack_head_taps  # noqa: E402
wdw = torch.randn((256, 128, 3, 3), generator=g, device=dev) * 0.02
P["dw"] = pack_conv(wdw, [128])
hwt = pack_head_taps(torch.randn((4, 256, 3, 3), generator=g, device=dev) * 0.02)
bdw = torch.zeros(256, device=dev)
head = torch.zeros((E, H, W, 4), device=dev)
w64 = torch.randn((64, 128, 3, 3), generator=g, device=dev) * 0.02
P["w64"] = pack_conv(w64, [128])
o64, b64 = t(64), torch.zeros(64, device=dev)
cases["64 direct"] = lambda: droid_backends.conv_nhwc_f16([(net, 0, 128)], P["w64"], 64, 3, bias=b64, act=1, out=o64)
cases["dwhead direct"] = lambda: droid_backends.conv_dw_head_f16([(net, 0, 128)], P["dw"], bdw, hwt, head)
flops = {"dwhead": 2.0 * E * H * W * 256 * 128 * 9, "64": 2.0 * E * H * W * 64 * 128 * 9,
         "zr": 2.0 * E * H * W * 256 * 320 * 9, "q": 2.0 * E * H * W * 128 * 320 * 9,
         "128": 2.0 * E * H * W * 128 * 128 * 9}
only = sys.argv[2] if len(sys.argv) > 2 else None
for name, fn in cases.items():
    if only and only not in name:
        continue
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(7):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    ms = min(ts)
    print("%-12s %8.3f ms  %6.0f TFLOP/s (direct-conv FLOPs)  [%s]" % (name, ms, flops[name.split()[0]] / ms / 1e9,
                                                                        os.path.basename(os.environ.get("DROID_HIP_LIB", "default"))),
          flush=True)
