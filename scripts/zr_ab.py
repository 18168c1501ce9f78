"""Factored z|r gate conv (conv_gru_pre_f16, EPI_GRU_ZR with the per-frame
term) at E edges of 48x64 on the library DROID_HIP_LIB names: HIP-event time
and sha256 digests of z and r*h, for a bitwise comparison between libraries.
usage: zr_ab.py E"""
import hashlib
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "droid-slam_amd"))
import torch

import droid_backends
from droid_backends import EPI_GRU_ZR
from droid_mi355x.fused import pack_conv

E = int(sys.argv[1])
H, W = 48, 64
F = max(1, E // 8)
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
t = lambda n, c, s=0.5: (torch.randn((n, H, W, c), generator=g, device=dev) * s).half()
h, cf, ff = torch.tanh(t(E, 128, 1.0)), t(E, 128), t(E, 64)
pre = t(F, 384)
idx = (torch.arange(E, device=dev) // 8).clamp(max=F - 1).to(torch.int64)
w = torch.randn((256, 320, 3, 3), generator=g, device=dev) * 0.02
b = torch.randn(256, generator=g, device=dev) * 0.1
bb = torch.randn((E, 256), generator=g, device=dev) * 0.1
wp = pack_conv(w, [128, 128, 64])
z = torch.empty((E, H, W, 128), dtype=torch.float16, device=dev)
rn = torch.empty_like(z)
ts = []
for it in range(12):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    droid_backends.conv_gru_pre_f16([(h, 0, 128), (cf, 0, 128), (ff, 0, 64)], wp, 256, b, bb, EPI_GRU_ZR, pre, idx,
                                    0, h=h, zout=z, rnet=rn)
    e.record()
    torch.cuda.synchronize()
    if it >= 2:
        ts.append(s.elapsed_time(e))
ts.sort()
dig = lambda x: hashlib.sha256(x.cpu().numpy().tobytes()).hexdigest()[:16]
print("lib %s E %d: min %.3f ms median %.3f ms  z %s  r*h %s" % (
    os.environ.get("DROID_HIP_LIB", "default"), E, ts[0], ts[len(ts) // 2], dig(z), dig(rn)), flush=True)
