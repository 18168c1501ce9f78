"""Fused delta/weight head conv (conv_dw_head_f16) at E edges of 48x64: HIP-event
time and the fp32 head output, saved for a bitwise comparison between two
libraries (DROID_HIP_LIB).  usage: dwh_ab.py E out.npy"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "droid-slam_amd"))
import numpy as np
import torch

import droid_backends
from droid_mi355x.fused import pack_conv, pack_head_taps

E = int(sys.argv[1])
H, W = 48, 64
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
net = (torch.randn((E, H, W, 128), generator=g, device=dev) * 0.5).half()
w0 = torch.randn((256, 128, 3, 3), generator=g, device=dev) * 0.02
hw = pack_head_taps(torch.randn((4, 256, 3, 3), generator=g, device=dev) * 0.02)
b0 = torch.randn(256, generator=g, device=dev) * 0.05
wp = pack_conv(w0, [128])
head = torch.zeros((E, H, W, 4), device=dev)
ts = []
for it in range(12):
    head.zero_()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    droid_backends.conv_dw_head_f16([(net, 0, 128)], wp, b0, hw, head)
    e.record()
    torch.cuda.synchronize()
    if it >= 2:
        ts.append(s.elapsed_time(e))
ts.sort()
print("lib %s E %d: min %.3f ms median %.3f ms" % (os.environ.get("DROID_HIP_LIB", "default"), E, ts[0], ts[len(ts) // 2]),
      flush=True)
np.save(sys.argv[2], head.cpu().numpy())
