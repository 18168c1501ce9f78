"""Time droid_flow_enc0_f16 (flow_encoder[0], 7x7 4 -> 128 + ReLU) at the C3 shape
(2048 edges of 48x64) with HIP events and print ms, output GB/s and a hash of
the output (DROID_FE_TP=128 / 256 selects the tile; the bytes must agree)."""
import hashlib
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "droid-slam_amd"))
import droid_backends  # noqa: E402
from droid_mi355x.fused import pack_flow_enc0  # noqa: E402

dev = torch.device("cuda:0")
E, H, W = 2048, 48, 64
g = torch.Generator(device=dev).manual_seed(5)
motn = (8 * torch.randn((E, 4, H, W), generator=g, device=dev)).clamp(-64, 64)
w = pack_flow_enc0(torch.randn((128, 4, 7, 7), generator=g, device=dev) / 14.0)
b = torch.randn(128, generator=g, device=dev) * 0.1
out = torch.empty((E, H, W, 128), dtype=torch.float16, device=dev)
for _ in range(3):
    droid_backends.flow_enc0_f16(motn, w, b, out=out)
torch.cuda.synchronize()
print("hash", hashlib.sha1(out.view(torch.int16).cpu().numpy().tobytes()).hexdigest())
ts = []
for _ in range(10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    droid_backends.flow_enc0_f16(motn, w, b, out=out)
    e.record()
    torch.cuda.synchronize()
    ts.append(s.elapsed_time(e))
ts.sort()
gb = out.numel() * 2 / 1e9 + motn.numel() * 4 / 1e9
print("DROID_FE_TP=%s: median %.3f ms (min %.3f), %.0f GB/s (output + input)" % (
    os.environ.get("DROID_FE_TP", "256"), ts[len(ts) // 2], ts[0], gb / ts[len(ts) // 2] * 1e3))
