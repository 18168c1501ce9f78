"""A/B of flow_encoder[0]'s kernels at the C3 shape (2048 edges of 48x64), one
process, interleaved rounds (A/B build: droid_fe_set_variant): 0 =
flow_enc0_kernel (16 waves, weights in LDS), 1 = flow_enc0_rw_kernel (8 waves,
weights in VGPRs, 64 pixels x 64 channels per wave), 2 = the same on 128 pixels x
32 channels per wave.  Prints each variant's output hash (they must agree: same
operands, same K order) and its median time.
Run with DROID_HIP_LIB=droid-slam_amd/lib/ab/libdroid_hip.so."""
import ctypes
import hashlib
import os
# its knobs are testing hooks (include/droid_backends_testing.h): the A/B library by default
os.environ.setdefault("DROID_HIP_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                                    "droid-slam_amd", "lib", "ab", "libdroid_hip.so"))
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "droid-slam_amd"))
import droid_backends  # noqa: E402
from droid_backends._lib import lib  # noqa: E402
from droid_mi355x.fused import pack_flow_enc0  # noqa: E402

lib.droid_fe_set_variant.argtypes = [ctypes.c_int]
lib.droid_fe_set_variant.restype = ctypes.c_int
dev = torch.device("cuda:0")
E, H, W = int(os.environ.get("E", "2048")), 48, 64
g = torch.Generator(device=dev).manual_seed(5)
motn = (8 * torch.randn((E, 4, H, W), generator=g, device=dev)).clamp(-64, 64)
w = pack_flow_enc0(torch.randn((128, 4, 7, 7), generator=g, device=dev) / 14.0)
b = torch.randn(128, generator=g, device=dev) * 0.1
outs = {v: torch.empty((E, H, W, 128), dtype=torch.float16, device=dev) for v in (0, 1, 2)}
for v in (0, 1, 2):
    lib.droid_fe_set_variant(v)
    droid_backends.flow_enc0_f16(motn, w, b, out=outs[v])
torch.cuda.synchronize()
for v in (0, 1, 2):
    print("variant %d hash %s" % (v, hashlib.sha1(outs[v].view(torch.int16).cpu().numpy().tobytes()).hexdigest()))
print("bitwise equal:", torch.equal(outs[0], outs[1]), torch.equal(outs[0], outs[2]))
ts = {0: [], 1: [], 2: []}
for r in range(10):
    for v in ((0, 1, 2) if r % 2 == 0 else (2, 1, 0)):
        lib.droid_fe_set_variant(v)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(5):
            droid_backends.flow_enc0_f16(motn, w, b, out=outs[v])
        e.record()
        torch.cuda.synchronize()
        ts[v].append(s.elapsed_time(e) / 5)
gb = outs[0].numel() * 2 / 1e9 + motn.numel() * 4 / 1e9
for v in (0, 1, 2):
    t = sorted(ts[v])
    print("variant %d: median %.3f ms (min %.3f), %.0f GB/s (output + input)" % (v, t[len(t) // 2], t[0],
                                                                              gb / t[len(t) // 2] * 1e3))
lib.droid_fe_set_variant(1)
