"""A/B of gru_glo_kernel's tile ring (A/B build: droid_glo_set_ring) at the C3
shape (2048 edges of 48x64 x 128 channels): ring 5 (80 KB, two workgroups per
CU) vs ring 3 (48 KB, three per CU) vs ring 2 (32 KB, five per CU), with 1 or 2 pixel ranges
per edge, interleaved rounds in one process; outputs must be bitwise equal
between rings at the same split.
Run with DROID_HIP_LIB=droid-slam_amd/lib/ab/libdroid_hip.so."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "droid-slam_amd"))
import droid_backends  # noqa: E402
from droid_backends._lib import lib  # noqa: E402

lib.droid_glo_set_ring.argtypes = [ctypes.c_int]
lib.droid_glo_set_ring.restype = ctypes.c_int
dev = torch.device("cuda:0")
E, HW = 2048, 48 * 64
g = torch.Generator(device=dev).manual_seed(23)
h = torch.tanh(torch.randn((E, HW, 128), generator=g, device=dev)).half()
w = (torch.randn((128, 128), generator=g, device=dev) / 11.3).half()
b = torch.randn(128, generator=g, device=dev) * 0.1
P = lambda t: ctypes.c_void_p(t.data_ptr())
cfgs = [(5, 1), (3, 1), (2, 1), (5, 2), (3, 2), (2, 2)]
outs = {c: torch.empty((c[1], E, 128), dtype=torch.float32, device=dev) for c in cfgs}
stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def run(c):
    lib.droid_glo_set_ring(c[0])
    assert lib.droid_gru_global_split_f16(P(h), P(w), P(b), P(outs[c]), c[1], E, HW, stream) == 0


for c in cfgs:
    run(c)
torch.cuda.synchronize()
print("rings 3, 2 == ring 5 bitwise: splits 1 %s, splits 2 %s" % (
    torch.equal(outs[(5, 1)], outs[(3, 1)]) and torch.equal(outs[(5, 1)], outs[(2, 1)]),
    torch.equal(outs[(5, 2)], outs[(3, 2)]) and torch.equal(outs[(5, 2)], outs[(2, 2)])))
ts = {c: [] for c in cfgs}
for r in range(10):
    for c in (cfgs if r % 2 == 0 else cfgs[::-1]):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(5):
            run(c)
        e.record()
        torch.cuda.synchronize()
        ts[c].append(s.elapsed_time(e) / 5)
for c in cfgs:
    t = sorted(ts[c])
    print("ring %d, splits %d: median %.3f ms (min %.3f), %.0f GB/s of h" % (c[0], c[1], t[len(t) // 2], t[0],
                                                                         h.numel() * 2 / t[len(t) // 2] / 1e6))
lib.droid_glo_set_ring(5)
