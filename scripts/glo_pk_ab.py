"""A/B of gru_glo_kernel's sigmoid sum on packed fp32 (A/B build:
droid_glo_set_pk) at the C3 shape (2048 edges of 48x64 x 128 channels), ring 3,
one pixel range per edge: scalar (the product until this A/B) vs packed (the
product after it), interleaved rounds in one process; the two differ by fp32
rounding only (the exp argument as one fma).  Result: profiles/r05/r05pk_glo_pk_ab.txt.
Run with DROID_HIP_LIB=droid-slam_amd/lib/ab/libdroid_hip.so."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "droid-slam_amd"))
import droid_backends  # noqa: E402,F401
from droid_backends._lib import lib  # noqa: E402

lib.droid_glo_set_pk.argtypes = [ctypes.c_int]
lib.droid_glo_set_pk.restype = ctypes.c_int
dev = torch.device("cuda:0")
E, HW = 2048, 48 * 64
g = torch.Generator(device=dev).manual_seed(23)
h = torch.tanh(torch.randn((E, HW, 128), generator=g, device=dev)).half()
w = (torch.randn((128, 128), generator=g, device=dev) / 11.3).half()
b = torch.randn(128, generator=g, device=dev) * 0.1
P = lambda t: ctypes.c_void_p(t.data_ptr())
outs = {v: torch.empty((E, 128), dtype=torch.float32, device=dev) for v in (0, 1)}
stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def run(v):
    lib.droid_glo_set_pk(v)
    assert lib.droid_gru_global_f16(P(h), P(w), P(b), P(outs[v]), E, HW, stream) == 0


for v in (0, 1):
    run(v)
torch.cuda.synchronize()
hf = h.float()
ref = (torch.sigmoid(hf @ w.float().t() + b) * hf).mean(1)
for v in (0, 1):
    print("pk %d: max |glo - torch fp32| %.3e" % (v, float((outs[v] - ref).abs().max())))
print("max |pk - scalar| %.3e" % float((outs[1] - outs[0]).abs().max()))
ts = {0: [], 1: []}
for r in range(12):
    for v in ((0, 1) if r % 2 == 0 else (1, 0)):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(5):
            run(v)
        e.record()
        torch.cuda.synchronize()
        ts[v].append(s.elapsed_time(e) / 5)
for v in (0, 1):
    t = sorted(ts[v])
    print("pk %d: median %.4f ms (min %.4f)" % (v, t[len(t) // 2], t[0]))
lib.droid_glo_set_pk(1)
