"""Per-stage timeline of corr_alt_ce0_kernel (profiling build: make -C
droid-slam_amd/csrc prof) on the C3 bench's coordinates (the reprojection of
the synthetic 256-KF trajectory along its 2048 edges): median shader clocks of
each phase, fast (whole-tile box prefetched) vs slow (split) stages.

usage: python scripts/alt_timeline.py"""
import os
import sys

_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "droid-slam_amd", "lib", "prof", "libdroid_hip.so")
os.environ.setdefault("DROID_HIP_LIB", _LIB)
sys.path[:0] = [os.path.dirname(os.path.abspath(__file__)), os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."),
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "droid-slam_amd")]
import ctypes  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

import droid_backends  # noqa: E402
from droid_backends._lib import lib  # noqa: E402
from c3_alt_inputs import c3_alt_inputs  # noqa: E402

dev = torch.device("cuda:0")
pyr, f1, f2, c, w, b = c3_alt_inputs(dev)
G = 256
prof = torch.zeros((G, 32, 8), dtype=torch.int64, device=dev)
lib.droid_alt_set_profile.argtypes = [ctypes.c_void_p]
for it in range(3):
    if it == 2:
        assert lib.droid_alt_set_profile(ctypes.c_void_p(prof.data_ptr())) == 0
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    droid_backends.corr_alt_ce0(pyr, f1, f2, c, w, b)
    e.record()
    torch.cuda.synchronize()
    print("launch %.3f ms" % s.elapsed_time(e))
lib.droid_alt_set_profile(ctypes.c_void_p(0))
p = prof.cpu().numpy()
st = p[:, 1:, :]                      # skip each workgroup's first stage (prologue)
slow = (st[..., 7] & 1) == 1
taps = st[..., 7] >> 1
names = ["box wait + B1", "C (MFMA)", "B2", "bilinear", "B3", "encoder/epilogue"]
order = [0, 1, 2, 3, 4, 5, 6]
if os.environ.get("ALT_CSTAMP") == "1":   # a DROID_ALT_CSTAMP=1 build: stamps 3/4/5 split the C phase
    names = ["box wait + B1", "next-box DMA issue", "box MFMA", "pixel boxes", "C rest", "bilinear..end"]
    order = [0, 1, 3, 4, 5, 2, 6]
d = np.diff(st[..., order], axis=-1)
lvl = 3 - np.arange(1, 32) % 4
for l in range(4):
    for kind, m in (("fast", ~slow), ("slow", slow)):
        sel = m & (lvl[None, :] == l)
        if sel.sum() == 0:
            continue
        print("level %d %s (%5d stages, taps %5.1f): " % (l, kind, sel.sum(), taps[sel].mean())
              + ", ".join("%s %6.0f" % (nm, np.median(d[..., k][sel])) for k, nm in enumerate(names))
              + "  total %6.0f" % np.median(d.sum(-1)[sel]))
