"""Per-tile phase timeline of corr_alt2_kernel (profiling build: make -C
droid-slam_amd/csrc prof) on the C3 bench's coordinates: median shader clocks
of each phase over the first 8 tiles of every workgroup (tile 0 skipped),
wave 0's view.

usage: python scripts/alt2_timeline.py [workgroups per CU: 1 | 2]"""
import os
import sys

_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "droid-slam_amd", "lib", "prof", "libdroid_hip.so")
os.environ.setdefault("DROID_HIP_LIB", _LIB)
if len(sys.argv) > 1:
    os.environ["DROID_ALT2_WG_PER_CU"] = sys.argv[1]
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
G = 2 * 256
prof = torch.zeros((G, 8, 16), dtype=torch.int64, device=dev)
lib.droid_alt_set_profile.argtypes = [ctypes.c_void_p]
droid_backends.alt_set_variant(2)
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
p = prof.cpu().numpy()[:, 1:7, :].reshape(-1, 16)
ok = (p[:, 0] > 0) & (p[:, 15] > 0) & (p[:, 1] > 0) & (p[:, 8] > 0)
p = p[ok]
names = ["A dma issue", "A wait+bar", "A C", "A bar", "A bilinear", "A bar", "A encoder+bar", "B dma issue",
         "B wait+bar", "B C", "B bilinear+bar", "B encoder+bar", "out staging+bar", "stores", "final bar"]
d = np.diff(p, axis=1)
print("tiles %d, total median %.0f clk" % (len(p), np.median(p[:, 15] - p[:, 0])))
for k, nm in enumerate(names):
    print("  %-18s median %6.0f  p90 %6.0f" % (nm, np.median(d[:, k]), np.percentile(d[:, k], 90)))
