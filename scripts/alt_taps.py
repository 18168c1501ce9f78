import os, sys
sys.path[:0] = ["scripts", ".", "droid-slam_amd"]
os.environ.setdefault("DROID_HIP_LIB", "droid-slam_amd/lib/prof/libdroid_hip.so")
import ctypes, numpy as np, torch
import droid_backends
from droid_backends._lib import lib
from c3_alt_inputs import c3_alt_inputs
dev = torch.device("cuda:0")
pyr, f1, f2, c, w, b = c3_alt_inputs(dev)
G = 256
# 32 stages per workgroup are recorded: tiles 0..7 of each workgroup
prof = torch.zeros((G, 32, 8), dtype=torch.int64, device=dev)
lib.droid_alt_set_profile.argtypes = [ctypes.c_void_p]
droid_backends.corr_alt_ce0(pyr, f1, f2, c, w, b)
assert lib.droid_alt_set_profile(ctypes.c_void_p(prof.data_ptr())) == 0
droid_backends.corr_alt_ce0(pyr, f1, f2, c, w, b)
torch.cuda.synchronize()
lib.droid_alt_set_profile(ctypes.c_void_p(0))
taps = (prof[..., 7].cpu().numpy() >> 1).reshape(G, 8, 4)   # stage st -> level 3 - st
l3, l2, l1, l0 = taps[..., 0], taps[..., 1], taps[..., 2], taps[..., 3]
s321 = l3 + l2 + l1
for name, v in (("l0", l0), ("l1", l1), ("l2", l2), ("l3", l3), ("l3+l2+l1", s321), ("l3+l2", l3 + l2)):
    v = v.ravel()
    print("%-9s median %5.0f p75 %5.0f p90 %5.0f p95 %5.0f p99 %5.0f max %5d" % (name, *np.percentile(v, [50, 75, 90, 95, 99]), v.max()))
for cap in (192, 208, 224, 240, 256, 288):
    print("cap %d: l0 over %.1f%%, l3+l2+l1 over %.1f%%, l1 over %.1f%%" % (cap, 100 * (l0 > cap).mean(), 100 * (s321 > cap).mean(), 100 * (l1 > cap).mean()))
