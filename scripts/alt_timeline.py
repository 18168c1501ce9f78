"""Per-stage timeline of corr_alt_ce0_kernel (profiling build: make -C
droid-slam_amd/csrc prof) on the C3 bench's coordinates (the reprojection of
the synthetic 256-KF trajectory along its 2048 edges): median shader clocks of
each phase, fast (whole-tile box prefetched) vs slow (split) stages.

usage: python scripts/alt_timeline.py"""
import os
import sys

_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "droid-slam_amd", "lib", "prof", "libdroid_hip.so")
os.environ.setdefault("DROID_HIP_LIB", _LIB)
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."),
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "droid-slam_amd")]
import ctypes  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

import droid_backends  # noqa: E402
from droid_backends._lib import lib  # noqa: E402
from droid_mi355x import synthetic  # noqa: E402
from droid_mi355x.corr import AltCorrBlock  # noqa: E402
from oracle import geometry as og  # noqa: E402

H, W, n = 48, 64, 256
rng = np.random.default_rng(1003)
ii, jj = synthetic.c3_edges(256, 2048, rng=np.random.default_rng(1003))
gt = synthetic.trajectory(n, rng)
poses, disps = synthetic.perturb(gt, synthetic.smooth_disps(n, H, W, rng), rng)
coords, _ = og.projective_transform(poses, disps, np.tile(synthetic.INTRINSICS, (n, 1)), ii, jj)
dev = torch.device("cuda:0")
fm = torch.randn((1, n, 128, H, W), device=dev).half()
pyr = [lv.view((-1,) + tuple(lv.shape[2:])) for lv in AltCorrBlock(fm).pyramid]
c = torch.from_numpy(coords.astype(np.float32)).to(dev).contiguous()
w = (torch.randn((128, 224), device=dev) / 14).half()
w[:, 196:] = 0
b = torch.zeros(128, device=dev)
f1 = torch.as_tensor(ii, dtype=torch.int32, device=dev)
f2 = torch.as_tensor(jj, dtype=torch.int32, device=dev)
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
d = np.diff(st[..., :7], axis=-1)
lvl = 3 - np.arange(1, 32) % 4
for l in range(4):
    for kind, m in (("fast", ~slow), ("slow", slow)):
        sel = m & (lvl[None, :] == l)
        if sel.sum() == 0:
            continue
        print("level %d %s (%5d stages, taps %5.1f): " % (l, kind, sel.sum(), taps[sel].mean())
              + ", ".join("%s %6.0f" % (nm, np.median(d[..., k][sel])) for k, nm in enumerate(names))
              + "  total %6.0f" % np.median(d.sum(-1)[sel]))
