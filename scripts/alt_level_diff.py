"""Debug aid: the product corr_alt2_kernel (variant 2) vs the A/B row-K kernel
(variant 5; both in the A/B library) per correlation level: corr_encoder[0]'s
weights zeroed outside one level's 49 channels, so a mismatch names the level
and the pixels it comes from."""
import os
import sys

_R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
os.environ["DROID_HIP_LIB"] = os.path.join(_R, "droid-slam_amd", "lib", "ab", "libdroid_hip.so")
sys.path[:0] = [os.path.join(_R, "droid-slam_amd"), _R]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import droid_backends  # noqa: E402
from droid_mi355x.corr import AltCorrBlock  # noqa: E402

DEV = torch.device("cuda:0")
for (noise, H, W, E) in ((1.5, 16, 24, 6), (1.5, 48, 64, 40)):
    rng = np.random.default_rng(43)
    NF = 8
    fm = torch.from_numpy(rng.normal(size=(NF, 128, H, W)).astype(np.float16)).to(DEV)
    ii = rng.integers(0, NF, E).astype(np.int32)
    jj = rng.integers(0, NF, E).astype(np.int32)
    pyr = [lv.view((-1,) + tuple(lv.shape[2:])) for lv in AltCorrBlock(fm[None]).pyramid]
    grid = np.stack(np.meshgrid(np.arange(W), np.arange(H)), -1)[None].astype(np.float32)
    coords = grid + rng.normal(0, noise, (E, H, W, 2)).astype(np.float32)
    c = torch.from_numpy(coords).to(DEV).contiguous()
    f1, f2 = torch.as_tensor(ii, device=DEV), torch.as_tensor(jj, device=DEV)
    g = torch.Generator(device=DEV).manual_seed(44)
    wfull = torch.randn((128, 196), generator=g, device=DEV) / 14.0
    b = torch.zeros(128, device=DEV)
    for lvl in range(4):
        w224 = torch.zeros((128, 224), device=DEV)
        w224[:, 49 * lvl:49 * lvl + 49] = wfull[:, 49 * lvl:49 * lvl + 49]
        w224 = w224.half().contiguous()
        outs = {}
        for v in (5, 2):
            droid_backends.alt_set_variant(v)
            outs[v] = droid_backends.corr_alt_ce0(pyr, f1, f2, c, w224, b).float()
        droid_backends.alt_set_variant(2)
        torch.cuda.synchronize()
        d = (outs[2] - outs[5]).abs().amax(-1)   # (E, H, W)
        bad = (d > 0).nonzero()
        print("HxW %dx%d level %d: max diff %.4g, %d of %d pixels differ%s" % (
            H, W, lvl, float(d.max()), bad.shape[0], d.numel(),
            "" if not bad.shape[0] else ", first (e, y, x): " + str(bad[:6].tolist())))
