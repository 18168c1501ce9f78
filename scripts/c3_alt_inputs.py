"""The C3 bench graph's on-demand lookup inputs (scripts only): the synthetic
256-KF trajectory, its 2048 edges, the reprojected coordinates (device
projective_transform), a feature pyramid of random frames and random
corr_encoder[0] weights - what corr_alt_ce0 sees in bench.py --lowmem."""
import numpy as np
import torch

import droid_backends
from droid_mi355x import synthetic
from droid_mi355x.corr import AltCorrBlock


def c3_alt_inputs(dev, H=48, W=64, n=256, E=2048):
    rng = np.random.default_rng(1003)
    ii, jj = synthetic.c3_edges(n, E, rng=np.random.default_rng(1003))
    gt = synthetic.trajectory(n, rng)
    poses, disps = synthetic.perturb(gt, synthetic.smooth_disps(n, H, W, rng), rng)
    f32 = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(dev)
    coords = droid_backends.projective_transform(
        f32(poses), f32(disps), f32(np.tile(synthetic.INTRINSICS, (n, 1))), torch.as_tensor(ii, device=dev),
        torch.as_tensor(jj, device=dev), with_valid=False)[0]
    fm = torch.randn((1, n, 128, H, W), device=dev).half()
    pyr = [lv.view((-1,) + tuple(lv.shape[2:])) for lv in AltCorrBlock(fm).pyramid]
    w = (torch.randn((128, 224), device=dev) / 14).half()
    w[:, 196:] = 0
    b = torch.zeros(128, device=dev)
    f1 = torch.as_tensor(ii, dtype=torch.int32, device=dev)
    f2 = torch.as_tensor(jj, dtype=torch.int32, device=dev)
    return pyr, f1, f2, coords.contiguous(), w, b
