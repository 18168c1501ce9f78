"""Where does corr_alt_ce0 disagree with the volume path?  Per-tile error map
(tile index = e * (H/8)(W/8) + row * W/8 + col) at 48x64."""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."),
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "droid-slam_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import droid_backends  # noqa: E402
from droid_mi355x.corr import AltCorrBlock, CorrBlock  # noqa: E402

dev = "cuda:0"
for E, noise in ((4, 1.5), (40, 1.5), (300, 1.5), (300, 0.0)):
    rng = np.random.default_rng(31)
    NF, H, W = 12, 48, 64
    fm = torch.from_numpy(rng.normal(size=(NF, 128, H, W)).astype(np.float16)).to(dev)
    ii = rng.integers(0, NF, E).astype(np.int64)
    jj = rng.integers(0, NF, E).astype(np.int64)
    with torch.no_grad():
        cb = CorrBlock(fm[ii][None], fm[jj][None])
    cbt = CorrBlock(fm[ii][None], fm[jj][None])        # grad mode on: torch GEMM + avg_pool2d path
    for lv in range(4):
        d = (cb.corr_pyramid[lv].float() - cbt.corr_pyramid[lv].float()).abs()
        per_edge = d.reshape(E, -1).amax(1).cpu().numpy()
        badv = np.nonzero(per_edge > 0.05)[0]
        print("  level %d kernel vs torch volume: max %.4f, bad edges %d %s" % (lv, per_edge.max(), len(badv), badv[:10]))
    pyr = [lv.view((-1,) + tuple(lv.shape[2:])) for lv in AltCorrBlock(fm[None]).pyramid]
    grid = np.stack(np.meshgrid(np.arange(W), np.arange(H)), -1)[None].astype(np.float32)
    coords = grid + rng.normal(0, noise, (E, H, W, 2)).astype(np.float32) + 2.0
    c = torch.from_numpy(coords).to(dev).contiguous()
    g = torch.Generator(device=dev).manual_seed(32)
    w224 = torch.zeros((128, 224), device=dev)
    w224[:, :196] = torch.randn((128, 196), generator=g, device=dev) / 14.0
    w224 = w224.half().contiguous()
    b = torch.randn(128, generator=g, device=dev) * 0.1
    with torch.no_grad():
        ref = droid_backends.corr_lookup_ce0(cb.corr_pyramid, c, w224, b).float()
        out = droid_backends.corr_alt_ce0(pyr, torch.as_tensor(ii, dtype=torch.int32, device=dev),
                                          torch.as_tensor(jj, dtype=torch.int32, device=dev), c, w224, b).float()
        # third opinion: grid_sample lookup of the torch volume, fp32 1x1 conv
        d = torch.arange(-3, 4, dtype=torch.float32, device=dev)
        outs = []
        for lvl, vol in enumerate(cbt.corr_pyramid):
            H2, W2 = vol.shape[-2:]
            cc = c.reshape(E * H * W, 1, 1, 2) / 2 ** lvl
            gx = (cc[..., 0] + d.view(1, 7, 1)).expand(E * H * W, 7, 7)
            gy = (cc[..., 1] + d.view(1, 1, 7)).expand(E * H * W, 7, 7)
            grid = torch.stack([2 * gx / (W2 - 1) - 1, 2 * gy / (H2 - 1) - 1], -1)
            smp = torch.nn.functional.grid_sample(vol.float().reshape(E * H * W, 1, H2, W2), grid, align_corners=True)
            outs.append(smp.view(E, H, W, 49))
        lk = torch.cat(outs, -1)
        ref3 = torch.relu(lk @ w224[:, :196].float().t() + b)
    scale = float(ref3.abs().max())
    for name, x in (("alt-vs-vol", out - ref), ("alt-vs-torch", out - ref3), ("vol-vs-torch", ref - ref3)):
        err = x.abs().amax(-1).cpu().numpy()              # (E,H,W)
        terr = err.reshape(E, H // 8, 8, W // 8, 8).max(axis=(2, 4)).reshape(-1) / scale
        bad = np.nonzero(terr > 0.02)[0]
        print("E=%d noise=%.1f %s tiles=%d bad=%d first bad tiles %s max %.3f" % (
            E, noise, name, len(terr), len(bad), bad[:20], terr.max()), flush=True)
