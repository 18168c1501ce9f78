"""Correlation restatements (numpy).

corr_volume / corr_pyramid : modules/corr.py:24-38, 63-71 (CorrBlock.__init__, .corr)
corr_index_forward         : src/correlation_kernels.cu:19-70, 126-155
corr_index_backward        : src/correlation_kernels.cu:73-124, 157-185
alt_pyramid                : modules/corr.py:92-104 (AltCorrBlock.__init__)
altcorr_forward            : src/altcorr_kernel.cu:27-149, 290-319 (race-free semantics)
altcorr_backward           : src/altcorr_kernel.cu:152-286, 321-356

The fp16 lookup emulates the reference's at::Half arithmetic exactly: each
bilinear weight is rounded to half, each product s*w is rounded to half, and
each `+=` rounds the running sum to half, in the kernel's loop order
(i = x-offset outer, j = y-offset inner).  The fp32/fp64 lookups use the
fused multiply-add nvcc emits for `corr += s * w`.
"""
import numpy as np


def avg_pool2(x):
    """F.avg_pool2d(x, 2, stride=2) over the last two axes (floor sizes)."""
    H2, W2 = x.shape[-2] // 2, x.shape[-1] // 2
    x = x[..., :2 * H2, :2 * W2]
    return 0.25 * (x[..., 0::2, 0::2] + x[..., 0::2, 1::2] + x[..., 1::2, 0::2] + x[..., 1::2, 1::2])


def corr_volume(fmap1, fmap2):
    """CorrBlock.corr (corr.py:63-71): fmap (B,N,C,H,W) -> (B*N, H, W, H, W) of <f1/4, f2/4>."""
    B, N, C, H, W = fmap1.shape
    f1 = fmap1.reshape(B * N, C, H * W) / 4.0
    f2 = fmap2.reshape(B * N, C, H * W) / 4.0
    return np.matmul(f1.transpose(0, 2, 1), f2).reshape(B * N, H, W, H, W)


def corr_pyramid(fmap1, fmap2, num_levels=4):
    """CorrBlock.__init__ (corr.py:24-38)."""
    vol = corr_volume(fmap1, fmap2)
    out = [vol]
    for _ in range(num_levels - 1):
        vol = avg_pool2(vol)
        out.append(vol)
    return out


def _taps(volume, coords, r):
    """Integer tap positions and the validity mask shared by fwd/bwd."""
    B, H, W, H2, W2 = volume.shape
    x0 = coords[:, 0].astype(np.float32)
    y0 = coords[:, 1].astype(np.float32)
    fx0 = np.floor(x0)
    fy0 = np.floor(y0)
    dx = (x0 - fx0).astype(np.float32)
    dy = (y0 - fy0).astype(np.float32)
    return fx0.astype(np.int64), fy0.astype(np.int64), dx, dy


def corr_index_forward(volume, coords, r):
    """corr_index_forward_kernel: volume (B,H,W,H2,W2), coords (B,2,H,W) ->
    corr (B, 2r+1, 2r+1, H, W) with corr[:, i, j] the bilinear sample at
    (x0 - r + i, y0 - r + j), zero padding (i is the x offset)."""
    B, H, W, H2, W2 = volume.shape
    rd = 2 * r + 1
    dt = volume.dtype
    xi0, yi0, dx, dy = _taps(volume, coords, r)
    one = np.float32(1.0)
    w_tab = {(1, 1): dx * dy, (1, 0): dx * (one - dy), (0, 1): (one - dx) * dy, (0, 0): (one - dx) * (one - dy)}
    bb, hh, ww = np.meshgrid(np.arange(B), np.arange(H), np.arange(W), indexing="ij")
    acc = np.zeros((B, rd, rd, H, W), dtype=dt)
    for i in range(rd + 1):
        for j in range(rd + 1):
            x1 = xi0 - r + i
            y1 = yi0 - r + j
            inb = (x1 >= 0) & (x1 < W2) & (y1 >= 0) & (y1 < H2)
            s = volume[bb, hh, ww, np.clip(y1, 0, H2 - 1), np.clip(x1, 0, W2 - 1)]
            # target (i-di, j-dj) gets weight w_tab[(di, dj)]; reference order :55-65
            for (di, dj) in ((1, 1), (1, 0), (0, 1), (0, 0)):
                a, b = i - di, j - dj
                if not (0 <= a < rd and 0 <= b < rd):
                    continue
                w = w_tab[(di, dj)]
                cur = acc[:, a, b]
                if dt == np.float16:
                    p = (s.astype(np.float32) * w.astype(np.float16).astype(np.float32)).astype(np.float16)
                    new = (cur.astype(np.float32) + p.astype(np.float32)).astype(np.float16)
                else:
                    new = (cur.astype(np.float64) + s.astype(np.float64) * w.astype(dt).astype(np.float64)).astype(dt)
                acc[:, a, b] = np.where(inb, new, cur)
    return acc


def corr_index_backward(volume, coords, corr_grad, r):
    """corr_index_backward_kernel: scatter bilinear-weighted grads into the volume."""
    B, H, W, H2, W2 = volume.shape
    rd = 2 * r + 1
    xi0, yi0, dx, dy = _taps(volume, coords, r)
    g = corr_grad.astype(np.float64)
    out = np.zeros(volume.shape, dtype=np.float64)
    bb, hh, ww = np.meshgrid(np.arange(B), np.arange(H), np.arange(W), indexing="ij")
    for i in range(rd + 1):
        for j in range(rd + 1):
            x1 = xi0 - r + i
            y1 = yi0 - r + j
            inb = (x1 >= 0) & (x1 < W2) & (y1 >= 0) & (y1 < H2)
            acc = np.zeros((B, H, W))
            if i > 0 and j > 0:
                acc += g[:, i - 1, j - 1] * dx * dy
            if i > 0 and j < rd:
                acc += g[:, i - 1, j] * dx * (1 - dy)
            if i < rd and j > 0:
                acc += g[:, i, j - 1] * (1 - dx) * dy
            if i < rd and j < rd:
                acc += g[:, i, j] * (1 - dx) * (1 - dy)
            np.add.at(out, (bb[inb], hh[inb], ww[inb], y1[inb], x1[inb]), acc[inb])
    return out.astype(volume.dtype)


def lookup_pyramid(pyramid, coords, r=3):
    """CorrBlock.__call__ (corr.py:40-50): coords (B,N,H,W,2) -> (B,N,4*(2r+1)^2,H,W)."""
    B, N, H, W, _ = coords.shape
    c = coords.transpose(0, 1, 4, 2, 3).reshape(B * N, 2, H, W).astype(np.float32)
    outs = []
    for i, vol in enumerate(pyramid):
        corr = corr_index_forward(vol, c / np.float32(2 ** i), r)
        outs.append(corr.reshape(B, N, -1, H, W))
    return np.concatenate(outs, axis=2)


def alt_pyramid(fmaps, num_levels=4):
    """AltCorrBlock.__init__ (corr.py:92-104): (B,N,C,H,W) -> list of (B,N,H_i,W_i,C)."""
    B, N, C, H, W = fmaps.shape
    f = fmaps.reshape(B * N, C, H, W) / 4.0
    out = []
    for i in range(num_levels):
        out.append(f.transpose(0, 2, 3, 1).reshape(B, N, H // 2 ** i, W // 2 ** i, C))
        f = avg_pool2(f)
    return out


def altcorr_forward(fmap1, fmap2, coords, r):
    """altcorr_forward_kernel semantics: fmap1 (B,H,W,C), fmap2 (B,H2,W2,C),
    coords (B,S,H,W,2) -> corr (B,S,(2r+1)^2,H,W); channel 7*ix + iy."""
    B, H, W, C = fmap1.shape
    _, H2, W2, _ = fmap2.shape
    S = coords.shape[1]
    rd = 2 * r + 1
    f1 = fmap1.astype(np.float64)
    f2 = fmap2.astype(np.float64)
    out = np.zeros((B, S, rd * rd, H, W))
    for b in range(B):
        for s in range(S):
            x = coords[b, s, ..., 0].astype(np.float32)
            y = coords[b, s, ..., 1].astype(np.float32)
            fx0 = np.floor(x)
            fy0 = np.floor(y)
            dx = (x - fx0).astype(np.float64)
            dy = (y - fy0).astype(np.float64)
            xi0 = fx0.astype(np.int64)
            yi0 = fy0.astype(np.int64)
            for iy in range(rd + 1):
                for ix in range(rd + 1):
                    h2 = yi0 - r + iy
                    w2 = xi0 - r + ix
                    inb = (h2 >= 0) & (h2 < H2) & (w2 >= 0) & (w2 < W2)
                    g = f2[b, np.clip(h2, 0, H2 - 1), np.clip(w2, 0, W2 - 1)]
                    sv = np.where(inb, np.einsum("hwc,hwc->hw", f1[b], g), 0.0)
                    if iy > 0 and ix > 0:
                        out[b, s, (iy - 1) + rd * (ix - 1)] += sv * dy * dx
                    if iy > 0 and ix < rd:
                        out[b, s, (iy - 1) + rd * ix] += sv * dy * (1 - dx)
                    if iy < rd and ix > 0:
                        out[b, s, iy + rd * (ix - 1)] += sv * (1 - dy) * dx
                    if iy < rd and ix < rd:
                        out[b, s, iy + rd * ix] += sv * (1 - dy) * (1 - dx)
    return out


def altcorr_backward(fmap1, fmap2, coords, corr_grad, r):
    """altcorr_backward semantics: grads of sum(corr * corr_grad) w.r.t. fmap1,
    fmap2; coords_grad is returned all-zero (altcorr_kernel.cu:321-356)."""
    B, H, W, C = fmap1.shape
    _, H2, W2, _ = fmap2.shape
    S = coords.shape[1]
    rd = 2 * r + 1
    f1 = fmap1.astype(np.float64)
    f2 = fmap2.astype(np.float64)
    g1 = np.zeros_like(f1)
    g2 = np.zeros_like(f2)
    G = corr_grad.astype(np.float64)
    for b in range(B):
        for s in range(S):
            x = coords[b, s, ..., 0].astype(np.float32)
            y = coords[b, s, ..., 1].astype(np.float32)
            fx0 = np.floor(x)
            fy0 = np.floor(y)
            dx = (x - fx0).astype(np.float64)
            dy = (y - fy0).astype(np.float64)
            xi0 = fx0.astype(np.int64)
            yi0 = fy0.astype(np.int64)
            for iy in range(rd + 1):
                for ix in range(rd + 1):
                    h2 = yi0 - r + iy
                    w2 = xi0 - r + ix
                    inb = (h2 >= 0) & (h2 < H2) & (w2 >= 0) & (w2 < W2)
                    g = np.zeros((H, W))
                    if iy > 0 and ix > 0:
                        g += G[b, s, (iy - 1) + rd * (ix - 1)] * dy * dx
                    if iy > 0 and ix < rd:
                        g += G[b, s, (iy - 1) + rd * ix] * dy * (1 - dx)
                    if iy < rd and ix > 0:
                        g += G[b, s, iy + rd * (ix - 1)] * (1 - dy) * dx
                    if iy < rd and ix < rd:
                        g += G[b, s, iy + rd * ix] * (1 - dy) * (1 - dx)
                    g = np.where(inb, g, 0.0)
                    hc = np.clip(h2, 0, H2 - 1)
                    wc = np.clip(w2, 0, W2 - 1)
                    g1[b] += g[..., None] * f2[b, hc, wc]
                    np.add.at(g2[b], (hc[inb], wc[inb]), (g[..., None] * f1[b])[inb])
    return g1, g2, np.zeros(coords.shape)


# --- torch CPU formulation (the "pure-PyTorch CPU path" of the baseline) ------
def corr_pyramid_torch(fmap1, fmap2, num_levels=4):
    """CorrBlock.__init__ (corr.py:24-38) in torch fp32: (B,N,C,H,W) float
    tensors -> list of (B*N, H, W, H_l, W_l) levels (matmul + avg_pool2d)."""
    import torch
    import torch.nn.functional as F
    B, N, C, H, W = fmap1.shape
    f1 = fmap1.reshape(B * N, C, H * W) / 4.0
    f2 = fmap2.reshape(B * N, C, H * W) / 4.0
    vol = torch.matmul(f1.transpose(1, 2), f2).reshape(B * N * H * W, 1, H, W)
    out = [vol.view(B * N, H, W, H, W)]
    for _ in range(num_levels - 1):
        vol = F.avg_pool2d(vol, 2, stride=2)
        out.append(vol.view(B * N, H, W, vol.shape[-2], vol.shape[-1]))
    return out


def lookup_pyramid_torch(pyramid, coords, r=3):
    """CorrBlock.__call__ (corr.py:40-50) as F.grid_sample(align_corners=True,
    zero padding) at (x0 - r + i, y0 - r + j) - the same bilinear sample as
    corr_index_forward (checked in tests/test_oracle_golden.py).  pyramid:
    corr_pyramid_torch levels; coords (B,H,W,2) -> (B, L*(2r+1)^2, H, W)."""
    import torch
    import torch.nn.functional as F
    B, H, W, _ = coords.shape
    rd = 2 * r + 1
    d = torch.arange(-r, r + 1, dtype=coords.dtype, device=coords.device)
    outs = []
    for lvl, vol in enumerate(pyramid):
        H2, W2 = vol.shape[-2:]
        assert H2 > 1 and W2 > 1, "grid_sample's align_corners mapping needs levels of >= 2 pixels a side"
        c = coords.reshape(B * H * W, 1, 1, 2) / 2 ** lvl
        gx = (c[..., 0] + d.view(1, rd, 1)).expand(B * H * W, rd, rd)   # [:, i, j]: x offset i
        gy = (c[..., 1] + d.view(1, 1, rd)).expand(B * H * W, rd, rd)   #            y offset j
        grid = torch.stack([2 * gx / (W2 - 1) - 1, 2 * gy / (H2 - 1) - 1], -1)
        # grid_sample indexes (N, C, H_out, W_out) with grid[..., (x, y)]: out[:, 0, i, j] samples (gx_i, gy_j)
        s = F.grid_sample(vol.reshape(B * H * W, 1, H2, W2), grid, align_corners=True, padding_mode="zeros")
        outs.append(s.view(B, H, W, rd * rd).permute(0, 3, 1, 2))
    return torch.cat(outs, 1)
