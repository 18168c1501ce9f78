"""Correlation blocks (mirror of modules/corr.py) on the HIP kernels.

CorrBlock builds the reference's volume pyramid (corr.py:24-38, 63-71) with ONE
hand-written kernel (droid_corr_volume_pyramid: MFMA GEMM of the frames' NHWC
features, the three 2x2 pooling levels formed in registers, every level
written once, optionally straight into the 8x8-tiled layout of the fused
lookup); its lookup runs all 4 levels in ONE kernel launch and writes the
concatenated (B, N, 196, H, W) tensor directly (corr.py:40-50 does 4 launches
+ cat).  Under autograd the volume comes from torch's GEMM + avg_pool2d and
the lookup uses the per-level CorrSampler so the backward kernel runs
(training path).
"""
import numpy as np
import torch
import torch.nn.functional as F

import droid_backends


class CorrSampler(torch.autograd.Function):
    """corr.py:6-20."""

    @staticmethod
    def forward(ctx, volume, coords, radius):
        ctx.save_for_backward(volume, coords)
        ctx.radius = radius
        corr, = droid_backends.corr_index_forward(volume, coords, radius)
        return corr

    @staticmethod
    def backward(ctx, grad_output):
        volume, coords = ctx.saved_tensors
        grad_volume, = droid_backends.corr_index_backward(volume, coords, grad_output.contiguous(), ctx.radius)
        return grad_volume, None, None


def _avg_pool2(x, max_elems=1 << 30):
    """F.avg_pool2d(x, 2, stride=2) in batch chunks: the ROCm kernel indexes
    with 32 bits and a 2048-edge level-0 volume has 1.9e10 elements."""
    n = x.shape[0]
    per = max(1, max_elems // max(1, x[0].numel()))
    if n <= per:
        return F.avg_pool2d(x, 2, stride=2)
    out = torch.empty((n, x.shape[1], x.shape[2] // 2, x.shape[3] // 2), dtype=x.dtype, device=x.device)
    for s in range(0, n, per):
        out[s:s + per] = F.avg_pool2d(x[s:s + per], 2, stride=2)
    return out


def tile8(level, chunk=256):
    """(E,H,W,H2,W2) -> 8x8-tiled (E,H,W,ceil(H2/8),W2/8,8,8), rows past H2 zero
    (the layout of droid_corr_lookup_ce0_tiled), in edge chunks to bound the
    transient memory of the copy."""
    E, H, W, H2, W2 = level.shape
    H2p = (H2 + 7) // 8 * 8
    out = torch.zeros((E, H, W, H2p // 8, W2 // 8, 8, 8), dtype=level.dtype, device=level.device)
    for s in range(0, E, chunk):
        x = level[s:s + chunk]
        if H2p != H2:
            x = F.pad(x, (0, 0, 0, H2p - H2))
        n = x.shape[0]
        out[s:s + n] = x.reshape(n, H, W, H2p // 8, 8, W2 // 8, 8).permute(0, 1, 2, 3, 5, 4, 6)
    return out


def untile8(level, H2, W2):
    """inverse of tile8: (E,H,W,H2p/8,W2/8,8,8) -> (E,H,W,H2,W2)."""
    E, H, W = level.shape[:3]
    H2p = level.shape[3] * 8
    x = level.permute(0, 1, 2, 3, 5, 4, 6).reshape(E, H, W, H2p, W2)
    return x[:, :, :, :H2].contiguous()


def upload(arr, device):
    """host array -> device tensor without draining the stream: a copy from
    pageable host memory waits for the stream's queued work first (the frontend's
    edge edits would stall the host on the previous update); this one is staged in
    pinned memory and copied asynchronously."""
    t = torch.from_numpy(np.ascontiguousarray(arr))
    if torch.device(device).type == "cuda":
        if torch.cuda.is_current_stream_capturing():
            # a captured copy would re-read this staging buffer at every replay,
            # after the host allocator has recycled it (FactorGraph._update_graphed)
            raise RuntimeError("upload() inside a HIP graph capture")
        t = t.pin_memory()
    return t.to(device, non_blocking=True)


class CorrBlock:
    """corr.py:23-71 (volume correlation pyramid).

    tiled=True (FactorGraph with the fused operator): the levels are stored in
    8x8 tiles (tile8) for droid_corr_lookup_ce0_tiled - same values, a layout
    whose lookup windows touch fewer DRAM lines; the reference layout is
    rebuilt on demand for the other lookups (reference_pyramid)."""

    def __init__(self, fmap1, fmap2, num_levels=4, radius=3, tiled=False, _levels=None):
        self.num_levels = num_levels
        self.radius = radius
        self.corr_pyramid = []   # (resets the slot pool state)
        if _levels is not None:                      # from_frames
            self.corr_pyramid, self.level_shapes, self.tiled = _levels
            return
        batch, num, dim, ht, wd = fmap1.shape
        self.level_shapes = [(ht // 2 ** i, wd // 2 ** i) for i in range(num_levels)]
        t = bool(tiled) and all(w % 8 == 0 for _, w in self.level_shapes)
        if (num_levels == 4 and dim == 128 and fmap1.is_cuda and not torch.is_grad_enabled()
                and droid_backends.corr_volume_pyramid_supported(ht, wd, t)):
            # the fused kernel: the edges' feature maps as 2E frames (NHWC / 4)
            E = batch * num
            f = torch.cat([fmap1.reshape(E, dim, ht, wd), fmap2.reshape(E, dim, ht, wd)], 0)
            f = (f.half() / 4.0).permute(0, 2, 3, 1).contiguous()
            idx = torch.arange(E, dtype=torch.int32, device=f.device)
            self.corr_pyramid = droid_backends.corr_volume_pyramid(f, idx, idx + E, t)
            self.tiled = t
            return
        vol = CorrBlock.corr(fmap1, fmap2)
        batch, num, h1, w1, h2, w2 = vol.shape
        self.level_shapes = [(h2 // 2 ** i, w2 // 2 ** i) for i in range(num_levels)]
        self.tiled = bool(tiled) and all(w % 8 == 0 for _, w in self.level_shapes)
        vol = vol.reshape(batch * num * h1 * w1, 1, h2, w2)
        for i in range(num_levels):
            lv = vol.view(batch * num, h1, w1, h2 // 2 ** i, w2 // 2 ** i)
            if i + 1 < num_levels:
                vol = _avg_pool2(vol)
            self.corr_pyramid.append(tile8(lv) if self.tiled else lv)
            del lv

    @classmethod
    def from_frames(cls, fmaps, f1, f2, tiled=False, num_levels=4, radius=3):
        """The pyramid of the edges (f1[e] -> f2[e]) straight from the frames'
        features: fmaps (NF,H,W,128) fp16 = fmap / 4 in NHWC (AltCorrBlock level
        0), f1 / f2 (E) int32 rows - no per-edge feature copies."""
        NF, H, W, _ = fmaps.shape
        shapes = [(H // 2 ** i, W // 2 ** i) for i in range(num_levels)]
        t = bool(tiled) and all(w % 8 == 0 for _, w in shapes)
        levels = droid_backends.corr_volume_pyramid(fmaps, f1, f2, t)
        return cls(None, None, num_levels, radius, _levels=(levels, shapes, t))

    def reference_pyramid(self):
        """the levels in the reference layout (E,H,W,H2,W2)."""
        if not self.tiled:
            return self.corr_pyramid
        return [untile8(lv, h2, w2) for lv, (h2, w2) in zip(self.corr_pyramid, self.level_shapes)]

    def __call__(self, coords):
        batch, num, ht, wd, _ = coords.shape
        if (self.tiled and self.radius == 3 and not torch.is_grad_enabled()
                and self._pyr[0].dtype == torch.float16):
            # the tiled slot pool read in place (no untile / gather copy), NCHW out
            c = coords.reshape(batch * num, ht, wd, 2).float().contiguous()
            out = droid_backends.corr_pyramid_lookup_tiled(self._pyr, self.level_shapes, c, self.slot_tensor())
            return out.view(batch, num, -1, ht, wd)
        pyr = self.reference_pyramid()
        if torch.is_grad_enabled() and any(v.requires_grad for v in pyr):
            c = coords.permute(0, 1, 4, 2, 3).contiguous().view(batch * num, 2, ht, wd)
            out = [CorrSampler.apply(pyr[i], c / 2 ** i, self.radius).view(batch, num, -1, ht, wd)
                   for i in range(self.num_levels)]
            return torch.cat(out, dim=2)
        c = coords.reshape(batch * num, ht, wd, 2).float().contiguous()
        out = droid_backends.corr_pyramid_lookup(pyr, c, self.radius)
        return out.view(batch, num, -1, ht, wd)

    def lookup_nhwc(self, coords):
        """fused-operator layout: (E,H,W,200) fp16 rows (196 used), one launch."""
        batch, num, ht, wd, _ = coords.shape
        c = coords.reshape(batch * num, ht, wd, 2).float().contiguous()
        return droid_backends.corr_pyramid_lookup_nhwc(self.reference_pyramid(), c, 200)

    # -- edge edits.  A tiled block (the fused operator's) is a SLOT POOL once
    # edited: its levels hold R >= E volumes, edge e's at row slots[e]; appending
    # edges fills free rows (the pool grows by half when full) and dropping edges
    # frees their rows, so the frontend's per-keyframe edits (factor_graph.py:
    # 85-160) move only the new edges' volumes, never the whole pyramid.  The
    # fused lookup reads the pool in place (droid_corr_lookup_ce0_tiled_slots);
    # corr_pyramid returns the edges' volumes in edge order (a gather).

    @property
    def corr_pyramid(self):
        if self._slots is None:
            return self._pyr
        idx = self.slot_tensor().long()
        return [lv.index_select(0, idx) for lv in self._pyr]

    @corr_pyramid.setter
    def corr_pyramid(self, levels):
        self._pyr = levels
        self._slots = None       # np.int32 (E): volume row of each edge; None = row e
        self._free = []
        self._slot_dev = None

    def num_edges(self):
        return len(self._slots) if self._slots is not None else self._pyr[0].shape[0]

    def pool_levels(self):
        return self._pyr

    def slot_tensor(self):
        """device int32 (E) slot map of a pooled block, None when row e is edge e."""
        if self._slots is None:
            return None
        if self._slot_dev is None:
            self._slot_dev = upload(self._slots, self._pyr[0].device)
        return self._slot_dev

    def _pool(self):
        if self._slots is None:
            self._slots = np.arange(self._pyr[0].shape[0], dtype=np.int32)
            self._free = []
            self._slot_dev = None

    def cat(self, other):
        """append other's edges (after this block's)."""
        if not self.tiled:
            for i in range(self.num_levels):
                self._pyr[i] = torch.cat([self._pyr[i], other.corr_pyramid[i]], 0)
            return self
        self._pool()
        new = other.corr_pyramid
        n = new[0].shape[0]
        if len(self._free) < n:
            rows = self._pyr[0].shape[0]
            grow = max(n - len(self._free), rows // 2)
            self._pyr = [torch.cat([lv, lv.new_empty((grow,) + tuple(lv.shape[1:]))], 0) for lv in self._pyr]
            self._free.extend(range(rows, rows + grow))
        rows = np.asarray(self._free[:n], np.int32)
        del self._free[:n]
        ridx = upload(rows.astype(np.int64), self._pyr[0].device)
        for lv, nv in zip(self._pyr, new):
            lv.index_copy_(0, ridx, nv)
        self._slots = np.concatenate([self._slots, rows])
        self._slot_dev = None
        return self

    def select(self, keep):
        """keep the edges where the host bool mask `keep` is set."""
        keep = np.asarray(keep, dtype=bool).reshape(-1)
        if not self.tiled:
            k = upload(keep, self._pyr[0].device)
            self._pyr = [lv[k] for lv in self._pyr]
            return self
        self._pool()
        self._free.extend(self._slots[~keep].tolist())
        self._slots = self._slots[keep]
        self._slot_dev = None
        return self

    def __getitem__(self, index):
        if isinstance(index, torch.Tensor) and index.dtype == torch.bool:
            return self.select(index.cpu().numpy())
        if self._slots is not None:
            raise RuntimeError("CorrBlock: index a pooled block with a bool mask (select)")
        for i in range(self.num_levels):
            self._pyr[i] = self._pyr[i][index]
        return self

    @staticmethod
    def corr(fmap1, fmap2):
        """all-pairs correlation <f1/4, f2/4> (corr.py:63-71)."""
        batch, num, dim, ht, wd = fmap1.shape
        f1 = fmap1.reshape(batch * num, dim, ht * wd) / 4.0
        f2 = fmap2.reshape(batch * num, dim, ht * wd) / 4.0
        return torch.matmul(f1.transpose(1, 2), f2).view(batch, num, ht, wd, ht, wd)


class CorrLayer(torch.autograd.Function):
    """corr.py:74-88."""

    @staticmethod
    def forward(ctx, fmap1, fmap2, coords, r):
        ctx.r = r
        ctx.save_for_backward(fmap1, fmap2, coords)
        corr, = droid_backends.altcorr_forward(fmap1, fmap2, coords, r)
        return corr

    @staticmethod
    def backward(ctx, grad_corr):
        fmap1, fmap2, coords = ctx.saved_tensors
        g1, g2, gc = droid_backends.altcorr_backward(fmap1, fmap2, coords, grad_corr.contiguous(), ctx.r)
        return g1, g2, gc, None


class AltCorrBlock:
    """corr.py:91-139 (on-the-fly correlation for update_lowmem)."""

    def __init__(self, fmaps, num_levels=4, radius=3):
        self.num_levels = num_levels
        self.radius = radius
        B, N, C, H, W = fmaps.shape
        f = fmaps.view(B * N, C, H, W) / 4.0
        self.pyramid = []
        for i in range(num_levels):
            self.pyramid.append(f.permute(0, 2, 3, 1).contiguous().view(B, N, H // 2 ** i, W // 2 ** i, C))
            if i + 1 < num_levels:
                f = F.avg_pool2d(f, 2, stride=2)

    def corr_fn(self, coords, ii, jj):
        B, N, H, W, S, _ = coords.shape
        coords = coords.permute(0, 1, 4, 2, 3, 5)
        out = []
        for i in range(self.num_levels):
            f1 = self.pyramid[0][:, ii].reshape((B * N,) + self.pyramid[0].shape[2:])
            f2 = self.pyramid[i][:, jj].reshape((B * N,) + self.pyramid[i].shape[2:])
            ci = (coords / 2 ** i).reshape(B * N, S, H, W, 2).contiguous()
            corr = CorrLayer.apply(f1.float().contiguous(), f2.float().contiguous(), ci, self.radius)
            out.append(corr.view(B, N, S, -1, H, W).permute(0, 1, 3, 4, 5, 2))
        return torch.cat(out, dim=2)

    def __call__(self, coords, ii, jj):
        squeeze = coords.dim() == 5
        if squeeze:
            coords = coords.unsqueeze(dim=-2)
        corr = self.corr_fn(coords, ii, jj)
        if squeeze:
            corr = corr.squeeze(dim=-1)
        return corr.contiguous()
