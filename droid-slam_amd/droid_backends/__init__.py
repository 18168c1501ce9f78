"""MI355X-native drop-in for the reference's `droid_backends` C extension.

Same module name, the same 9 functions and argument conventions as
/root/reference/src/droid.cpp:237-250, so `modules/corr.py`, `depth_video.py`
and `factor_graph.py` can import it unchanged.  Every call validates
contiguity like the reference (`RuntimeError: x must be contiguous`,
droid.cpp:84-85), then calls the hand-written gfx950 kernels of
libdroid_hip.so through its C ABI (include/droid_backends.h) on the caller's
current HIP stream.  There is no CPU fallback: host tensors raise.

Extensions beyond the reference surface (used by the MI355X-native host
mirror in `droid_mi355x`): `corr_pyramid_lookup`, `projective_transform`,
`BaPlan`, and optional host copies of ii/jj for `ba` (avoids the D2H sync).
"""
import ctypes
import os
from collections import OrderedDict

import numpy as np
import torch

from . import _lib
from ._lib import EXPORTS, check, lib

__all__ = ["ba", "frame_distance", "projmap", "depth_filter", "iproj", "altcorr_forward",
           "altcorr_backward", "corr_index_forward", "corr_index_backward",
           "corr_pyramid_lookup", "projective_transform", "BaPlan", "check_status", "EXPORTS"]

_DTYPES = {torch.float16: 0, torch.float32: 1, torch.float64: 2}


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _stream(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _check_inputs(names, tensors):
    dev = None
    for name, t in zip(names, tensors):
        if not isinstance(t, torch.Tensor):
            raise TypeError("%s must be a torch.Tensor" % name)
        if not t.is_contiguous():
            raise RuntimeError("%s must be contiguous" % name)
        if t.device.type != "cuda":
            raise RuntimeError("droid_backends: %s must be a HIP device tensor (no CPU path)" % name)
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise RuntimeError("droid_backends: all tensors must be on one device")
    return dev


def _need(t, dtype, name):
    if t.dtype != dtype:
        raise RuntimeError("%s must be %s (got %s)" % (name, dtype, t.dtype))


# ---------------------------------------------------------------------------
# correlation
# ---------------------------------------------------------------------------
def corr_index_forward(volume, coords, radius):
    """correlation_kernels.cu:126-155: volume (B,H,W,H2,W2), coords (B,2,H,W)
    -> [corr (B,2r+1,2r+1,H,W)] in volume's dtype."""
    _check_inputs(("volume", "coords"), (volume, coords))
    _need(coords, torch.float32, "coords")
    if volume.dtype not in _DTYPES:
        raise RuntimeError("volume must be float16/float32/float64")
    B, H, W, H2, W2 = volume.shape
    rd = 2 * radius + 1
    corr = torch.empty((B, rd, rd, H, W), dtype=volume.dtype, device=volume.device)
    with torch.cuda.device(volume.device):
        check(lib.droid_corr_index_forward(_DTYPES[volume.dtype], _ptr(volume), _ptr(coords), _ptr(corr),
                                           B, H, W, H2, W2, int(radius), _stream(volume)),
              "corr_index_forward")
    return [corr]


def corr_index_backward(volume, coords, corr_grad, radius):
    """correlation_kernels.cu:157-185 -> [volume_grad]."""
    _check_inputs(("volume", "coords", "corr_grad"), (volume, coords, corr_grad))
    B, H, W, H2, W2 = volume.shape
    if corr_grad.dtype != volume.dtype:
        raise RuntimeError("corr_grad must have the volume's dtype")
    grad = torch.zeros_like(volume)
    with torch.cuda.device(volume.device):
        check(lib.droid_corr_index_backward(_DTYPES[volume.dtype], _ptr(coords), _ptr(corr_grad),
                                            _ptr(grad), B, H, W, H2, W2, int(radius), _stream(volume)),
              "corr_index_backward")
    return [grad]


def corr_pyramid_lookup(levels, coords, radius, out=None):
    """All levels of CorrBlock.__call__ (modules/corr.py:40-50) in one launch.

    levels: list of (E,H,W,H2_l,W2_l) volumes; coords (E,H,W,2) f32 at level-0
    scale -> (E, L*(2r+1)^2, H, W)."""
    _check_inputs(["level%d" % i for i in range(len(levels))] + ["coords"], list(levels) + [coords])
    _need(coords, torch.float32, "coords")
    E, H, W = levels[0].shape[:3]
    dt = levels[0].dtype
    L = len(levels)
    rd = 2 * radius + 1
    if out is None:
        out = torch.empty((E, L * rd * rd, H, W), dtype=dt, device=coords.device)
    ptrs = (ctypes.c_void_p * L)(*[lv.data_ptr() for lv in levels])
    h2s = (ctypes.c_int * L)(*[lv.shape[3] for lv in levels])
    w2s = (ctypes.c_int * L)(*[lv.shape[4] for lv in levels])
    with torch.cuda.device(coords.device):
        check(lib.droid_corr_pyramid_lookup(_DTYPES[dt], ptrs, h2s, w2s, L, _ptr(coords), _ptr(out),
                                            E, H, W, int(radius), _stream(coords)),
              "corr_pyramid_lookup")
    return out


def corr_pyramid_lookup_tiled(levels, level_shapes, coords, slots=None, out=None):
    """CorrBlock.__call__ over the 8x8-tiled slot pool (fp16, r=3): levels[l]
    (R,H,W,ceil(H2/8),W2/8,8,8), level_shapes [(H2, W2)], slots (E) int32 device
    volume rows (None: row e), coords (E,H,W,2) f32 -> (E, L*49, H, W) fp16."""
    _check_inputs(["level%d" % i for i in range(len(levels))] + ["coords"], list(levels) + [coords])
    _need(coords, torch.float32, "coords")
    for lv in levels:
        _need(lv, torch.float16, "levels")
    E, H, W = coords.shape[:3]
    if slots is not None:
        _check_inputs(("slots",), (slots,))
        _need(slots, torch.int32, "slots")
        if slots.numel() != E:
            raise RuntimeError("corr_pyramid_lookup_tiled: one slot per edge")
    elif levels[0].shape[0] < E:
        raise RuntimeError("corr_pyramid_lookup_tiled: fewer volume rows than edges")
    L = len(levels)
    if out is None:
        out = torch.empty((E, L * 49, H, W), dtype=torch.float16, device=coords.device)
    ptrs = (ctypes.c_void_p * L)(*[lv.data_ptr() for lv in levels])
    h2s = (ctypes.c_int * L)(*[int(h) for h, _ in level_shapes])
    w2s = (ctypes.c_int * L)(*[int(w) for _, w in level_shapes])
    with torch.cuda.device(coords.device):
        check(lib.droid_corr_pyramid_lookup_tiled(ptrs, h2s, w2s, _ptr(slots) if slots is not None else None, L,
                                                  _ptr(coords), _ptr(out), E, H, W, _stream(coords)),
              "corr_pyramid_lookup_tiled")
    return out


def corr_pyramid_lookup_nhwc(levels, coords, out_cstride=200, out=None):
    """CorrBlock lookup (fp16, r=3, 4 levels) -> channels-last (E,H,W,out_cstride)
    rows, zero past channel 196 (A operand of the fused update operator)."""
    _check_inputs(["level%d" % i for i in range(len(levels))] + ["coords"], list(levels) + [coords])
    _need(coords, torch.float32, "coords")
    E, H, W = levels[0].shape[:3]
    if out is None:
        out = torch.empty((E, H, W, out_cstride), dtype=torch.float16, device=coords.device)
    L = len(levels)
    ptrs = (ctypes.c_void_p * L)(*[lv.data_ptr() for lv in levels])
    h2s = (ctypes.c_int * L)(*[lv.shape[3] for lv in levels])
    w2s = (ctypes.c_int * L)(*[lv.shape[4] for lv in levels])
    with torch.cuda.device(coords.device):
        check(lib.droid_corr_pyramid_lookup_nhwc(ptrs, h2s, w2s, L, _ptr(coords), _ptr(out), int(out_cstride),
                                                 E, H, W, _stream(coords)), "corr_pyramid_lookup_nhwc")
    return out


def corr_volume_pyramid(fmaps, f1, f2, tiled, num_levels=4):
    """CorrBlock pyramid of E edges (include/droid_backends.h:
    droid_corr_volume_pyramid): fmaps (NF,H,W,128) fp16 = frame features / 4,
    NHWC; f1/f2 (E) int32 frame rows -> 4 levels, (E,H,W,H_l,W_l) or, tiled,
    (E,H,W,ceil(H_l/8),W_l/8,8,8) fp16."""
    _check_inputs(("fmaps", "f1", "f2"), (fmaps, f1, f2))
    _need(fmaps, torch.float16, "fmaps")
    _need(f1, torch.int32, "f1")
    _need(f2, torch.int32, "f2")
    if num_levels != 4 or fmaps.dim() != 4 or fmaps.shape[-1] != 128:
        raise RuntimeError("corr_volume_pyramid: fmaps must be (NF,H,W,128) and 4 levels")
    NF, H, W, _ = fmaps.shape
    E = f1.numel()
    if f2.numel() != E:
        raise RuntimeError("corr_volume_pyramid: f1 and f2 must have one entry per edge")
    levels = []
    for l in range(4):
        h, w = H >> l, W >> l
        shape = (E, H, W, (h + 7) // 8, w // 8, 8, 8) if tiled else (E, H, W, h, w)
        levels.append(torch.empty(shape, dtype=torch.float16, device=fmaps.device))
    ptrs = (ctypes.c_void_p * 4)(*[lv.data_ptr() for lv in levels])
    with torch.cuda.device(fmaps.device):
        check(lib.droid_corr_volume_pyramid(_ptr(fmaps), _ptr(f1), _ptr(f2), E, NF, H, W, ptrs, int(bool(tiled)),
                                            _stream(fmaps)), "corr_volume_pyramid")
    return levels


def corr_volume_pyramid_supported(H, W, tiled):
    """Shapes droid_corr_volume_pyramid accepts."""
    return H % 8 == 0 and W % 8 == 0 and (not tiled or W % 64 == 0)


def corr_lookup_ce0_supported(levels, H, W):
    """Shapes droid_corr_lookup_ce0 accepts: 4 levels, H*W % 128 == 0."""
    return len(levels) == 4 and (H * W) % 128 == 0


def corr_lookup_ce0(levels, coords, w, bias, out=None, tiled_shapes=None, slots=None):
    """Fused CorrBlock lookup + corr_encoder[0] (include/droid_backends.h:
    droid_corr_lookup_ce0): levels 4 x (E,H,W,H2,W2) fp16, coords (E,H,W,2) f32,
    w [128][224] fp16, bias [128] f32 -> (E,H,W,128) fp16 = relu(w . lookup + b).
    tiled_shapes [(H2,W2)] x 4: the levels are 8x8-tiled (corr.tile8) and go to
    droid_corr_lookup_ce0_tiled.  slots (E) int32 (tiled only): the levels are a
    pool of R >= E volumes, edge e's at row slots[e]
    (droid_corr_lookup_ce0_tiled_slots)."""
    _check_inputs(["level%d" % i for i in range(len(levels))] + ["coords", "w", "bias"],
                  list(levels) + [coords, w, bias])
    _need(coords, torch.float32, "coords")
    _need(w, torch.float16, "w")
    _need(bias, torch.float32, "bias")
    E, H, W = coords.shape[:3]
    if slots is not None:
        _need(slots, torch.int32, "slots")
        if tiled_shapes is None:
            raise RuntimeError("corr_lookup_ce0: a slot pool needs the tiled layout")
        if slots.shape != (E,) or slots.device != coords.device or not slots.is_contiguous():
            raise RuntimeError("corr_lookup_ce0: slots must be a contiguous (E,) int32 tensor on the coords' device")
    elif tuple(levels[0].shape[:3]) != (E, H, W):
        raise RuntimeError("corr_lookup_ce0: level 0 %s does not match coords %s"
                           % (tuple(levels[0].shape), tuple(coords.shape)))
    if out is None:
        out = torch.empty((E, H, W, 128), dtype=torch.float16, device=coords.device)
    L = len(levels)
    ptrs = (ctypes.c_void_p * L)(*[lv.data_ptr() for lv in levels])
    if tiled_shapes is not None:
        for lv, (h2, w2) in zip(levels, tiled_shapes):
            if tuple(lv.shape[3:]) != ((h2 + 7) // 8, w2 // 8, 8, 8):
                raise RuntimeError("corr_lookup_ce0: level shape %s is not the 8x8 tiling of %dx%d"
                                   % (tuple(lv.shape), h2, w2))
        h2s = (ctypes.c_int * L)(*[h for h, _ in tiled_shapes])
        w2s = (ctypes.c_int * L)(*[w_ for _, w_ in tiled_shapes])
        if slots is not None:
            with torch.cuda.device(coords.device):
                check(lib.droid_corr_lookup_ce0_tiled_slots(ptrs, h2s, w2s, _ptr(slots), _ptr(coords), _ptr(w),
                                                            _ptr(bias), _ptr(out), E, H, W, _stream(coords)),
                      "corr_lookup_ce0_tiled_slots")
            return out
        fn, name = lib.droid_corr_lookup_ce0_tiled, "corr_lookup_ce0_tiled"
    else:
        h2s = (ctypes.c_int * L)(*[lv.shape[3] for lv in levels])
        w2s = (ctypes.c_int * L)(*[lv.shape[4] for lv in levels])
        fn, name = lib.droid_corr_lookup_ce0, "corr_lookup_ce0"
    with torch.cuda.device(coords.device):
        check(fn(ptrs, h2s, w2s, _ptr(coords), _ptr(w), _ptr(bias), _ptr(out), E, H, W, _stream(coords)), name)
    return out


def corr_alt_ce0(pyramid, f1, f2, coords, w, bias, out=None, order=None):
    """On-the-fly correlation lookup + corr_encoder[0] (include/droid_backends.h:
    droid_corr_alt_ce0): pyramid 4 x (NF,H_l,W_l,128) fp16 (AltCorrBlock layout),
    f1/f2 (E) int32 pyramid rows, coords (E,H,W,2) f32, w [128][224] fp16,
    bias [128] f32 -> (E,H,W,128) fp16.  order: optional (E) int32 device
    permutation the tiles are walked in (droid_corr_alt_ce0_ordered; same output)."""
    _check_inputs(["level%d" % i for i in range(len(pyramid))] + ["f1", "f2", "coords", "w", "bias"],
                  list(pyramid) + [f1, f2, coords, w, bias])
    _need(coords, torch.float32, "coords")
    _need(f1, torch.int32, "f1")
    _need(f2, torch.int32, "f2")
    _need(w, torch.float16, "w")
    _need(bias, torch.float32, "bias")
    if len(pyramid) != 4:
        raise RuntimeError("corr_alt_ce0: needs 4 pyramid levels")
    E, H, W, _ = coords.shape
    if out is None:
        out = torch.empty((E, H, W, 128), dtype=torch.float16, device=coords.device)
    ptrs = (ctypes.c_void_p * 4)(*[lv.data_ptr() for lv in pyramid])
    hs = (ctypes.c_int * 4)(*[lv.shape[-3] for lv in pyramid])
    ws = (ctypes.c_int * 4)(*[lv.shape[-2] for lv in pyramid])
    if order is not None:
        _check_inputs(("order",), (order,))
        _need(order, torch.int32, "order")
        if order.numel() != E:
            raise RuntimeError("corr_alt_ce0: order must hold one entry per edge")
    with torch.cuda.device(coords.device):
        check(lib.droid_corr_alt_ce0_ordered(ptrs, hs, ws, _ptr(f1), _ptr(f2), _ptr(order), _ptr(coords), _ptr(w),
                                             _ptr(bias), _ptr(out), E, H, W, _stream(coords)), "corr_alt_ce0")
    return out


BA_ORDERS = ("identity", "rcm", "mindeg", "nd")


def ba_set_order(order):
    """Pose order of the BA plans built from now on (droid_ba_set_order):
    None = chosen per plan (default) or one of BA_ORDERS.  Returns the previous
    setting (None or a name).  Cached plans keep their order."""
    prev = lib.droid_ba_set_order(-1 if order is None else BA_ORDERS.index(order))
    if prev == -2:
        raise RuntimeError("ba_set_order: order must be None or one of %s" % (BA_ORDERS,))
    return None if prev < 0 else BA_ORDERS[prev]


# the library's build (droid_build_info): the A/B build carries the dropped
# kernel variants and reads the DROID_* experiment knobs; the product does not
AB_BUILD = bool(lib.droid_build_info() & 1)

CHOL_INJECT_OFF, CHOL_INJECT_ALL, CHOL_INJECT_ONCE, CHOL_INJECT_STALE = 0, 1, 2, 3


def chol_set_fault_inject(mode):
    """Test hook (droid_chol_set_fault_inject): CHOL_INJECT_ALL makes every
    dataflow solve abort as on a dependency-wait timeout, CHOL_INJECT_ONCE only
    the next one, CHOL_INJECT_STALE launches the next solve on a sync area that
    was not zeroed (the kernel's entry check reports it)."""
    check(_lib.testing_hook("droid_chol_set_fault_inject")(int(mode)), "chol_set_fault_inject")


def alt_set_variant(v):
    """A/B hook (droid_alt_set_variant): 2 = corr_alt2_kernel (the product); the A/B
    build adds 1 = corr_alt_ce0_kernel, 3 = corr_alt2_kernel<V3>, 4 = the round-4 V2,
    5 = V2 with the row-K lookup tile, 6 = V2 with the pixel-major C layout."""
    check(_lib.testing_hook("droid_alt_set_variant")(int(v)), "alt_set_variant")


def lookup_set_coop(on):
    """A/B hook (droid_lookup_set_coop): the cooperative NCHW lookup (1, default) or the per-thread kernel (0)."""
    check(_lib.testing_hook("droid_lookup_set_coop")(1 if on else 0), "lookup_set_coop")


def alt_set_chunk(edges):
    """A/B hook (droid_alt_set_chunk): edges per XCD chunk of corr_alt2_kernel's walk, 0 = interleaved."""
    check(_lib.testing_hook("droid_alt_set_chunk")(int(edges)), "alt_set_chunk")


def conv_set_tile(mode):
    """Tile policy of the W=64 3x3 band convs (droid_conv_set_tile): -1 default,
    0 = 8-wave band tiles only, 1 = the two-workgroups-per-CU tile wherever it
    applies.  Returns the previous policy."""
    prev = _lib.testing_hook("droid_conv_set_tile")(int(mode))
    if prev == -2:
        raise RuntimeError("conv_set_tile: mode must be -1, 0 or 1")
    return prev


def conv_gate_tile(epi, B, H, W):
    """droid_conv_gate_tile: the kernel a gate conv of this shape runs on
    (1 band2, 0 the 8-wave band tile, 2 the 4-wave z|r tile, -1 none)."""
    return int(_lib.testing_hook("droid_conv_gate_tile")(int(epi), int(B), int(H), int(W)))


EPI_ACT, EPI_GRU_ZR, EPI_GRU_Q, EPI_HEAD, EPI_GLO = 0, 1, 2, 3, 4


def _conv_operands(fn, B, H, W, cout, dev, bias=None, bbias=None, maps16=(), out32=None):
    """Dtype / layout / size checks of the conv entry points' side operands (the
    kernels read them through raw pointers: an fp16 bias from an autocast region,
    say, would be read as fp32 past its end)."""
    def vec(t, name, n):
        if t is None:
            return
        if (t.dtype != torch.float32 or not t.is_contiguous() or t.device != dev or t.numel() < n):
            raise RuntimeError("%s: %s must be a contiguous float32 tensor of >= %d elements on %s"
                               % (fn, name, n, dev))
    vec(bias, "bias", cout)
    vec(bbias, "bbias", B * cout)
    for name, t in maps16:
        if t is not None and (t.dtype != torch.float16 or not t.is_contiguous() or t.device != dev
                              or t.dim() != 4 or tuple(t.shape[:3]) != (B, H, W)):
            raise RuntimeError("%s: %s must be a contiguous fp16 (B,H,W,C) tensor matching the sources" % (fn, name))
    if out32 is not None and (out32.dtype != torch.float32 or not out32.is_contiguous() or out32.device != dev
                              or out32.shape[0] != B):
        raise RuntimeError("%s: out32 must be a contiguous float32 tensor with one row per image" % fn)


def conv_nhwc_f16(sources, wp, cout, ks, bias=None, bbias=None, act=0, epi=EPI_ACT, out=None, out_coff=0,
                  h=None, z=None, zout=None, rnet=None, out32=None, gru_ch=128):
    """Implicit-GEMM MFMA conv (include/droid_backends.h: droid_conv_nhwc_f16).

    sources: list of (tensor, channel_offset, channels); each tensor NHWC fp16
    contiguous (B,H,W,cstride).  wp: packed weights (droid_mi355x.fused.pack_conv)."""
    t0 = sources[0][0]
    B, H, W = t0.shape[:3]
    n = len(sources)
    ptrs = (ctypes.c_void_p * n)(*[t.data_ptr() + 2 * off for t, off, _ in sources])
    cs = (ctypes.c_int * n)(*[c for _, _, c in sources])
    strides = (ctypes.c_int * n)(*[t.shape[-1] for t, _, _ in sources])
    for t, _, _ in sources:
        if t.dtype != torch.float16 or not t.is_contiguous() or t.shape[:3] != (B, H, W):
            raise RuntimeError("conv_nhwc_f16: sources must be contiguous fp16 (B,H,W,C) tensors")
    _conv_operands("conv_nhwc_f16", B, H, W, int(cout), t0.device, bias, bbias,
                   (("out", out), ("h", h), ("z", z), ("zout", zout), ("rnet", rnet)), out32)
    out_cs = out.shape[-1] if out is not None else 0
    if epi == EPI_HEAD:
        out_cs = out32.shape[-1]
    with torch.cuda.device(t0.device):
        check(lib.droid_conv_nhwc_f16(ptrs, cs, strides, n, _ptr(wp), _ptr(bias), _ptr(bbias), B, H, W, int(cout),
                                      int(ks), int(act), int(epi), _ptr(out), int(out_cs), int(out_coff),
                                      _ptr(h), h.shape[-1] if h is not None else 0, _ptr(z),
                                      z.shape[-1] if z is not None else 0, _ptr(zout), _ptr(rnet), int(gru_ch),
                                      _ptr(out32), _stream(t0)), "conv_nhwc_f16")
    return out


def gru_pre_supported(H, W):
    """Shapes droid_conv_gru_pre_f16 accepts for both gates (z|r on the 256x256
    band tile, q on the 384x128 one)."""
    return W in (16, 32, 64) and (H * W) % 768 == 0


def conv_gru_pre_f16(sources, wp, cout, bias, bbias, epi, pre, pre_idx, pre_coff, h, z=None, zout=None,
                     rnet=None, out=None, gru_ch=128):
    """ConvGRU gate conv with the per-source-frame term factored out
    (include/droid_backends.h: droid_conv_gru_pre_f16): the gate argument is
    conv3x3(sources) + bias + bbias[b] + pre[pre_idx[b], :, :, pre_coff:pre_coff+cout].
    pre (F,H,W,Cp) fp16 contiguous; pre_idx (B,) int64 on the device."""
    t0 = sources[0][0]
    B, H, W = t0.shape[:3]
    n = len(sources)
    for t, _, _ in sources:
        if t.dtype != torch.float16 or not t.is_contiguous() or t.shape[:3] != (B, H, W):
            raise RuntimeError("conv_gru_pre_f16: sources must be contiguous fp16 (B,H,W,C) tensors")
    _check_inputs(("pre", "pre_idx"), (pre, pre_idx))
    _need(pre, torch.float16, "pre")
    _need(pre_idx, torch.int64, "pre_idx")
    if pre.dim() != 4 or tuple(pre.shape[1:3]) != (H, W) or pre_idx.numel() != B:
        raise RuntimeError("conv_gru_pre_f16: pre must be (F,H,W,C) and pre_idx hold one frame per image")
    _conv_operands("conv_gru_pre_f16", B, H, W, int(cout), t0.device, bias, bbias,
                   (("out", out), ("h", h), ("z", z), ("zout", zout), ("rnet", rnet)))
    ptrs = (ctypes.c_void_p * n)(*[t.data_ptr() + 2 * off for t, off, _ in sources])
    cs = (ctypes.c_int * n)(*[c for _, _, c in sources])
    strides = (ctypes.c_int * n)(*[t.shape[-1] for t, _, _ in sources])
    with torch.cuda.device(t0.device):
        check(lib.droid_conv_gru_pre_f16(ptrs, cs, strides, n, _ptr(wp), _ptr(bias), _ptr(bbias), B, H, W, int(cout),
                                         int(epi), _ptr(out), out.shape[-1] if out is not None else 0, 0, _ptr(h),
                                         h.shape[-1], _ptr(z), z.shape[-1] if z is not None else 0, _ptr(zout),
                                         _ptr(rnet), int(gru_ch), _ptr(pre), _ptr(pre_idx), pre.shape[-1],
                                         int(pre_coff), _stream(t0)), "conv_gru_pre_f16")
    return out


def wino_supported(H, W, cout):
    """Whether the update operator takes the Winograd tile: only with the A/B
    library (make ab; DROID_HIP_LIB) and opted in with DROID_CONV_WINO=1 (it
    measures slower than the direct band tile on MI355X,
    csrc/conv_kernels.hip: conv_wino_kernel) and a shape droid_conv_wino_f16
    accepts (W == 64, whole 4-row tiles, 128-channel output tiles)."""
    return (AB_BUILD and W == 64 and H % 4 == 0 and cout % 128 == 0
            and os.environ.get("DROID_CONV_WINO", "0") == "1")


def conv_wino_f16(sources, wt, cout, bias=None, bbias=None, act=0, epi=EPI_ACT, out=None, out_coff=0,
                  pre=None, pre_idx=None, pre_coff=0, h=None, z=None, zout=None, rnet=None, gru_ch=128):
    """3x3 conv as Winograd F(2,3) along x (include/droid_backends.h:
    droid_conv_wino_f16).  wt: transformed weights (droid_mi355x.fused.pack_conv_wino);
    epi EPI_ACT (act 0 / 1 -> out) or EPI_GRU_ZR / EPI_GRU_Q with the per-source-frame
    term pre / pre_idx / pre_coff as in conv_gru_pre_f16."""
    t0 = sources[0][0]
    B, H, W = t0.shape[:3]
    n = len(sources)
    for t, _, _ in sources:
        if t.dtype != torch.float16 or not t.is_contiguous() or t.shape[:3] != (B, H, W):
            raise RuntimeError("conv_wino_f16: sources must be contiguous fp16 (B,H,W,C) tensors")
    _need(wt, torch.float16, "wt")
    if epi != EPI_ACT:
        _check_inputs(("pre", "pre_idx"), (pre, pre_idx))
        _need(pre, torch.float16, "pre")
        _need(pre_idx, torch.int64, "pre_idx")
        if pre.dim() != 4 or tuple(pre.shape[1:3]) != (H, W) or pre_idx.numel() != B:
            raise RuntimeError("conv_wino_f16: pre must be (F,H,W,C) and pre_idx hold one frame per image")
    _conv_operands("conv_wino_f16", B, H, W, int(cout), t0.device, bias, bbias,
                   (("out", out), ("h", h), ("z", z), ("zout", zout), ("rnet", rnet)))
    ptrs = (ctypes.c_void_p * n)(*[t.data_ptr() + 2 * off for t, off, _ in sources])
    cs = (ctypes.c_int * n)(*[c for _, _, c in sources])
    strides = (ctypes.c_int * n)(*[t.shape[-1] for t, _, _ in sources])
    with torch.cuda.device(t0.device):
        check(lib.droid_conv_wino_f16(ptrs, cs, strides, n, _ptr(wt), _ptr(bias), _ptr(bbias), B, H, W, int(cout),
                                      int(act), int(epi), _ptr(out), out.shape[-1] if out is not None else 0,
                                      int(out_coff), _ptr(h), h.shape[-1] if h is not None else 0, _ptr(z),
                                      z.shape[-1] if z is not None else 0, _ptr(zout), _ptr(rnet), int(gru_ch),
                                      _ptr(pre), _ptr(pre_idx), pre.shape[-1] if pre is not None else 0,
                                      int(pre_coff), _stream(t0)), "conv_wino_f16")
    return out


def transpose_f16(src, R, C, ldd=None, out=None):
    """dst[b][c][r] = src[b][r][c] (r < R), zero for R <= r < ldd
    (include/droid_backends.h: droid_transpose_f16): src viewed as (B, R, C) fp16
    contiguous -> out (B, C, ldd) fp16."""
    _check_inputs(("src",), (src,))
    _need(src, torch.float16, "src")
    ldd = R if ldd is None else int(ldd)
    if R * C == 0 or src.numel() % (R * C):
        raise RuntimeError("transpose_f16: src is not a whole number of (R, C) blocks")
    B = src.numel() // (R * C)
    if out is None:
        out = torch.empty((B, C, ldd), dtype=torch.float16, device=src.device)
    elif out.dtype != torch.float16 or not out.is_contiguous() or out.numel() != B * C * ldd:
        raise RuntimeError("transpose_f16: out must be a contiguous fp16 tensor of B*C*ldd elements")
    with torch.cuda.device(src.device):
        check(lib.droid_transpose_f16(_ptr(src), _ptr(out), int(B), int(R), int(C), int(ldd), _stream(src)),
              "transpose_f16")
    return out


def conv1x1_nchw_f16(src, w, bias, relu=True, out=None):
    """corr_encoder[0] on an NCHW lookup (include/droid_backends.h:
    droid_conv1x1_nchw_f16): src (E, C, H, W) fp16 contiguous, w [128][K] fp16
    (K % 32 == 0, columns >= C zero), bias [128] f32 -> (E, H, W, 128) fp16."""
    _check_inputs(("src", "w", "bias"), (src, w, bias))
    _need(src, torch.float16, "src")
    _need(w, torch.float16, "w")
    _need(bias, torch.float32, "bias")
    E, C, H, W = src.shape
    if w.dim() != 2 or w.shape[0] != 128 or bias.numel() != 128:
        raise RuntimeError("conv1x1_nchw_f16: w must be (128, K) and bias (128,)")
    if out is None:
        out = torch.empty((E, H, W, 128), dtype=torch.float16, device=src.device)
    with torch.cuda.device(src.device):
        check(lib.droid_conv1x1_nchw_f16(_ptr(src), int(C), _ptr(w), int(w.shape[1]), _ptr(bias), _ptr(out), int(E),
                                         int(H * W), int(bool(relu)), _stream(src)), "conv1x1_nchw_f16")
    return out


def dw_head_supported(H, W):
    """Shapes droid_conv_dw_head_f16 accepts (the band tile: W in {16,32,64}, H*W % 256 == 0)."""
    return W in (16, 32, 64) and (H * W) % 256 == 0


def conv_dw_head_f16(sources, wp, bias, head_w, out32):
    """Fused delta/weight heads (include/droid_backends.h: droid_conv_dw_head_f16):
    relu(conv3x3(sources) + bias) -> 256 channels, kept on chip, then the 3x3
    256->4 head conv accumulated into out32 (B,H,W,4) fp32 (zeroed by the caller)."""
    t0 = sources[0][0]
    B, H, W = t0.shape[:3]
    n = len(sources)
    for t, _, _ in sources:
        if t.dtype != torch.float16 or not t.is_contiguous() or t.shape[:3] != (B, H, W):
            raise RuntimeError("conv_dw_head_f16: sources must be contiguous fp16 (B,H,W,C) tensors")
    if out32.dtype != torch.float32 or not out32.is_contiguous() or tuple(out32.shape) != (B, H, W, 4):
        raise RuntimeError("conv_dw_head_f16: out32 must be a contiguous (B,H,W,4) float32 tensor")
    _conv_operands("conv_dw_head_f16", B, H, W, 256, t0.device, bias)
    ptrs = (ctypes.c_void_p * n)(*[t.data_ptr() + 2 * off for t, off, _ in sources])
    cs = (ctypes.c_int * n)(*[c for _, _, c in sources])
    strides = (ctypes.c_int * n)(*[t.shape[-1] for t, _, _ in sources])
    with torch.cuda.device(t0.device):
        check(lib.droid_conv_dw_head_f16(ptrs, cs, strides, n, _ptr(wp), _ptr(bias), B, H, W, _ptr(head_w),
                                         _ptr(out32), _stream(t0)), "conv_dw_head_f16")
    return out32


def head_finish(head, b, base=None, target_ba=None, weight_ba=None, row0=0):
    """The heads' finish (include/droid_backends.h: droid_head_finish_f32):
    head (E,H,W,4) f32 raw head sums, b (4) f32, base (E,H,W,2) f32 or None ->
    (target, weight) (E,H,W,2) f32 = (base + delta, sigmoid(w)); target_ba /
    weight_ba (R,2,H,W) f32: also written at rows row0 .. row0 + E - 1."""
    E, H, W, _ = head.shape
    _check_inputs(("head", "b"), (head, b))
    for t, nm in ((head, "head"), (b, "b")):
        _need(t, torch.float32, nm)
    if base is not None:
        _check_inputs(("base",), (base,))
        _need(base, torch.float32, "base")
        if tuple(base.shape) != (E, H, W, 2):
            raise RuntimeError("head_finish: base must be (E,H,W,2)")
    if (target_ba is None) != (weight_ba is None):
        raise RuntimeError("head_finish: target_ba and weight_ba go together")
    if target_ba is not None:
        for t, nm in ((target_ba, "target_ba"), (weight_ba, "weight_ba")):
            _check_inputs((nm,), (t,))
            _need(t, torch.float32, nm)
            if t.dim() != 4 or tuple(t.shape[1:]) != (2, H, W) or row0 < 0 or row0 + E > t.shape[0]:
                raise RuntimeError("head_finish: %s must be (R,2,H,W) with rows %d..%d" % (nm, row0, row0 + E - 1))
    target = torch.empty((E, H, W, 2), dtype=torch.float32, device=head.device)
    weight = torch.empty((E, H, W, 2), dtype=torch.float32, device=head.device)
    with torch.cuda.device(head.device):
        check(lib.droid_head_finish_f32(_ptr(head), _ptr(b), _ptr(base) if base is not None else None, _ptr(target),
                                        _ptr(weight), _ptr(target_ba) if target_ba is not None else None,
                                        _ptr(weight_ba) if weight_ba is not None else None, int(row0), E, H * W,
                                        _stream(head)), "head_finish_f32")
    return target, weight


def eta_damping(er, map_, frames, state, ep):
    """GraphAgg's damping into the BA (include/droid_backends.h:
    droid_eta_damping_f32): er (U,H,W,1) fp16 raw eta conv, map_ / frames (K)
    int32 (row of er or -1, frame id), state (N,H,W) f32 (updated in place) ->
    (K,H,W) f32 = 0.2 state[frames] + ep."""
    U, H, W = er.shape[:3]
    _check_inputs(("er", "map", "frames", "state"), (er, map_, frames, state))
    _need(er, torch.float16, "er")
    _need(map_, torch.int32, "map")
    _need(frames, torch.int32, "frames")
    _need(state, torch.float32, "state")
    if tuple(state.shape[1:]) != (H, W) or map_.shape != frames.shape:
        raise RuntimeError("eta_damping: state must be (N,H,W) and map / frames the same (K) shape")
    out = torch.empty((frames.shape[0], H, W), dtype=torch.float32, device=er.device)
    with torch.cuda.device(er.device):
        check(lib.droid_eta_damping_f32(_ptr(er), _ptr(map_), _ptr(frames), _ptr(state), _ptr(out), frames.shape[0],
                                        H * W, float(ep), _stream(er)), "eta_damping_f32")
    return out


def flow_enc0_supported(H, W):
    """Shapes droid_flow_enc0_f16 accepts."""
    return W in (16, 32, 64, 128) and (H * W) % 128 == 0


def flow_enc0_f16(motn, w, bias, out=None):
    """flow_encoder[0] (include/droid_backends.h: droid_flow_enc0_f16): motn (E,4,H,W)
    f32, w [128][416] fp16 (droid_mi355x.fused.pack_flow_enc0), bias [128] f32 ->
    (E,H,W,128) fp16 = relu(conv7x7(motn) + bias)."""
    _check_inputs(("motn", "w", "bias"), (motn, w, bias))
    _need(motn, torch.float32, "motn")
    _need(w, torch.float16, "w")
    _need(bias, torch.float32, "bias")
    E, C, H, W = motn.shape
    if C != 4 or tuple(w.shape) != (128, 416):
        raise RuntimeError("flow_enc0_f16: motn must have 4 channels and w be 128x416")
    if out is None:
        out = torch.empty((E, H, W, 128), dtype=torch.float16, device=motn.device)
    with torch.cuda.device(motn.device):
        check(lib.droid_flow_enc0_f16(_ptr(motn), _ptr(w), _ptr(bias), _ptr(out), E, H, W, _stream(motn)),
              "flow_enc0_f16")
    return out


def gru_glo_gates(h, w, bias, gw, gb):
    """The ConvGRU global-context branch end to end: glo = mean_px sigmoid(w h +
    bias) h (droid_gru_global[_split]_f16), then its three 1x1 gate convs
    (droid_glo_gates_f32): h (E,H,W,128) fp16, w [128][128] fp16, bias [128],
    gw (384,128) f32, gb (384) f32 -> ((E,256) f32 z | r terms, (E,128) f32 q terms)."""
    _check_inputs(("h", "w", "bias", "gw", "gb"), (h, w, bias, gw, gb))
    _need(gw, torch.float32, "gw")
    _need(gb, torch.float32, "gb")
    E, H, W, C = h.shape
    if tuple(gw.shape) != (384, 128) or gb.numel() != 384:
        raise RuntimeError("gru_glo_gates: gw must be (384,128) and gb (384)")
    splits = max(1, min((H * W) // 256, -(-512 // max(E, 1))))
    part = torch.empty((splits, E, 128), dtype=torch.float32, device=h.device)
    out_zr = torch.empty((E, 256), dtype=torch.float32, device=h.device)
    out_q = torch.empty((E, 128), dtype=torch.float32, device=h.device)
    with torch.cuda.device(h.device):
        if splits == 1:
            check(lib.droid_gru_global_f16(_ptr(h), _ptr(w), _ptr(bias), _ptr(part), E, H * W, _stream(h)),
                  "gru_global_f16")
        else:
            check(lib.droid_gru_global_split_f16(_ptr(h), _ptr(w), _ptr(bias), _ptr(part), splits, E, H * W,
                                                 _stream(h)), "gru_global_split_f16")
        check(lib.droid_glo_gates_f32(_ptr(part), splits, _ptr(gw), _ptr(gb), _ptr(out_zr), _ptr(out_q), E,
                                      _stream(h)), "glo_gates_f32")
    return out_zr, out_q


def gru_global_f16(h, w, bias, out=None):
    """ConvGRU global context (include/droid_backends.h: droid_gru_global_f16):
    h (E,H,W,128) fp16, w [128][128] fp16, bias [128] f32 -> (E,128) f32."""
    _check_inputs(("h", "w", "bias"), (h, w, bias))
    _need(h, torch.float16, "h")
    _need(w, torch.float16, "w")
    _need(bias, torch.float32, "bias")
    E, H, W, C = h.shape
    if C != 128 or tuple(w.shape) != (128, 128):
        raise RuntimeError("gru_global_f16: h must have 128 channels and w be 128x128")
    # a small graph (the frontend's ~100 edges) gets several workgroups per edge:
    # ~512 in all, each at least 4 tiles of 64 pixels; their partial means are
    # added in order (deterministic)
    splits = max(1, min((H * W) // 256, -(-512 // max(E, 1))))
    with torch.cuda.device(h.device):
        if splits == 1:
            if out is None:
                out = torch.empty((E, 128), dtype=torch.float32, device=h.device)
            check(lib.droid_gru_global_f16(_ptr(h), _ptr(w), _ptr(bias), _ptr(out), E, H * W, _stream(h)),
                  "gru_global_f16")
            return out
        part = torch.empty((splits, E, 128), dtype=torch.float32, device=h.device)
        check(lib.droid_gru_global_split_f16(_ptr(h), _ptr(w), _ptr(bias), _ptr(part), splits, E, H * W,
                                             _stream(h)), "gru_global_split_f16")
    if out is None:
        return part.sum(0)
    return torch.sum(part, 0, out=out)


def segment_mean_f16(src, seg_ptr, seg_idx, num_segments, out=None):
    """GraphAgg scatter_mean (include/droid_backends.h: droid_segment_mean_f16):
    src (E, ...) fp16 contiguous; seg_ptr (U+1) / seg_idx (E) int64 CSR of the
    edges per segment -> out (U, ...) fp16 = per-segment mean of src rows."""
    _check_inputs(("src", "seg_ptr", "seg_idx"), (src, seg_ptr, seg_idx))
    _need(src, torch.float16, "src")
    _need(seg_ptr, torch.int64, "seg_ptr")
    _need(seg_idx, torch.int64, "seg_idx")
    if seg_ptr.numel() != num_segments + 1:
        raise RuntimeError("seg_ptr must have num_segments + 1 entries")
    row = src[0].numel() if src.shape[0] else 0
    if out is None:
        out = torch.empty((num_segments,) + tuple(src.shape[1:]), dtype=torch.float16, device=src.device)
    if num_segments == 0 or row == 0:
        return out
    with torch.cuda.device(src.device):
        check(lib.droid_segment_mean_f16(_ptr(src), _ptr(seg_ptr), _ptr(seg_idx), _ptr(out), int(num_segments),
                                         int(row), _stream(src)), "segment_mean_f16")
    return out


def altcorr_forward(fmap1, fmap2, coords, radius):
    """altcorr_kernel.cu:290-319: fmap1 (B,H,W,C), fmap2 (B,H2,W2,C),
    coords (B,S,H,W,2) -> [corr (B,S,(2r+1)^2,H,W)]."""
    _check_inputs(("fmap1", "fmap2", "coords"), (fmap1, fmap2, coords))
    _need(coords, torch.float32, "coords")
    if fmap1.dtype not in (torch.float16, torch.float32) or fmap2.dtype != fmap1.dtype:
        raise RuntimeError("fmaps must both be float16 or float32")
    B, H, W, C = fmap1.shape
    _, H2, W2, _ = fmap2.shape
    S = coords.shape[1]
    rd = 2 * radius + 1
    corr = torch.empty((B, S, rd * rd, H, W), dtype=fmap1.dtype, device=fmap1.device)
    with torch.cuda.device(fmap1.device):
        check(lib.droid_altcorr_forward(_DTYPES[fmap1.dtype], _ptr(fmap1), _ptr(fmap2), _ptr(coords),
                                        _ptr(corr), B, S, H, W, H2, W2, C, int(radius), _stream(fmap1)),
              "altcorr_forward")
    return [corr]


def altcorr_backward(fmap1, fmap2, coords, corr_grad, radius):
    """altcorr_kernel.cu:321-356 (fp32) -> [fmap1_grad, fmap2_grad, coords_grad(=0)]."""
    _check_inputs(("fmap1", "fmap2", "coords", "corr_grad"), (fmap1, fmap2, coords, corr_grad))
    for n, t in (("fmap1", fmap1), ("fmap2", fmap2), ("coords", coords), ("corr_grad", corr_grad)):
        _need(t, torch.float32, n)
    B, H, W, C = fmap1.shape
    _, H2, W2, _ = fmap2.shape
    S = coords.shape[1]
    g1 = torch.zeros_like(fmap1)
    g2 = torch.zeros_like(fmap2)
    gc = torch.zeros((B, S, H, W, 2), dtype=fmap1.dtype, device=fmap1.device)
    with torch.cuda.device(fmap1.device):
        check(lib.droid_altcorr_backward(_ptr(fmap1), _ptr(fmap2), _ptr(coords), _ptr(corr_grad),
                                         _ptr(g1), _ptr(g2), B, S, H, W, H2, W2, C, int(radius),
                                         _stream(fmap1)), "altcorr_backward")
    return [g1, g2, gc]


# ---------------------------------------------------------------------------
# geometry
# ---------------------------------------------------------------------------
def projective_transform(poses, disps, intrinsics, ii, jj, target=None, with_valid=True):
    """pops.projective_transform semantics (projective_ops.py:96-125), lietorch-free.

    poses (N,7), disps (N,H,W), intrinsics (N,4), ii/jj (E) int64 ->
    coords (E,H,W,2), valid (E,H,W,1) or None, and - when `target` (E,H,W,2)
    is given - the clamped update() motion features motn (E,4,H,W)."""
    args = [poses, disps, intrinsics, ii, jj] + ([target] if target is not None else [])
    _check_inputs(("poses", "disps", "intrinsics", "ii", "jj", "target")[:len(args)], args)
    for n, t in (("poses", poses), ("disps", disps), ("intrinsics", intrinsics)):
        _need(t, torch.float32, n)
    _need(ii, torch.int64, "ii")
    _need(jj, torch.int64, "jj")
    E = ii.shape[0]
    _, H, W = disps.shape
    coords = torch.empty((E, H, W, 2), dtype=torch.float32, device=poses.device)
    valid = torch.empty((E, H, W, 1), dtype=torch.float32, device=poses.device) if with_valid else None
    motn = None
    if target is not None:
        _need(target, torch.float32, "target")
        motn = torch.empty((E, 4, H, W), dtype=torch.float32, device=poses.device)
    with torch.cuda.device(poses.device):
        check(lib.droid_projective_transform(_ptr(poses), _ptr(disps), _ptr(intrinsics), _ptr(ii), _ptr(jj),
                                             E, H, W, _ptr(coords), _ptr(valid), _ptr(target), _ptr(motn),
                                             _stream(poses)), "projective_transform")
    if target is not None:
        return coords, valid, motn
    return coords, valid


def frame_distance(poses, disps, intrinsics, ii, jj, beta):
    """droid_kernels.cu:1438-1460 -> dist (E)."""
    _check_inputs(("poses", "disps", "intrinsics", "ii", "jj"), (poses, disps, intrinsics, ii, jj))
    E = ii.shape[0]
    _, H, W = disps.shape
    dist = torch.zeros((E,), dtype=torch.float32, device=poses.device)
    with torch.cuda.device(poses.device):
        check(lib.droid_frame_distance(_ptr(poses), _ptr(disps), _ptr(intrinsics), _ptr(ii), _ptr(jj),
                                       E, H, W, float(beta), _ptr(dist), _stream(poses)), "frame_distance")
    return dist


def proximity_select(d, t0, t1, t, rad, nms, thresh, ei, ej, stereo, n_cap):
    """add_proximity_factors' candidate walk on the device (include/droid_backends.h:
    droid_proximity_select): d (t-t0)*(t-t1) f32 distances, ei/ej int32 existing
    edges -> (pairs (n, 2) int32 device tensor in acceptance order)."""
    _check_inputs(("d", "ei", "ej"), (d, ei, ej))
    _need(d, torch.float32, "d")
    _need(ei, torch.int32, "ei")
    _need(ej, torch.int32, "ej")
    n = (t - t0) * (t - t1)
    if d.numel() != n or ei.numel() != ej.numel():
        raise RuntimeError("proximity_select: d must hold (t-t0)*(t-t1) distances, ei/ej the same length")
    dev = d.device
    ws = torch.empty((int(lib.droid_proximity_workspace(t0, t1, t)),), dtype=torch.uint8, device=dev)
    out = torch.empty((2, max(int(n_cap), 1)), dtype=torch.int32, device=dev)
    cnt = torch.zeros((1,), dtype=torch.int32, device=dev)
    with torch.cuda.device(dev):
        check(lib.droid_proximity_select(_ptr(d), t0, t1, t, int(rad), int(nms), float(thresh), _ptr(ei), _ptr(ej),
                                         ei.numel(), int(bool(stereo)), int(n_cap), _ptr(out[0]), _ptr(out[1]),
                                         _ptr(cnt), _ptr(ws), ws.numel(), _stream(d)), "proximity_select")
    k = int(cnt.item())
    return out[:, :k].t()


NORM_RELU, NORM_RES_RELU, NORM_ADD_RELU, NORM_ONLY = 0, 1, 2, 3


def instance_norm_act_f16(x, mode=NORM_RELU, res=None, out=None, eps=1e-5):
    """nn.InstanceNorm2d(affine=False) + the encoder's ReLU / residual add
    (include/droid_backends.h: droid_instance_norm_act_f16) on an NCHW fp16
    tensor in channels_last memory format; returns a tensor of the same kind."""
    if x.dtype != torch.float16 or x.dim() != 4 or not x.is_contiguous(memory_format=torch.channels_last):
        raise RuntimeError("instance_norm_act_f16: x must be a channels_last fp16 (N,C,H,W) tensor")
    N, C, H, W = x.shape
    if res is not None and (res.shape != x.shape or res.dtype != torch.float16 or
                            not res.is_contiguous(memory_format=torch.channels_last)):
        raise RuntimeError("instance_norm_act_f16: res must match x (channels_last fp16)")
    if out is None:
        out = torch.empty_like(x, memory_format=torch.channels_last)
    ws = torch.empty((int(lib.droid_instance_norm_workspace(N, H * W, C)),), dtype=torch.uint8, device=x.device)
    with torch.cuda.device(x.device):
        check(lib.droid_instance_norm_act_f16(_ptr(x), _ptr(res), _ptr(out), N, H * W, C, int(mode), float(eps),
                                              _ptr(ws), ws.numel(), _stream(x)), "instance_norm_act_f16")
    return out


def projmap(poses, disps, intrinsics, ii, jj):
    """droid_kernels.cu:1463-1488 -> [coords (E,H,W,3), valid (E,H,W,1)]."""
    _check_inputs(("poses", "disps", "intrinsics", "ii", "jj"), (poses, disps, intrinsics, ii, jj))
    E = ii.shape[0]
    _, H, W = disps.shape
    coords = torch.empty((E, H, W, 3), dtype=torch.float32, device=poses.device)
    valid = torch.empty((E, H, W, 1), dtype=torch.float32, device=poses.device)
    with torch.cuda.device(poses.device):
        check(lib.droid_projmap(_ptr(poses), _ptr(disps), _ptr(intrinsics), _ptr(ii), _ptr(jj), E, H, W,
                                _ptr(coords), _ptr(valid), _stream(poses)), "projmap")
    return [coords, valid]


def iproj(poses, disps, intrinsics):
    """droid_kernels.cu:1518-1541 -> points (N,H,W,3)."""
    _check_inputs(("poses", "disps", "intrinsics"), (poses, disps, intrinsics))
    N, H, W = disps.shape
    pts = torch.empty((N, H, W, 3), dtype=torch.float32, device=poses.device)
    with torch.cuda.device(poses.device):
        check(lib.droid_iproj(_ptr(poses), _ptr(disps), _ptr(intrinsics), N, H, W, _ptr(pts), _stream(poses)),
              "iproj")
    return pts


def depth_filter(poses, disps, intrinsics, ix, thresh):
    """droid_kernels.cu:1491-1515 -> counter (n,H,W)."""
    _check_inputs(("poses", "disps", "intrinsics", "ix", "thresh"), (poses, disps, intrinsics, ix, thresh))
    num, H, W = disps.shape
    n = ix.shape[0]
    counter = torch.empty((n, H, W), dtype=torch.float32, device=poses.device)
    with torch.cuda.device(poses.device):
        check(lib.droid_depth_filter(_ptr(poses), _ptr(disps), _ptr(intrinsics), _ptr(ix), _ptr(thresh),
                                     n, num, H, W, _ptr(counter), _stream(poses)), "depth_filter")
    return counter


# ---------------------------------------------------------------------------
# dense bundle adjustment
# ---------------------------------------------------------------------------
class BaPlan:
    """Host-built structure of one ba() call plus its device workspace.

    Built from host copies of ii/jj (no device sync), uploaded once; reused by
    every ba() with the same edge set.  `own` = (lo, hi) restricts the depth
    rows to poses owned by this rank (edge-sharded multi-GPU BA); `gedges` =
    (gii, gjj) is then the global edge list the pose order and the factor's
    tile structure derive from, identical on every rank."""

    def __init__(self, ii, jj, num_frames, ht, wd, t0, t1, eta_rows, motion_only, device, own=None, gedges=None):
        ii = np.ascontiguousarray(np.asarray(ii, dtype=np.int64))
        jj = np.ascontiguousarray(np.asarray(jj, dtype=np.int64))
        lo, hi = own if own is not None else (0, 2 ** 31 - 1)
        h = ctypes.c_void_p()
        if gedges is None:
            check(lib.droid_ba_plan_create(ii.ctypes.data_as(ctypes.c_void_p), jj.ctypes.data_as(ctypes.c_void_p),
                                           len(ii), int(num_frames), int(ht), int(wd), int(t0), int(t1),
                                           int(eta_rows), int(bool(motion_only)), int(lo), int(hi),
                                           ctypes.byref(h)), "ba plan")
        else:
            gii = np.ascontiguousarray(np.asarray(gedges[0], dtype=np.int64))
            gjj = np.ascontiguousarray(np.asarray(gedges[1], dtype=np.int64))
            check(lib.droid_ba_plan_create_sharded(
                ii.ctypes.data_as(ctypes.c_void_p), jj.ctypes.data_as(ctypes.c_void_p), len(ii),
                gii.ctypes.data_as(ctypes.c_void_p), gjj.ctypes.data_as(ctypes.c_void_p), len(gii),
                int(num_frames), int(ht), int(wd), int(t0), int(t1), int(eta_rows), int(bool(motion_only)),
                int(lo), int(hi), ctypes.byref(h)), "ba plan")
        self._h = h
        self.device = torch.device(device)
        self.t0, self.t1, self.motion_only = int(t0), int(t1), bool(motion_only)
        K, P, nblk, nbm = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(lib.droid_ba_plan_info(h, ctypes.byref(K), ctypes.byref(P), ctypes.byref(nblk), ctypes.byref(nbm)),
              "ba plan info")
        self.K, self.P, self.nblocks, self.nb_max = K.value, P.value, nblk.value, nbm.value
        kx = np.zeros(max(self.K, 1), dtype=np.int64)
        check(lib.droid_ba_plan_kx(h, kx.ctypes.data_as(ctypes.c_void_p)), "ba plan kx")
        self.kx = kx[:self.K]
        kind, nwide, ntasks = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        perm = np.zeros(max(self.P, 1), dtype=np.int32)
        check(lib.droid_ba_plan_order(h, ctypes.byref(kind), perm.ctypes.data_as(ctypes.c_void_p),
                                      ctypes.byref(nwide), ctypes.byref(ntasks)), "ba plan order")
        self.order = ("identity", "rcm", "mindeg", "nd")[kind.value]
        self.perm = perm[:self.P]
        self.num_wide, self.ntasks = nwide.value, ntasks.value
        nbytes = lib.droid_ba_plan_workspace_bytes(h)
        self.workspace = torch.empty((nbytes,), dtype=torch.uint8, device=self.device)
        off, sz, foff = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
        check(lib.droid_ba_plan_system_region(h, ctypes.byref(off), ctypes.byref(sz)), "ba plan region")
        check(lib.droid_ba_plan_flag_offset(h, ctypes.byref(foff)), "ba plan flag")
        self.n = 6 * self.P
        # the reduced system's input tiles (64x64 fp64, permuted lower triangle of
        # A - S, rhs as row n): the contiguous region a multi-GPU caller all-reduces
        self.system = self.workspace[off.value:off.value + sz.value].view(torch.float64).view(-1, 64, 64)
        self._flag = self.workspace[foff.value:foff.value + 8].view(torch.int32)   # [this solve, sticky]
        self._status = torch.zeros(2, dtype=torch.int32, pin_memory=True)
        self._status_evt = None
        self.name = "ba plan (%d edges, poses [%d, %d), %d depth frames%s)" % (
            len(ii), self.t0, self.t1, self.K, ", motion only" if self.motion_only else "")
        with torch.cuda.device(self.device):
            check(lib.droid_ba_plan_upload(h, _ptr(self.workspace), _stream(self.workspace)), "ba plan upload")

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and lib is not None:   # lib is None during interpreter teardown
            lib.droid_ba_plan_destroy(h)
            self._h = None

    def _record_status(self, flag=None):
        """queue a copy of the status words of the call just enqueued (checked
        lazily); `flag` = a device copy to read instead (the sharded BA's
        all-reduced status)."""
        self._status.copy_(self._flag if flag is None else flag, non_blocking=True)
        self._status_evt = torch.cuda.Event()
        self._status_evt.record(torch.cuda.current_stream(self.device))

    def check_status(self):
        """Raise if a solve of the last ba() call on this plan timed out (status
        bit 1 in this solve's or the sticky word): that solve left poses and
        disparities unchanged.  Waits for that call."""
        evt, self._status_evt = self._status_evt, None
        if evt is None:
            return
        evt.synchronize()
        st = int(self._status[0]) | int(self._status[1])
        if st & 4:
            raise RuntimeError("ba: the dataflow Cholesky found its state corrupt (a sync counter not zeroed "
                               "before the launch, or a task record outside the plan) in %s; that Gauss-Newton "
                               "step left poses and disparities unchanged" % self.name)
        if st & 2:
            raise RuntimeError("ba: the dataflow Cholesky timed out (dependency wait exceeded) in %s; that "
                               "Gauss-Newton step left poses and disparities unchanged" % self.name)

    def clear_status(self):
        """zero both status words (stream-ordered): the start of a staged ba call."""
        with torch.cuda.device(self.device):
            check(lib.droid_ba_plan_clear_status(self._h, _ptr(self.workspace), _stream(self.workspace)),
                  "ba clear_status")

    def build_system(self, poses, disps, intrinsics, disps_sens, targets, weights, eta):
        with torch.cuda.device(self.device):
            check(lib.droid_ba_build_system(self._h, _ptr(self.workspace), _ptr(poses), _ptr(disps),
                                            _ptr(intrinsics), _ptr(disps_sens), _ptr(targets), _ptr(weights),
                                            _ptr(eta), _stream(poses)), "ba build_system")

    def solve_update(self, poses, disps, intrinsics, disps_sens, targets, weights, eta, lm, ep, dx, dz):
        """one damped solve + back-substitution + retraction; the status words
        accumulate on the device (clear_status / status_words, no host wait)."""
        with torch.cuda.device(self.device):
            check(lib.droid_ba_solve_update(self._h, _ptr(self.workspace), _ptr(poses), _ptr(disps),
                                            _ptr(intrinsics), _ptr(disps_sens), _ptr(targets), _ptr(weights),
                                            _ptr(eta), float(lm), float(ep), _ptr(dx), _ptr(dz), _stream(poses)),
                  "ba solve_update")

    def solve_system(self, lm, ep, dx):
        """damping + Cholesky of the (all-reduced) system -> dx and status word 0."""
        with torch.cuda.device(self.device):
            check(lib.droid_ba_solve_system(self._h, _ptr(self.workspace), float(lm), float(ep), _ptr(dx),
                                            _stream(self.workspace)), "ba solve_system")

    def apply_update(self, poses, disps, intrinsics, disps_sens, targets, weights, eta, dx, dz):
        """back-substitution + retraction, skipped when status bit 1 is set."""
        with torch.cuda.device(self.device):
            check(lib.droid_ba_apply_update(self._h, _ptr(self.workspace), _ptr(poses), _ptr(disps),
                                            _ptr(intrinsics), _ptr(disps_sens), _ptr(targets), _ptr(weights),
                                            _ptr(eta), _ptr(dx), _ptr(dz), _stream(poses)), "ba apply_update")

    def ints_region(self):
        """the plan's packed int section in the workspace (a uint8 view; read-only
        after the upload - diagnostics compare it across calls)."""
        off, sz = ctypes.c_size_t(), ctypes.c_size_t()
        check(lib.droid_ba_plan_ints_region(self._h, ctypes.byref(off), ctypes.byref(sz)), "ba_plan_ints_region")
        return self.workspace[off.value:off.value + sz.value]

    def status_words(self):
        """the device status words (int32 [this solve, sticky]), a view."""
        return self._flag

    def run(self, poses, disps, intrinsics, disps_sens, targets, weights, eta, iterations, lm, ep):
        dx = torch.empty((self.P, 6), dtype=torch.float32, device=poses.device)
        dz = None if self.motion_only else torch.empty((self.K, disps.shape[1] * disps.shape[2]),
                                                      dtype=torch.float32, device=poses.device)
        if iterations <= 0:
            return dx.zero_(), dz
        capturing = torch.cuda.is_current_stream_capturing()
        if not capturing:
            self.check_status()
        with torch.cuda.device(poses.device):
            check(lib.droid_ba_run(self._h, _ptr(self.workspace), _ptr(poses), _ptr(disps), _ptr(intrinsics),
                                   _ptr(disps_sens), _ptr(targets), _ptr(weights), _ptr(eta), int(iterations),
                                   float(lm), float(ep), _ptr(dx), _ptr(dz), _stream(poses)), "ba")
            if not capturing:   # a captured run's status is recorded after each replay
                self._record_status()
        return dx, dz


_PLAN_CACHE = OrderedDict()
_PLAN_CACHE_SIZE = 8
_LAST_PLAN = [None]


def last_plan():
    """the plan of the last ba() call (a caller replaying a captured ba keeps it
    alive with the graph and records its status after each replay)."""
    return _LAST_PLAN[0]


def check_status():
    """Raise RuntimeError if a cached BA plan's last solve timed out (see
    BaPlan.check_status); waits for the solves still in flight."""
    for plan in list(_PLAN_CACHE.values()):
        plan.check_status()


def dense_spd_solve(A, b, lm=0.0, ep=0.0):
    """Damped dense SPD solve on the dataflow Cholesky (include/droid_backends.h:
    droid_chol_*): A (n,n) fp64 HIP tensor (lower triangle read), b (n) fp64 ->
    (dx (n) fp32, failed bool).  diag += ep + lm*diag first, as SparseBlock::solve."""
    _check_inputs(("A", "b"), (A, b))
    _need(A, torch.float64, "A")
    _need(b, torch.float64, "b")
    n = int(b.numel())
    if tuple(A.shape) != (n, n):
        raise RuntimeError("dense_spd_solve: A must be (n, n) with n = len(b)")
    h = ctypes.c_void_p()
    check(lib.droid_chol_plan_create(n, ctypes.byref(h)), "chol plan")
    try:
        nt, foff, ns, nsa = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(lib.droid_chol_plan_info(h, ctypes.byref(nt), ctypes.byref(foff), ctypes.byref(ns), ctypes.byref(nsa)),
              "chol plan info")
        ws = torch.zeros((lib.droid_ba_plan_workspace_bytes(h),), dtype=torch.uint8, device=A.device)
        dx = torch.empty(n, dtype=torch.float32, device=A.device)
        with torch.cuda.device(A.device):
            check(lib.droid_ba_plan_upload(h, _ptr(ws), _stream(A)), "chol upload")
            check(lib.droid_chol_set_system(h, _ptr(ws), _ptr(A), n, _ptr(b), _stream(A)), "chol set_system")
            check(lib.droid_chol_solve(h, _ptr(ws), float(lm), float(ep), _ptr(dx), _stream(A)), "chol solve")
        flag = int(ws[foff.value:foff.value + 4].view(torch.int32).item())
        if flag & 4:
            raise RuntimeError("dense_spd_solve: the dataflow Cholesky found its state corrupt")
        if flag & 2:
            raise RuntimeError("dense_spd_solve: the dataflow Cholesky timed out")
        return dx, bool(flag & 1)
    finally:
        lib.droid_ba_plan_destroy(h)


def get_plan(ii_host, jj_host, num_frames, ht, wd, t0, t1, eta_rows, motion_only, device, own=None, gedges=None):
    ii_host = np.ascontiguousarray(np.asarray(ii_host, dtype=np.int64))
    jj_host = np.ascontiguousarray(np.asarray(jj_host, dtype=np.int64))
    gkey = None if gedges is None else (np.asarray(gedges[0], np.int64).tobytes(),
                                        np.asarray(gedges[1], np.int64).tobytes())
    key = (ii_host.tobytes(), jj_host.tobytes(), int(num_frames), int(ht), int(wd), int(t0), int(t1),
           int(eta_rows), bool(motion_only), str(device), own, gkey)
    plan = _PLAN_CACHE.get(key)
    if plan is None:
        if torch.cuda.is_current_stream_capturing():
            # its workspace would live in the graph's pool and its upload be a
            # captured host copy: a plan must exist before a capture
            raise RuntimeError("ba: no plan for this edge set inside a HIP graph capture")
        plan = BaPlan(ii_host, jj_host, num_frames, ht, wd, t0, t1, eta_rows, motion_only, device, own, gedges)
        _PLAN_CACHE[key] = plan
        while len(_PLAN_CACHE) > _PLAN_CACHE_SIZE:
            # the evicted plan's last call: its failure names that plan, not this call
            _PLAN_CACHE.popitem(last=False)[1].check_status()
    else:
        _PLAN_CACHE.move_to_end(key)
    return plan


def ba(poses, disps, intrinsics, disps_sens, targets, weights, eta, ii, jj, t0, t1, iterations, lm, ep,
       motion_only, ii_host=None, jj_host=None):
    """droid.cpp:88-117 / ba_cuda: dense BA over poses [t0,t1) and the disparity
    maps of unique([t0,t1) U ii); mutates poses/disps in place and returns
    [dx (P,6), dz (K,H*W) or None if motion_only].

    ii_host/jj_host (numpy) are an optional extension: with them no device ->
    host copy of the edge list is needed (the reference copies it every call)."""
    _check_inputs(("targets", "weights", "poses", "disps", "intrinsics", "disps_sens", "ii", "jj", "eta"),
                  (targets, weights, poses, disps, intrinsics, disps_sens, ii, jj, eta))
    for n, t in (("poses", poses), ("disps", disps), ("intrinsics", intrinsics), ("disps_sens", disps_sens),
                 ("targets", targets), ("weights", weights), ("eta", eta)):
        _need(t, torch.float32, n)
    _need(ii, torch.int64, "ii")
    _need(jj, torch.int64, "jj")
    N, H, W = disps.shape
    E = ii.shape[0]
    if targets.shape != (E, 2, H, W) or weights.shape != (E, 2, H, W):
        raise RuntimeError("targets/weights must be (E,2,H,W)")
    # the reference-style call (no host copies of the edge list) synchronises
    # like the reference's ba (its D2H copies) and reports a failed solve at
    # once; with ii_host/jj_host the check is deferred to the next solve on the
    # plan (or droid_backends.check_status()) so update() never stalls the host
    sync = ii_host is None or jj_host is None
    if ii_host is None:
        ii_host = ii.cpu().numpy()
    if jj_host is None:
        jj_host = jj.cpu().numpy()
    eta_rows = eta.numel() // (H * W) if eta.numel() else 0
    plan = get_plan(ii_host, jj_host, N, H, W, int(t0), int(t1), eta_rows, motion_only, poses.device)
    _LAST_PLAN[0] = plan
    dx, dz = plan.run(poses, disps, intrinsics, disps_sens, targets, weights, eta, int(iterations), lm, ep)
    if sync:
        plan.check_status()
    return [dx, dz]
