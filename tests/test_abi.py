"""The C-ABI library loads on a GPU-less host and exports every entry point
include/droid_backends.h declares and none of include/droid_backends_testing.h
(the A/B and profiling builds export both); host-only plan construction works
(no device calls are made here)."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols(name="droid_backends.h"):
    text = open(os.path.join(ROOT, "include", name)).read()
    return sorted(set(re.findall(r"\b(droid_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_header():
    import droid_backends
    from droid_backends import _lib
    syms = _header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(_lib.lib, s), s
    assert set(syms) == set(_lib.EXPORTS)
    assert _lib.lib.droid_abi_version() == 1
    # the boundary a maintainer binds carries no testing hook:
    # those are declared apart and exported by the A/B and profiling builds only
    test_syms = _header_symbols("droid_backends_testing.h")
    assert len(test_syms) == 9 and not set(test_syms) & set(syms)
    assert set(test_syms) == set(_lib.TEST_EXPORTS)
    for s in test_syms:
        assert not hasattr(_lib.lib, s), s
    assert not _lib.HAS_TESTING_HOOKS
    with pytest.raises(RuntimeError, match="testing hook"):
        droid_backends.alt_set_variant(2)
    for sub in ("ab", "prof"):
        path = os.path.join(ROOT, "droid-slam_amd", "lib", sub, "libdroid_hip.so")
        if os.path.exists(path):
            other = ctypes.CDLL(path)
            for s in syms + test_syms:
                assert hasattr(other, s), (sub, s)
    for name in ("ba", "frame_distance", "projmap", "depth_filter", "iproj", "altcorr_forward",
                 "altcorr_backward", "corr_index_forward", "corr_index_backward"):
        assert callable(getattr(droid_backends, name))


def test_product_library_takes_no_kernel_choice_from_env(monkeypatch):
    """the product library is not the A/B build, ships only
    the default kernels (the dropped variants answer 'unsupported') and reads
    no DROID_* experiment knob; the A/B library (make ab) exports the same
    entry points and reports its build."""
    import ctypes as ct
    from droid_backends import _lib
    assert _lib.lib.droid_build_info() == 0
    assert not hasattr(_lib.lib, "droid_alt_set_variant")   # no variant setter at all
    # an order forced through the ABI, not the environment: DROID_BA_ORDER is ignored
    monkeypatch.setenv("DROID_BA_ORDER", "rcm")
    from droid_mi355x import synthetic
    ii, jj = synthetic.c3_edges(num_kf=64, num_edges=512, rng=np.random.default_rng(5))
    st, h = _plan(ii, jj, N=64, t0=1, t1=64)
    assert st == 0
    kind, nwide, ntasks = ct.c_int(), ct.c_int(), ct.c_int()
    perm = np.zeros(63, np.int32)
    assert _lib.lib.droid_ba_plan_order(h, ct.byref(kind), perm.ctypes.data_as(ct.c_void_p), ct.byref(nwide),
                                        ct.byref(ntasks)) == 0
    _lib.lib.droid_ba_plan_destroy(h)
    assert kind.value == 0   # the plan's own choice on this dense-at-tile-level graph: identity
    prev = _lib.lib.droid_ba_set_order(1)
    try:
        st, h = _plan(ii, jj, N=64, t0=1, t1=64)
        assert st == 0
        assert _lib.lib.droid_ba_plan_order(h, ct.byref(kind), perm.ctypes.data_as(ct.c_void_p), ct.byref(nwide),
                                            ct.byref(ntasks)) == 0
        _lib.lib.droid_ba_plan_destroy(h)
        assert kind.value == 1
    finally:
        _lib.lib.droid_ba_set_order(prev)
    ab = os.path.join(ROOT, "droid-slam_amd", "lib", "ab", "libdroid_hip.so")
    if os.path.exists(ab):
        lab = ct.CDLL(ab)
        assert lab.droid_build_info() & 1
        for s in _header_symbols():
            assert hasattr(lab, s), s
        assert all(lab.droid_alt_set_variant(v) == 0 for v in (1, 3, 4, 5, 6, 2))   # the dropped variants live here


def _plan(ii, jj, N=6, H=4, W=6, t0=1, t1=5, eta_rows=None, motion_only=0, own=(0, 2 ** 31 - 1)):
    from droid_backends._lib import lib
    ii = np.ascontiguousarray(ii, dtype=np.int64)
    jj = np.ascontiguousarray(jj, dtype=np.int64)
    if eta_rows is None:
        eta_rows = len(np.unique(np.concatenate([np.arange(t0, t1), ii])))
    h = ctypes.c_void_p()
    st = lib.droid_ba_plan_create(ii.ctypes.data_as(ctypes.c_void_p), jj.ctypes.data_as(ctypes.c_void_p),
                                  len(ii), N, H, W, t0, t1, eta_rows, motion_only, own[0], own[1], ctypes.byref(h))
    return st, h


def test_plan_structure_host_only():
    from droid_backends._lib import lib
    ii = np.array([1, 2, 2, 3, 0, 4], np.int64)
    jj = np.array([2, 1, 3, 2, 1, 3], np.int64)
    st, h = _plan(ii, jj)
    assert st == 0, lib.droid_last_error()
    K, P, nb, nbm = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    assert lib.droid_ba_plan_info(h, ctypes.byref(K), ctypes.byref(P), ctypes.byref(nb), ctypes.byref(nbm)) == 0
    assert (K.value, P.value) == (5, 4)        # kx = {0,1,2,3,4}, poses [1,5)
    kx = np.zeros(5, np.int64)
    lib.droid_ba_plan_kx(h, kx.ctypes.data_as(ctypes.c_void_p))
    np.testing.assert_array_equal(kx, [0, 1, 2, 3, 4])
    assert lib.droid_ba_plan_workspace_bytes(h) > 0
    lib.droid_ba_plan_destroy(h)


def test_plan_errors_like_reference():
    from droid_backends._lib import lib
    ii = np.array([1, 2], np.int64)
    jj = np.array([2, 1], np.int64)
    st, _ = _plan(ii, jj, eta_rows=7)          # eta rows != len(kx): reference raises a size mismatch
    assert st != 0 and b"eta" in lib.droid_last_error()
    st, _ = _plan(ii, np.array([2, 9], np.int64))
    assert st != 0 and b"out of range" in lib.droid_last_error()
    st, _ = _plan(ii, jj, t0=3, t1=3)
    assert st != 0


def test_python_layer_rejects_host_tensors():
    import torch
    import droid_backends
    vol = torch.zeros(1, 2, 2, 4, 4)
    coords = torch.zeros(1, 2, 2, 2)
    with pytest.raises(RuntimeError, match="HIP device"):
        droid_backends.corr_index_forward(vol, coords, 3)
    with pytest.raises(RuntimeError, match="contiguous"):
        droid_backends.corr_index_forward(vol.transpose(3, 4), coords, 3)


def test_tile8_round_trip_host_only():
    """corr.tile8 / untile8 (the 8x8-tiled volume layout of
    droid_corr_lookup_ce0_tiled) on CPU tensors: element (y, x) lands at
    ((y//8)*(W2//8) + x//8)*64 + (y%8)*8 + x%8 of its slice, padded rows zero."""
    import torch
    from droid_mi355x.corr import tile8, untile8
    for H2, W2 in [(48, 64), (12, 16), (6, 8), (3, 8)]:
        lv = torch.randn(3, 2, 5, H2, W2).half()
        t = tile8(lv, chunk=2)
        H2p = (H2 + 7) // 8 * 8
        assert t.shape == (3, 2, 5, H2p // 8, W2 // 8, 8, 8)
        flat = t.reshape(3, 2, 5, -1)
        for y, x in [(0, 0), (H2 - 1, W2 - 1), (H2 // 2, 3), (min(7, H2 - 1), 7)]:
            k = ((y // 8) * (W2 // 8) + x // 8) * 64 + (y % 8) * 8 + x % 8
            assert torch.equal(flat[..., k], lv[..., y, x])
        if H2p != H2:
            assert not t.reshape(3, 2, 5, H2p // 8, W2 // 8, 8, 8)[:, :, :, -1, :, H2 % 8:, :].any()
        assert torch.equal(untile8(t, H2, W2), lv)


def test_c4_stereo_edges_host_only():
    """bench.py --config C4 graph: one (i, i) edge per keyframe, +-1..+-3
    temporal edges, bidirectional loop edges, no duplicates (~1k edges)."""
    from droid_mi355x import synthetic
    ii, jj = synthetic.c4_edges(128)
    assert (ii == jj).sum() == 128
    pairs = set(zip(ii.tolist(), jj.tolist()))
    assert len(pairs) == len(ii) and 900 < len(ii) < 1100
    assert all((j, i) in pairs for i, j in pairs)
    d = np.abs(ii - jj)
    assert ((d >= 1) & (d <= 3)).sum() == 2 * (127 + 126 + 125)


def test_conv_side_operands_are_validated_before_launch():
    """The conv entry points read bias / bbias / the GRU maps through raw
    pointers: a wrong dtype (e.g. an fp16 bias produced inside an autocast
    region) is refused on the host before anything is launched."""
    import torch
    import droid_backends
    x = torch.zeros((1, 8, 16, 64), dtype=torch.float16)
    wp = torch.zeros((128, 9, 64), dtype=torch.float16)
    out = torch.zeros((1, 8, 16, 128), dtype=torch.float16)
    for kw in (dict(bias=torch.zeros(128, dtype=torch.float16)),          # fp16 bias
               dict(bias=torch.zeros(64)),                                 # too short
               dict(bias=torch.zeros(128), bbias=torch.zeros((1, 128), dtype=torch.float16)),
               dict(bias=torch.zeros(128), h=torch.zeros((1, 8, 16, 128)))):   # fp32 hidden map
        with pytest.raises(RuntimeError):
            droid_backends.conv_nhwc_f16([(x, 0, 64)], wp, 128, 3, out=out, **kw)
