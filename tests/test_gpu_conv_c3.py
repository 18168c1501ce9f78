"""The update operator's gate convs at the benchmark's shape (C3/C4: 48x64
feature maps, thousands of edges), on BOTH W=64 tiles the library can pick.

The band-conv entry points route the ConvGRU z|r gate conv to the two-
workgroups-per-CU tile (conv_band2_kernel) on small grids and to the 8-wave
band tile (conv_band_kernel<256,256,..,ZRP>) above 8 x 256 tiles of 256
pixels, i.e. above 170 edges at 48x64 - the C3 bench path; the q gate takes
conv_band2_kernel at every size since round 4 (its 8-wave tile,
conv_band_kernel<384,128,..,QP>, stays reachable with policy 0).
droid_conv_set_tile (a testing hook: the A/B library) forces either tile per
call, so both are compared with torch fp32 in one process here, and the
product library's default with them (reference: modules/gru.py:19-32,
droid_net.py:111-143)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from fill import det_fill

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _maxdiff(a, b):
    return float((a.float() - b.float()).abs().max())


def _conv_ref(xs, w, bias, bb):
    xin = torch.cat([x.float() for x in xs], -1).permute(0, 3, 1, 2)
    return (F.conv2d(xin, w.half().float(), bias, padding=1) + bb[:, :, None, None]).permute(0, 2, 3, 1)


@pytest.fixture
def tiles(ab_backends):
    """the A/B library's module instance, its tile policy restored afterwards
    (droid_conv_set_tile is a testing hook: include/droid_backends_testing.h)"""
    prev = ab_backends.conv_set_tile(-1)
    yield ab_backends
    ab_backends.conv_set_tile(prev)


def _gates(B, H, W, F_, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    mk = lambda n, c: torch.randn((n, H, W, c), generator=g, device=DEV).half()
    idx = torch.arange(B, device=DEV) * F_ // B          # B/F_ consecutive edges per source frame, as in C3
    inp_f = mk(F_, 128)
    h = torch.tanh(mk(B, 128).float()).half()
    cf, ff = mk(B, 128), mk(B, 64)
    wzr = torch.randn((256, 448, 3, 3), generator=g, device=DEV) / (448 * 9) ** 0.5
    wq = torch.randn((128, 448, 3, 3), generator=g, device=DEV) / (448 * 9) ** 0.5
    bzr, bq = torch.randn(256, generator=g, device=DEV), torch.randn(128, generator=g, device=DEV)
    bbzr, bbq = torch.randn((B, 256), generator=g, device=DEV), torch.randn((B, 128), generator=g, device=DEV)
    return dict(idx=idx, inp_f=inp_f, h=h, cf=cf, ff=ff, wzr=wzr, wq=wq, bzr=bzr, bq=bq, bbzr=bbzr, bbq=bbq)


def _pre_term(t, H, W):
    """the per-source-frame gate term conv3x3(inp_frames) (a plain conv: its own
    tile choice, so it is computed once and shared by the runs compared)."""
    import droid_backends   # the product library
    from droid_mi355x.fused import pack_conv
    pre = torch.empty((t["inp_f"].shape[0], H, W, 384), dtype=torch.float16, device=DEV)
    droid_backends.conv_nhwc_f16([(t["inp_f"], 0, 128)],
                                 pack_conv(torch.cat([t["wzr"][:, 128:256], t["wq"][:, 128:256]]), [128]),
                                 384, 3, out=pre)
    return pre


def _run_gates(t, H, W, pre, droid_backends):
    """z, r*h and the GRU update through droid_conv_gru_pre_f16 (per-frame inp
    term) of the given module instance (the product or the A/B library)."""
    from droid_backends import EPI_GRU_Q, EPI_GRU_ZR
    from droid_mi355x.fused import pack_conv
    B = t["h"].shape[0]
    keep = lambda w: torch.cat([w[:, :128], w[:, 256:]], 1)
    z = torch.empty((B, H, W, 128), dtype=torch.float16, device=DEV)
    rn = torch.empty_like(z)
    droid_backends.conv_gru_pre_f16([(t["h"], 0, 128), (t["cf"], 0, 128), (t["ff"], 0, 64)],
                                    pack_conv(keep(t["wzr"]), [128, 128, 64]), 256, t["bzr"], t["bbzr"],
                                    EPI_GRU_ZR, pre, t["idx"], 0, h=t["h"], zout=z, rnet=rn)
    hn = torch.empty_like(z)
    droid_backends.conv_gru_pre_f16([(rn, 0, 128), (t["cf"], 0, 128), (t["ff"], 0, 64)],
                                    pack_conv(keep(t["wq"]), [128, 128, 64]), 128, t["bq"], t["bbq"],
                                    EPI_GRU_Q, pre, t["idx"], 256, h=t["h"], z=z, out=hn)
    torch.cuda.synchronize()
    return z, rn, hn


@pytest.mark.parametrize("B", [192, 256])
def test_conv_gru_gates_c3_shape_both_tiles(B, tiles):
    """z|r and q gates at 48x64 over B >= 192 edges (above the band2 threshold)
    on the 8-wave band tiles (policy 0, and the default, which must pick them
    here: bitwise the same outputs) and on the two-workgroup tile (policy 1),
    each vs torch fp32 over the full 448 input channels.  The tiles are forced
    on the A/B library (a testing hook); the product library runs the default
    and must give its bytes."""
    import droid_backends as product
    droid_backends = tiles
    from droid_backends import EPI_GRU_Q, EPI_GRU_ZR
    H, W = 48, 64
    t = _gates(B, H, W, B // 8, seed=31)
    xs = [t["h"], t["inp_f"][t["idx"]].contiguous(), t["cf"], t["ff"]]
    gates = torch.sigmoid(_conv_ref(xs, t["wzr"], t["bzr"], t["bbzr"]))
    pre = _pre_term(t, H, W)
    outs = {}
    # (mode, z|r tile, q tile): the default runs z|r on the 8-wave tile and q on
    # the two-workgroup tile at this size
    for mode, tzr, tq in ((0, 0, 0), (1, 1, 1), (-1, 0, 1)):
        droid_backends.conv_set_tile(mode)
        # the kernel each gate conv is routed to (the rocprof trace of this test,
        # profiles/r04/, shows conv_band_kernel<256,256,..,6,8> / <384,128,..,7,8>)
        assert droid_backends.conv_gate_tile(EPI_GRU_ZR, B, H, W) == tzr, mode
        assert droid_backends.conv_gate_tile(EPI_GRU_Q, B, H, W) == tq, mode
        outs[mode] = _run_gates(t, H, W, pre, droid_backends)
    for mode in (0, 1, -1):
        z, rn, hn = outs[mode]
        assert _maxdiff(z, gates[..., :128]) < 3e-3, mode
        assert _maxdiff(rn, gates[..., 128:] * t["h"].float()) < 3e-3, mode
    del gates
    for mode in (0, 1, -1):
        z, rn, hn = outs[mode]
        q = torch.tanh(_conv_ref([rn] + xs[1:], t["wq"], t["bq"], t["bbq"]))
        ref = (1 - z.float()) * t["h"].float() + z.float() * q
        assert _maxdiff(hn, ref) < 4e-3, mode
        del q, ref
    # the default's z|r is policy 0's bit for bit; the two tiles sum the same
    # MFMA products in a different order (fp32), so they agree to an fp16 ulp
    # or two of the gates
    for a, b in zip(outs[-1][:2], outs[0][:2]):
        assert torch.equal(a, b)
    for a, b in zip(_run_gates(t, H, W, pre, product), outs[-1]):
        assert torch.equal(a, b)
    for a, b in zip(outs[1], outs[0]):
        assert _maxdiff(a, b) < 4e-3


def test_conv_gru_gates_small_grid_default_is_band2(tiles):
    """Below the threshold (96 edges, C2) the default takes the two-workgroup
    tile (policy forced on the A/B library; the product's default: the same bytes)."""
    import droid_backends as product
    droid_backends = tiles
    from droid_backends import EPI_GRU_Q, EPI_GRU_ZR
    H, W, B = 48, 64, 96
    t = _gates(B, H, W, 12, seed=37)
    pre = _pre_term(t, H, W)
    outs = {}
    for mode in (1, -1):
        droid_backends.conv_set_tile(mode)
        assert droid_backends.conv_gate_tile(EPI_GRU_ZR, B, H, W) == 1
        assert droid_backends.conv_gate_tile(EPI_GRU_Q, B, H, W) == 1
        outs[mode] = _run_gates(t, H, W, pre, droid_backends)
    for a, b in zip(outs[-1], outs[1]):
        assert torch.equal(a, b)
    for a, b in zip(_run_gates(t, H, W, pre, product), outs[-1]):
        assert torch.equal(a, b)


def test_fused_update_matches_reference_module_c3_edges(tiles):
    """FusedUpdateModule vs the pinned UpdateModule (update_module.npz) at the
    bench shape: 256 edges of 48x64 over 32 source frames, 8 edges per frame -
    the product's default policy runs the gate convs on the 8-wave band tiles
    here (the other tile at this shape: test_conv_gru_gates_c3_shape_both_tiles)."""
    from droid_mi355x.fused import FusedUpdateModule, edge_segments
    from droid_mi355x.update import UpdateModule
    E, H, W, NF = 256, 48, 64, 32
    assert tiles.conv_gate_tile(tiles.EPI_GRU_ZR, E, H, W) == 0   # the default policy (same code as the product)
    m = UpdateModule().to(DEV).eval()
    det_fill(m)
    f = FusedUpdateModule(m)
    g = torch.Generator(device=DEV).manual_seed(23)
    ii = torch.arange(E, device=DEV) // (E // NF)
    jj = (ii + 1 + torch.randint(0, NF - 1, (E,), generator=g, device=DEV)) % NF
    net = torch.tanh(torch.randn((1, E, 128, H, W), generator=g, device=DEV)).half()
    inp_f = torch.relu(torch.randn((NF, 128, H, W), generator=g, device=DEV)).half()
    corr = (2 * torch.randn((1, E, 196, H, W), generator=g, device=DEV)).half()
    flow = (4 * torch.randn((1, E, 4, H, W), generator=g, device=DEV)).clamp(-64, 64)
    nhwc = lambda t: t[0].permute(0, 2, 3, 1).contiguous()
    with torch.no_grad():
        rn, rd, rw, re, _ = m(net.float(), inp_f[ii][None].float(), corr.float(), flow, ii, jj)
        rn = nhwc(rn)
        c200 = torch.zeros((E, H, W, 200), dtype=torch.float16, device=DEV)
        c200[..., :196] = nhwc(corr)
        del corr
        uq, inv = torch.unique(ii, return_inverse=True)
        ptr, idx = edge_segments(inv.cpu().numpy(), len(uq))
        segs = (torch.as_tensor(ptr, device=DEV), torch.as_tensor(idx, device=DEV))
        inp_frames = inp_f.permute(0, 2, 3, 1).contiguous()
        fn, fd, fw, fe = f(nhwc(net), None, c200, flow[0], inv, len(uq), segments=segs, inp_frames=inp_frames)
        torch.cuda.synchronize()
    assert _maxdiff(fn, rn) < 1.5e-2
    assert _maxdiff(fd, rd) < 3e-2 * max(1.0, float(rd.abs().max()))
    assert _maxdiff(fw, rw) < 1.5e-2
    assert _maxdiff(fe, re) < 1e-3 + 2e-2 * float(re.abs().max())
    assert np.isfinite(float(fn.float().abs().max()))
