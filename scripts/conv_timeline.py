"""Per-workgroup timeline of the band conv kernel (droid_conv_set_profile):
prologue (entry -> first stage's operands landed), main loop, epilogue, and the
gap between consecutive workgroups on the same CU, in shader clocks.

usage: python scripts/conv_timeline.py [edges] [zr|q|zrp|qp|ce2|dw|dwh]
(zrp / qp: the gates with the inp term per source frame, droid_conv_gru_pre_f16)
(runs on the profiling build: make -C droid-slam_amd/csrc prof)"""
import os
import sys

_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "droid-slam_amd", "lib", "prof", "libdroid_hip.so")
os.environ.setdefault("DROID_HIP_LIB", _LIB)

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "droid-slam_amd"))
import ctypes

import numpy as np
import torch

import droid_backends
from droid_backends._lib import lib
from droid_mi355x.fused import pack_conv

E = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
which = sys.argv[2] if len(sys.argv) > 2 else "zr"
H, W = 48, 64
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
t = lambda c: (torch.randn((E, H, W, c), generator=g, device=dev) * 0.5).half()
net, inp, cf, ff = t(128), t(128), t(128), t(64)
srcs4 = [(net, 0, 128), (inp, 0, 128), (cf, 0, 128), (ff, 0, 64)]
srcs3 = [(net, 0, 128), (cf, 0, 128), (ff, 0, 64)]
cfg = {"zr": (srcs4, 256), "q": (srcs4, 128), "ce2": ([(net, 0, 128)], 128), "dw": ([(net, 0, 128)], 256),
       "dwh": ([(net, 0, 128)], 256), "zrp": (srcs3, 256), "qp": (srcs3, 128)}[which]
srcs, cout = cfg
cin = sum(c for _, _, c in srcs)
w = torch.randn((cout, cin, 3, 3), generator=g, device=dev) * 0.02
wp = pack_conv(w, [c for _, _, c in srcs])
bias = torch.zeros(cout, device=dev)
out = torch.empty((E, H, W, cout), dtype=torch.float16, device=dev)
if which == "dwh":   # delta.0 || weight.0 with both heads fused (EPI_DWHEAD)
    from droid_mi355x.fused import pack_head_taps
    hw = pack_head_taps(torch.randn((4, 256, 3, 3), generator=g, device=dev) * 0.02)
    head = torch.zeros((E, H, W, 4), device=dev)
    run = lambda: droid_backends.conv_dw_head_f16(srcs, wp, bias, hw, head)
elif which in ("zrp", "qp"):   # 8 edges per source frame, as in the C3 graph
    pre = t(384)[: E // 8].contiguous()
    pidx = torch.arange(E, device=dev) // 8
    if os.environ.get("TL_PIDX0"):   # experiment: every edge reads frame 0's pre map (L2-resident)
        pidx.zero_()
    zo, rn = t(128), t(128)
    epi = droid_backends.EPI_GRU_ZR if which == "zrp" else droid_backends.EPI_GRU_Q
    kw = dict(zout=zo, rnet=rn) if which == "zrp" else dict(z=zo, out=out)
    run = lambda: droid_backends.conv_gru_pre_f16(srcs, wp, cout, bias, None, epi, pre, pidx,
                                                  0 if which == "zrp" else 256, h=net, **kw)
else:
    run = lambda: droid_backends.conv_nhwc_f16(srcs, wp, cout, 3, bias=bias, act=1, out=out)
if os.environ.get("TL_TILE"):   # tile policy (droid_conv_set_tile): 0 8-wave, 2 the 4-wave z|r tile
    droid_backends.conv_set_tile(int(os.environ["TL_TILE"]))
for _ in range(3):
    run()
torch.cuda.synchronize()
warm = float(os.environ.get("TL_WARM_S", "0"))   # back-to-back launches first (MI355X_MICROARCH.md, DVFS item 6)
if warm > 0:
    import time
    t_end = time.time() + warm
    nw = 0
    while time.time() < t_end:
        for _ in range(8):
            run()
        torch.cuda.synchronize()
        nw += 8
    print("%d back-to-back launches over %.1f s before the profiled one" % (nw, warm))
tile = {256: 256, 128: 384}[cout]
nwg = E * H * W // tile
prof = torch.zeros(nwg * 12, dtype=torch.int64, device=dev)
lib.droid_conv_set_profile(ctypes.c_void_p(prof.data_ptr()))
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
run()
e.record()
torch.cuda.synchronize()
lib.droid_conv_set_profile(None)
ms = s.elapsed_time(e)
p = prof.view(nwg, 12).cpu().numpy()
assert (p[:, 1] > 0).all(), "profile not written (kernel not the band kernel?)"
hw = p[:, 0]
cu = ((hw >> 32) & 15) * 256 + ((hw >> 8) & 0xff)   # XCC id, then SE_ID[15:13] | SH_ID[12] | CU_ID[11:8]
pro, loop, epi, drain = p[:, 2] - p[:, 1], p[:, 3] - p[:, 2], p[:, 4] - p[:, 3], p[:, 5] - p[:, 4]
gaps = []
for c in np.unique(cu):
    q = p[cu == c]
    q = q[np.argsort(q[:, 1])]
    gaps.extend((q[1:, 1] - np.maximum(q[:-1, 5], q[:-1, 9])).tolist())
gaps = np.asarray(gaps)
tot = pro + loop + epi + drain
span_clk = np.median(tot) * nwg / len(np.unique(cu)) + np.median(gaps) * (nwg / len(np.unique(cu)) - 1)
print("%s: %d edges, %d workgroups on %d CUs, %.3f ms (HIP events)" % (which, E, nwg, len(np.unique(cu)), ms))
for name, v in (("prologue", pro), ("main loop", loop), ("epilogue issue", epi), ("store drain", drain),
                ("gap to next WG", gaps)):
    print("  %-15s median %8.0f clk  mean %8.0f  p90 %8.0f  (%.1f %% of a WG's median cycle)"
          % (name, np.median(v), v.mean(), np.percentile(v, 90), 100 * np.median(v) / (np.median(tot) + np.median(gaps))))
stages = (cin // 64 if cin % 64 == 0 else cin // 64 + 1) * 9
tn = 256 if cout == 256 else 128
floor = 64 * (tile // 64) * (tn // 32)   # 2 waves/SIMD x 2*FM*FN MFMAs x 16 clk
if which == "dwh" and (p[:, 6] > 0).all():   # dwhead_epilogue sub-phases
    for name, v in (("  pass 1 + head weights", p[:, 6] - p[:, 3]), ("  head GEMM (wave 0)", p[:, 7] - p[:, 6]),
                    ("  GEMM barrier + Y stores", p[:, 8] - p[:, 7]), ("  tap sums + atomics", p[:, 4] - p[:, 8]),
                    ("last wave drained after wave 0", p[:, 9] - p[:, 5])):
        print("  %-30s median %8.0f clk  p90 %8.0f" % (name, np.median(v), np.percentile(v, 90)))
elif (p[:, 6] > 0).all():   # band_epilogue sub-phases (wave 0) and the last wave's drain
    for name, v in (("  pass 1 (acc -> LDS)", p[:, 6] - p[:, 3]), ("  pass-2 load issue", p[:, 7] - p[:, 6]),
                    ("  staging barrier", p[:, 8] - p[:, 7]), ("  pass 2 + stores", p[:, 4] - p[:, 8]),
                    ("last wave drained after wave 0", p[:, 9] - p[:, 5])):
        print("  %-30s median %8.0f clk  p90 %8.0f" % (name, np.median(v), np.percentile(v, 90)))
print("  main loop per stage: %.0f clk (%d stages); MFMA-only floor %d clk/stage" % (np.median(loop) / stages, stages,
                                                                                     floor))
print("  implied clock: %.2f GHz (median WG cycle x WGs per CU / kernel time)" % (span_clk / (ms * 1e-3) / 1e9))
if (p[:, 11] > p[:, 10]).all():   # in-kernel clock over the main loop: s_memtime ticks per s_memrealtime (100 MHz)
    clk = (p[:, 3] - p[:, 2]) / ((p[:, 11] - p[:, 10]) / 100e6) / 1e9
    flops = {"zr": 2 * 256 * 448 * 9, "zrp": 2 * 256 * 320 * 9, "q": 2 * 128 * 448 * 9, "qp": 2 * 128 * 320 * 9,
             "ce2": 2 * 128 * 128 * 9, "dw": 2 * 256 * 128 * 9, "dwh": 2 * 256 * 128 * 9}[which] * E * H * W
    print("  in-kernel clock over the main loop: median %.3f GHz (p10 %.3f, p90 %.3f); %.1f TFLOP/s over the launch "
          "= %.3f of the 2.5 PF spec, %.3f of the fp16 MFMA peak at that clock"
          % (np.median(clk), np.percentile(clk, 10), np.percentile(clk, 90), flops / (ms * 1e-3) / 1e12,
             flops / (ms * 1e-3) / 2.5e15, flops / (ms * 1e-3) / (2.5e15 * np.median(clk) / 2.4)))
