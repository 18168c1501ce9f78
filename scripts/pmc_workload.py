"""Workload for the PMC traffic passes (run under rocprofv3 --pmc; see
scripts/pmc_traffic.sh): a 1 GiB device copy (calibration of the FETCH/WRITE
counters on a known byte count), then the C3 ZR gate conv as update() runs it
(over net | corr | flow, the inp term per source frame of bench.py's C3 edge
list: droid_conv_gru_pre_f16) and the C3 4-level
correlation lookup fused with corr_encoder[0] (corr_lookup_ce0 on the 8x8-tiled volume) and the
reference API's NCHW lookup on the same volume (corr_pyramid_lookup_tiled), then the
on-demand lookup (corr_alt_ce0) on the C3 graph's reprojected coordinates, each
launched 3 times on synthetic data."""
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.abspath(__file__)),
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "droid-slam_amd")]
import numpy as np
import torch

import droid_backends
from droid_mi355x.corr import CorrBlock
from droid_mi355x import synthetic
from droid_mi355x.fused import pack_conv

E, H, W = 2048, 48, 64
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)

x = torch.empty(1 << 29, dtype=torch.float16, device=dev).fill_(1.0)   # 1 GiB
y = torch.empty_like(x)
for _ in range(3):
    y.copy_(x)
torch.cuda.synchronize()
del x, y

t = lambda c: (torch.randn((E, H, W, c), generator=g, device=dev) * 0.5).half()
net, cf, ff = t(128), t(128), t(64)
ii_c3, _ = synthetic.c3_edges(256, E, rng=np.random.default_rng(1003))   # bench.py's C3 graph
uniq, inverse = np.unique(ii_c3, return_inverse=True)
pre = (torch.randn((len(uniq), H, W, 384), generator=g, device=dev) * 0.5).half()
pidx = torch.as_tensor(inverse.astype(np.int64), device=dev)
w = torch.randn((256, 320, 3, 3), generator=g, device=dev) * 0.02
wp = pack_conv(w, [128, 128, 64])
bias = torch.zeros(256, device=dev)
bb = torch.zeros((E, 256), device=dev)
z, rn = torch.empty_like(net), torch.empty_like(net)
for _ in range(3):
    droid_backends.conv_gru_pre_f16([(net, 0, 128), (cf, 0, 128), (ff, 0, 64)], wp, 256, bias, bb,
                                    droid_backends.EPI_GRU_ZR, pre, pidx, 0, h=net, zout=z, rnet=rn)
torch.cuda.synchronize()
del net, cf, ff, z, rn, pre

nf = 256
f = torch.randn((1, nf, 128, H, W), generator=g, device=dev).half()
rng = np.random.default_rng(0)
ii = torch.as_tensor(rng.integers(0, nf, E), device=dev)
jj = torch.as_tensor(rng.integers(0, nf, E), device=dev)
cb = CorrBlock(f[:, ii], f[:, jj], tiled=True)   # the layout FactorGraph builds for the fused operator
coords = torch.stack(torch.meshgrid(torch.arange(W, device=dev), torch.arange(H, device=dev), indexing="xy"), -1)
coords = (coords[None, None].float() + torch.randn((1, E, H, W, 2), generator=g, device=dev) * 3).contiguous()
w224 = (torch.randn((128, 224), generator=g, device=dev) * 0.05).half()
b128 = torch.zeros(128, device=dev)
c = coords.view(E, H, W, 2).contiguous()
with torch.no_grad():
    for _ in range(3):
        droid_backends.corr_lookup_ce0(cb.corr_pyramid, c, w224, b128, tiled_shapes=cb.level_shapes)
    torch.cuda.synchronize()
    for _ in range(3):   # the reference API's NCHW lookup on the same pool (corr_lookup_coop_kernel)
        droid_backends.corr_pyramid_lookup_tiled(cb.corr_pyramid, cb.level_shapes, c)
torch.cuda.synchronize()
del cb, f

from c3_alt_inputs import c3_alt_inputs  # noqa: E402
pyr, f1, f2, ca, wa, ba = c3_alt_inputs(dev)
for _ in range(3):
    droid_backends.corr_alt_ce0(pyr, f1, f2, ca, wa, ba)
torch.cuda.synchronize()
print("ok")
