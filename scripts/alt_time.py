"""Median launch time of corr_alt_ce0 on the C3 bench coordinates (2048 edges,
48x64) for the library in $DROID_HIP_LIB (scripts/alt_ablate.sh variants), and
corr_alt2_kernel's walk: edge order vs edges grouped by target frame, times the
XCD chunk size (droid_alt_set_chunk)."""
import os
# its knobs are testing hooks (include/droid_backends_testing.h): the A/B library by default
os.environ.setdefault("DROID_HIP_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                                    "droid-slam_amd", "lib", "ab", "libdroid_hip.so"))
import sys

sys.path[:0] = [os.path.dirname(os.path.abspath(__file__)), os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."),
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "droid-slam_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import droid_backends  # noqa: E402
from c3_alt_inputs import c3_alt_inputs  # noqa: E402

dev = torch.device("cuda:0")
pyr, f1, f2, c, w, b = c3_alt_inputs(dev)


def timed(**kw):
    ts = []
    for it in range(8):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        o = droid_backends.corr_alt_ce0(pyr, f1, f2, c, w, b, **kw)
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    return o, float(np.median(ts[2:])), min(ts)


outs = {}
# droid_alt_set_variant: 2 = the product; the A/B build (DROID_HIP_LIB=.../lib/ab/libdroid_hip.so)
# adds 1 = the one-workgroup kernel, 4 = the round-4 corr_alt2_kernel, 6 = its pixel-major C
# alone, 5 = its row-K lookup tile alone, 3 = V3
variants = (1, 4, 6, 5, 3, 2) if droid_backends.AB_BUILD else (2,)
for variant in variants:
    droid_backends.alt_set_variant(variant)
    outs[variant], med, mn = timed()
    print("%s variant %d: median %.3f ms (min %.3f)" % (os.environ.get("DROID_HIP_LIB", "default"), variant, med, mn))
if droid_backends.AB_BUILD:
    print("C3 outputs bitwise equal (1, 4, 6):", bool(torch.equal(outs[1], outs[4]) and torch.equal(outs[1], outs[6])))
    print("C3 outputs bitwise equal (2, 3, 5):", bool(torch.equal(outs[2], outs[3]) and torch.equal(outs[2], outs[5])))
    d = (outs[2].float() - outs[4].float()).abs()
    print("product vs round-4 V2: max diff %.3g of scale %.3g, identical fraction %.4f" % (
        float(d.max()), float(outs[4].float().abs().max()), float((d == 0).float().mean())))
droid_backends.alt_set_variant(2)
if "--quick" in sys.argv:   # the variants only (PMC passes: scripts/pmc_alt.sh)
    sys.exit(0)
order = torch.argsort(f2.long(), stable=True).to(torch.int32)
for chunk in (0, 1, 2, 4, 8, 16, 32):
    droid_backends.alt_set_chunk(chunk)
    for name, o_ in (("edge order", None), ("by target frame", order)):
        o, med, mn = timed(order=o_)
        print("variant 2, chunk %2d edges, %-15s: median %.3f ms (min %.3f) bitwise %s" % (
            chunk, name, med, mn, bool(torch.equal(o, outs[2]))))
droid_backends.alt_set_chunk(0)
