"""Turn the FETCH_SIZE / WRITE_SIZE passes of scripts/pmc_workload.py into
profiles/pmc_conv_zr.json and profiles/pmc_corr_lookup.json.  The counters'
unit is calibrated on the 1 GiB device copy (the first three
__amd_rocclr_copyBuffer launches: read 1 GiB, write 1 GiB) in the same
process: FETCH_SIZE reads 0.5 GiB in KB there (the gfx950 half-the-bytes quirk
for 16-B-per-lane streaming reads, MI355X_MICROARCH.md §HBM), WRITE_SIZE 1 GiB.
The same factors are applied to the measured kernels (both read 16 B per
lane; the lookup's row windows are unaligned gathers, so its fetch figure
carries the guide's "uncalibrated width" caveat)."""
import csv
import glob
import json
import os
import sys

src, dst = sys.argv[1], sys.argv[2]
E = 2048
# the library the passes measured (bench.py reports a record only for this build)
LIB_SHA16 = open(os.path.join(src, "lib_sha16.txt")).read().strip()


KNAME = {}


def per_kernel(counter):
    f = glob.glob(os.path.join(src, counter, "**", "*counter_collection.csv"), recursive=True)[0]
    out = {}
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        key = ("copy" if name.startswith("__amd_rocclr_copyBuffer") and len(out.get("copy", [])) < 3 else
               "zr" if ("conv_band_kernel<256, 256, false, false, 6>" in name or
                        "conv_band_kernel<256, 256, false, false, 6, 8" in name) else
               "lookup" if ("corr_ce0_kernel" in name or "corr_pyramid_f16_r3_kernel" in name) else
               "lookup_nchw" if "corr_lookup_coop_kernel" in name else
               "alt" if ("corr_alt_ce0_kernel" in name or "corr_alt2_kernel" in name) else None)
        if key:
            out.setdefault(key, []).append(float(r["Counter_Value"]))
            KNAME[key] = name
    return out


fetch, write = per_kernel("FETCH_SIZE"), per_kernel("WRITE_SIZE")
GiB = float(1 << 30)
# calibration: last copy launch (warm) moves exactly 1 GiB each way
kf = GiB / fetch["copy"][-1]
kw = GiB / write["copy"][-1]
res = {"calibration": {"fetch_bytes_per_unit": kf, "write_bytes_per_unit": kw,
                       "raw_fetch": fetch["copy"], "raw_write": write["copy"]}}
# fused lookup + corr_encoder[0]: window reads + coords + 128-channel fp16 output per edge
LOOKUP_CE0 = 4 * 64 * 2 * 3072 + 2 * 4 * 3072 + 128 * 2 * 3072
# z|r gates with the inp term per source frame: 3x3 over net | corr | flow (320 channels)
# on-demand lookup: query + target feature-pyramid rows, coords, 128-channel fp16 output per edge (bench.py)
ALT = 786432 + 1044480 + 24576 + 128 * 2 * 3072
# the reference API's NCHW lookup: SURVEY.md §8d's volume-API bytes (bench.py LOOKUP_BYTES_PER_EDGE)
LOOKUP_NCHW = 2801664
for key, name, algo in (("zr", "conv_zr", 2 * 256 * 320 * 9 * 3072 * E), ("lookup", "corr_lookup", LOOKUP_CE0 * E),
                        ("lookup_nchw", "corr_lookup_nchw", LOOKUP_NCHW * E),
                        ("alt", "corr_alt", ALT * E)):
    fb = kf * min(fetch[key])
    wb = kw * min(write[key])
    if key not in fetch or key not in write:
        continue
    d = {"edges": E, "kernel": KNAME.get(key), "lib_sha16": LIB_SHA16, "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
         "traffic_bytes_per_launch": fb + wb, "raw_fetch": fetch[key], "raw_write": write[key],
         "calibration": res["calibration"],
         "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; units calibrated on a "
                   "1 GiB device copy in the same process (min over 3 launches)"}
    if algo:
        d["algorithmic_flops_per_launch" if key == "zr" else "algorithmic_bytes_per_launch"] = algo
    with open(os.path.join(dst, "pmc_%s.json" % name), "w") as f:
        json.dump(d, f, indent=1)
    print(name, "fetch %.3g B, write %.3g B" % (fb, wb))
print("calibration fetch x%.4g write x%.4g" % (kf, kw))
