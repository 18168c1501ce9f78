"""Per-kernel averages of rocprofv3 --pmc passes.
usage: python scripts/pmc_counters.py <dir with pass subdirs> [kernel substring]"""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if flt and flt not in name:
            continue
        vals[name[:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in vals.items():
    print(k)
    for c, v in sorted(d.items()):
        print("   %-32s n=%-3d mean=%.4g" % (c, len(v), sum(v) / len(v)))
