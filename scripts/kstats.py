"""Print a bench JSON line's value and the rocprofv3 average duration of the
kernels whose names contain any of the given substrings.

usage: python scripts/kstats.py BENCH_JSON KERNEL_STATS_CSV [substring ...]"""
import csv
import json
import sys

d = json.load(open(sys.argv[1]))
print("%.2f %s" % (d["value"], d["unit"]))
keys = sys.argv[3:]
for r in csv.DictReader(open(sys.argv[2])):
    if not keys or any(k in r["Name"] for k in keys):
        print("%-60s %4s %8.3f ms" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e6))
