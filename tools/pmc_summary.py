#!/usr/bin/env python3
"""Average PMC counters per kernel (and per wave) from a rocprofv3 counter_collection.csv.
    python tools/pmc_summary.py DIR [name-filter]"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if flt in n:
            agg[n.split("(")[0][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for n, c in agg.items():
    waves = sum(c["SQ_WAVES"]) / max(1, len(c["SQ_WAVES"])) if "SQ_WAVES" in c else 0
    print(n)
    for k, v in sorted(c.items()):
        avg = sum(v) / len(v)
        print(f"   {k:20s} {avg:16.0f}" + (f"   per wave {avg / waves:10.1f}" if waves else ""))
