#!/usr/bin/env python3
"""Per-kernel SQ counter averages from rocprofv3 --pmc counter_collection.csv files, per wave.

  python tools/sq_summary.py DIR [DIR ...]
SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_* count quad-cycles (MI355X_MICROARCH.md).
"""
import collections
import csv
import glob
import os
import sys


def main():
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                name = row.get("Kernel_Name", "")[:90]
                vals[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for name, cs in sorted(vals.items()):
        w = cs.get("SQ_WAVES")
        if not w:
            continue
        waves = sum(w) / len(w)
        print(f"{name}\n  dispatches {len(w)}  waves {waves:.0f}")
        for c in sorted(cs):
            v = sum(cs[c]) / len(cs[c])
            print(f"  {c:24s} {v:16.0f}  per wave {v / max(waves, 1):10.1f}")


if __name__ == "__main__":
    main()
