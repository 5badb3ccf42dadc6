#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 rocpd database (results.db), like --stats' CSV.

  python tools/kstats.py gpurun_out/x/prof/run_results.db [--csv out.csv]
"""
import argparse
import sqlite3


def main():
    p = argparse.ArgumentParser()
    p.add_argument("db")
    p.add_argument("--csv")
    p.add_argument("--top", type=int, default=20)
    a = p.parse_args()
    c = sqlite3.connect(a.db)
    rows = list(c.execute("select name, count(*), sum(end - start), avg(end - start), min(end - start), "
                          "max(end - start) from kernels group by name order by sum(end - start) desc"))
    total = sum(r[2] for r in rows) or 1
    lines = ["Name,Calls,TotalDurationNs,AverageNs,Percentage,MinNs,MaxNs"]
    for name, n, tot, avg, mn, mx in rows:
        lines.append(f'"{name}",{n},{tot},{avg:.1f},{100.0 * tot / total:.2f},{mn},{mx}')
    for l in lines[:a.top + 1]:
        print(l[:160])
    if a.csv:
        with open(a.csv, "w") as f:
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
