#!/usr/bin/env python3
"""Static instruction histogram of one kernel in a hipcc --save-temps .s file.

  python tools/isa_hist.py FILE.s SYMBOL_SUBSTRING [--top 40] [--dump OUT.s]
Counts instructions by mnemonic and by class (VALU / SALU / VMEM / SMEM / LDS / branch)
between the kernel's label and its .Lfunc_end marker.
"""
import argparse
import collections
import re


def main():
    p = argparse.ArgumentParser()
    p.add_argument("file")
    p.add_argument("sym")
    p.add_argument("--top", type=int, default=40)
    p.add_argument("--dump")
    a = p.parse_args()
    lines = open(a.file).read().split("\n")
    start = None
    for i, l in enumerate(lines):
        if l.startswith("_Z") and l.split(":")[0].endswith(a.sym) or (l.startswith("_Z") and ":" in l and a.sym in l.split(":")[0]):
            start = i
            break
    if start is None:
        raise SystemExit("symbol not found")
    name = lines[start].split(":")[0]
    body = []
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        body.append(l)
    if a.dump:
        open(a.dump, "w").write("\n".join(body))
    hist = collections.Counter()
    cls = collections.Counter()
    for l in body:
        s = l.strip()
        if not s or s.startswith(";") or s.startswith(".") or s.endswith(":"):
            continue
        op = s.split()[0]
        hist[op] += 1
        if op.startswith("v_"):
            c = "VALU"
        elif op.startswith("s_") and op.startswith(("s_load", "s_buffer_load")):
            c = "SMEM"
        elif op.startswith(("s_cbranch", "s_branch")):
            c = "branch"
        elif op.startswith("s_waitcnt"):
            c = "waitcnt"
        elif op.startswith("s_"):
            c = "SALU"
        elif op.startswith(("global_", "buffer_", "flat_")):
            c = "VMEM"
        elif op.startswith("ds_"):
            c = "LDS"
        else:
            c = "other"
        cls[c] += 1
    print(name)
    print("classes:", dict(cls), "total", sum(cls.values()))
    for op, n in hist.most_common(a.top):
        print(f"{n:6d} {op}")


if __name__ == "__main__":
    main()
