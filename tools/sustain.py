#!/usr/bin/env python3
"""Per-step kernel times over a long back-to-back run of bench.py's step (encode then
reconstruct, RS(10,3) B=1024, 100 000 groups): shows whether sustained load drifts
(clock/power) relative to short bursts with idle gaps between them.

  python tools/sustain.py [--steps 300] [--bucket 20]
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import quicknet_amd as qa  # noqa: E402
from quicknet_amd.synth import erasure_marks, marks_to_rs_layout  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=300)
    p.add_argument("--bucket", type=int, default=20)
    p.add_argument("--k", type=int, default=10)
    p.add_argument("--m", type=int, default=3)
    p.add_argument("--block", type=int, default=1024)
    p.add_argument("--groups", type=int, default=100_000)
    a = p.parse_args()
    k, m, B, G = a.k, a.m, a.block, a.groups
    dev = torch.device("cuda:0")
    code = qa.Code.cauchy(k, m)
    data = torch.empty((G, k, B), dtype=torch.uint8, device=dev)
    qa.synth_fill(data, 0x5EED0002)
    par = torch.empty((G, m, B), dtype=torch.uint8, device=dev)
    gm = erasure_marks(0x5EED0003, G, k + m, 3)
    marks = torch.from_numpy(marks_to_rs_layout(gm, k)).to(dev)
    work = data.clone()
    code.encode(data, par)
    code.prepare_reconstruct()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()

    def run(steps, gap):
        ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
        for i in range(steps):
            ev[i][0].record(s)
            code.encode(data, par)
            ev[i][1].record(s)
            code.reconstruct(work, par, marks)
            ev[i][2].record(s)
            if gap:
                torch.cuda.synchronize()
                torch.cuda._sleep(gap)
        torch.cuda.synchronize()
        return [(e[0].elapsed_time(e[1]) * 1e3, e[1].elapsed_time(e[2]) * 1e3) for e in ev]

    for label, steps, gap in (("back-to-back", a.steps, 0), ("synchronised, ~1 ms idle between steps", 60, 2_000_000)):
        t = run(steps, gap)
        print(f"{label}: {steps} steps")
        for b0 in range(0, steps, a.bucket):
            chunk = t[b0:b0 + a.bucket]
            enc = statistics.mean(x[0] for x in chunk)
            rec = statistics.mean(x[1] for x in chunk)
            print(f"  steps {b0:4d}-{b0 + len(chunk) - 1:4d}: encode {enc:6.1f} us  reconstruct {rec:6.1f} us  "
                  f"step {enc + rec:6.1f} us")
    assert torch.equal(work, data)


if __name__ == "__main__":
    main()
