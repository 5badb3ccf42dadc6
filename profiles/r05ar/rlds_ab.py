import os, sys, statistics
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import quicknet_amd as qa
sys.argv = [sys.argv[0]]
from tools.occ_ab import shape
shapes = {"RS(10,3) B=1024": shape(10, 3, 1024, 100_000, 3, 0x5EED0002), "RS(16,4) B=1400": shape(16, 4, 1400, 250_000, 4, 0x5EED0004)}
vals = ("0", "9000", "11000", "13653", "16384")
s = torch.cuda.current_stream()
times = {}
for r in range(6):
    for sn, S in shapes.items():
        for v in vals:
            os.environ["QFEC_RLDS"] = v
            fn = lambda: S["code"].reconstruct(S["work"], S["par"], S["marks"], S["B"])
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(10):
                fn()
            e1.record(s)
            torch.cuda.synchronize()
            times.setdefault((sn, v), []).append(e0.elapsed_time(e1) / 10)
os.environ["QFEC_RLDS"] = "0"
for (sn, v), t in times.items():
    print(sn, v, f"{statistics.median(t)*1e3:.1f} us min {min(t)*1e3:.1f}", flush=True)
print("ok", all(torch.equal(S["work"], S["data"]) for S in shapes.values()))
