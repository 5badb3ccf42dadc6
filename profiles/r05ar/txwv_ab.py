import os, sys, statistics
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import quicknet_amd as qa
k, m, S, G = 10, 3, 1024, 100_000
n = k + m
dev = torch.device("cuda:0")
code = qa.Code.vandermonde(k, m)
payload = torch.empty(G * k * S + 16, dtype=torch.uint8, device=dev)
qa.synth_fill(payload, 77)
offsets = torch.arange(G * k, dtype=torch.int64, device=dev) * S
sizes = torch.full((G * k,), S, dtype=torch.int32, device=dev)
seq = torch.stack([torch.arange(G, dtype=torch.int32, device=dev) * n, torch.arange(G, dtype=torch.int32, device=dev) * k], 1).contiguous()
sp = (S + 4 + 15) // 16 * 16
wp = (sp + 13 + 63) // 64 * 64
fp = (sp + 13 + 4 + 63) // 64 * 64
L = qa.lib()
shards = torch.empty((G, n, sp), dtype=torch.uint8, device=dev)
wire = torch.empty((G, n, wp), dtype=torch.uint8, device=dev)
wlen = torch.empty((G, n), dtype=torch.int32, device=dev)
masks = (torch.arange(G * n, dtype=torch.int32, device=dev) * 7 & 0xFF).to(torch.uint8)
frames = torch.empty((G, n, fp), dtype=torch.uint8, device=dev)
flen = torch.empty((G, n), dtype=torch.int32, device=dev)
s = torch.cuda.current_stream()
st = s.cuda_stream
def pack():
    assert L.qfec_pack_datagrams(code._h, payload.data_ptr(), offsets.data_ptr(), sizes.data_ptr(), seq.data_ptr(), G, 1, shards.data_ptr(), sp, wire.data_ptr(), wp, wlen.data_ptr(), st) == 0
def pack_frames():
    assert L.qfec_pack_frames(code._h, payload.data_ptr(), offsets.data_ptr(), sizes.data_ptr(), seq.data_ptr(), G, 1, shards.data_ptr(), sp, masks.data_ptr(), None, 0x3C, 0x11, 0xFF, frames.data_ptr(), fp, flen.data_ptr(), st) == 0
ref = {}
for name, fn, out in (("pack", pack, wire), ("frames", pack_frames, frames)):
    for key in ("QFEC_TXWV", "QFEC_FRWV"):
        os.environ.pop(key, None)
    out.zero_(); fn(); torch.cuda.synchronize(); ref[name] = out.clone()
times = {}
same = True
for r in range(8):
    for name, fn, out, key in (("pack", pack, wire, "QFEC_TXWV"), ("frames", pack_frames, frames, "QFEC_FRWV")):
        for on in (False, True):
            if on: os.environ[key] = "1"
            else: os.environ.pop(key, None)
            out.zero_(); fn(); torch.cuda.synchronize()
            same &= bool(torch.equal(out, ref[name]))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(10): fn()
            e1.record(s); torch.cuda.synchronize()
            times.setdefault((name, on), []).append(e0.elapsed_time(e1) / 10)
    os.environ.pop("QFEC_TXWV", None); os.environ.pop("QFEC_FRWV", None)
for (name, on), t in times.items():
    print(name, "more waves" if on else "default", f"median {statistics.median(t)*1e3:.1f} us min {min(t)*1e3:.1f}", flush=True)
print("outputs identical:", same)
