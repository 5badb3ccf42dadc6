"""Which /proc/self/maps mapping holds each kind of pointer the rs.h host path can be handed:
device tensors (small and large), pinned host tensors, numpy (pageable) arrays.  Prints one line per
pointer: kind, address, and the mapping's range / permissions / path.  Evidence for classifying
shard pointers by mapping instead of one runtime probe per pointer.
"""
import numpy as np
import torch


def maps():
    out = []
    with open("/proc/self/maps") as f:
        for line in f:
            parts = line.split(None, 5)
            lo, hi = (int(x, 16) for x in parts[0].split("-"))
            out.append((lo, hi, parts[1], parts[5].strip() if len(parts) > 5 else ""))
    return out


def where(p, mp):
    for lo, hi, perm, path in mp:
        if lo <= p < hi:
            return f"{lo:#x}-{hi:#x} {perm} {path or '[anon]'} ({(hi - lo) >> 20} MiB)"
    return "no mapping"


def main():
    dev = torch.device("cuda:0")
    objs = {
        "dev 4 KiB": torch.empty(4096, dtype=torch.uint8, device=dev),
        "dev 1 MiB": torch.empty(1 << 20, dtype=torch.uint8, device=dev),
        "dev 256 MiB": torch.empty(256 << 20, dtype=torch.uint8, device=dev),
        "dev 4 GiB": torch.empty(4 << 30, dtype=torch.uint8, device=dev),
        "pinned 1 MiB": torch.empty(1 << 20, dtype=torch.uint8).pin_memory(),
        "pinned 256 MiB": torch.empty(256 << 20, dtype=torch.uint8).pin_memory(),
    }
    nps = {"numpy 1 KiB": np.zeros(1024, np.uint8), "numpy 1 MiB": np.zeros(1 << 20, np.uint8),
           "numpy 1 GiB": np.zeros(1 << 30, np.uint8)}
    mp = maps()
    for name, t in objs.items():
        p = t.data_ptr()
        print(f"{name:16s} {p:#x}  {where(p, mp)}")
        print(f"{'':16s} end-1 {p + t.numel() - 1:#x}  {where(p + t.numel() - 1, mp)}")
    for name, a in nps.items():
        p = a.ctypes.data
        print(f"{name:16s} {p:#x}  {where(p, mp)}")
    devs = [(lo, hi, perm, path) for lo, hi, perm, path in mp if "/dev/" in path]
    print(f"{len(mp)} mappings, {len(devs)} from /dev/ files:")
    seen = {}
    for lo, hi, perm, path in devs:
        seen.setdefault((perm, path), [0, 0])
        seen[(perm, path)][0] += 1
        seen[(perm, path)][1] += hi - lo
    for (perm, path), (cnt, tot) in sorted(seen.items()):
        print(f"  {perm} {path}: {cnt} mappings, {tot >> 20} MiB")
    none = [(lo, hi) for lo, hi, perm, path in mp if perm.startswith("---")]
    print(f"{len(none)} PROT_NONE mappings, {sum(h - l for l, h in none) >> 30} GiB")


if __name__ == "__main__":
    main()
