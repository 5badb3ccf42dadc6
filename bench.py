#!/usr/bin/env python3
"""bench.py -- RS(k,m) FEC encode+decode GiB/s, device-resident, on 1..8 MI355X.

One step = the BASELINE.json configs[1] + configs[2] workload on one batch held in HBM:
  encode      RS(10,3) of 1 000 000 x 1 KiB packets = 100 000 groups   (module/rs.c:574)
  reconstruct the same 100 000 groups with 3 random erasures per group out of 13
              (seed 0x5EED0003), rs.c survivor rule                     (module/rs.c:598)
Cauchy matrix (bit-exact with module/rs.c).  Weak scaling: every rank owns its own
100 000 groups (distinct seeds); value = all ranks' data bytes / the slowest rank's time.

Beside the headline, every rank also runs (inside barriers, max-over-ranks timing):
  config4     RS(16,4) encode + 4-erasure reconstruct of 250 000 x 1400 B groups, split
              contiguously over the ranks (strong scaling: the job is fixed), and
  host_mixed  config 5: mixed (4,2)/(10,3)/(16,4) batches streamed host -> device -> host
              through the qfec_pipe engine (pinned buffers, 3 HIP streams per GPU).

  python bench.py [--gpus N] [--steps K] [--warmup W]
      --gpus N > 1 without WORLD_SIZE: this process starts N rank processes itself (before
      any GPU call) and exits with the worst of their return codes.
  torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, the same protocol)

Prints ONE JSON line (rank 0).  Data GiB/s counts payload bytes: k*B per encoded group and
k*B per decoded group (groups with no erased data shard cost nothing, rs.c:620).
"""
import argparse
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from quicknet_amd import topology  # noqa: E402  (sysfs only: no torch, no HIP)
from quicknet_amd.sharding import rank_seed, shard_range  # noqa: E402

# numpy / torch / the codec are imported by _load(), after the launcher decision: the parent of
# `bench.py --gpus N` starts its ranks without ever importing torch
np = torch = qa = None
SEED_DECODE = SEED_ENCODE = SEED_RS16 = erasure_marks = marks_to_rs_layout = None


def _load():
    global np, torch, qa, SEED_DECODE, SEED_ENCODE, SEED_RS16, erasure_marks, marks_to_rs_layout
    if torch is not None:
        return
    import numpy
    import torch as _torch

    import quicknet_amd  # libqfec.so is loaded lazily, at the first codec call
    from quicknet_amd import synth
    np, torch, qa = numpy, _torch, quicknet_amd
    SEED_DECODE, SEED_ENCODE, SEED_RS16 = synth.SEED_DECODE, synth.SEED_ENCODE, synth.SEED_RS16
    erasure_marks, marks_to_rs_layout = synth.erasure_marks, synth.marks_to_rs_layout

METRIC = "RS(k,m) FEC encode+decode GiB/s (device-resident) at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
GIB = float(1 << 30)
# the kernel sources whose PMC traffic profiles/traffic.json holds (stale if they change)
KERNEL_SOURCES = ("quicknet_amd/csrc/qfec_kernels.hip", "quicknet_amd/csrc/qfec_internal.hpp",
                  "quicknet_amd/csrc/qfec_device.hpp")
# ... and those of the datagram / framing legs (their own traffic.json entry)
WIRE_KERNEL_SOURCES = KERNEL_SOURCES + ("quicknet_amd/csrc/qfec_wire.hip", "quicknet_amd/csrc/qfec_rx.hip",
                                        "quicknet_amd/csrc/qfec_frame.hip", "quicknet_amd/csrc/qfec_wire_device.hpp")
TRAFFIC_PATH = os.path.join(ROOT, "profiles", "traffic.json")


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1, help="ranks (one per GPU); >1 without WORLD_SIZE spawns them")
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--spinup-ms", type=float, default=25.0,
                   help="setup: run the step for this long before the W warmup steps (clock ramp, tools/sustain.py)")
    p.add_argument("--k", type=int, default=10)
    p.add_argument("--m", type=int, default=3)
    p.add_argument("--block", type=int, default=1024)
    p.add_argument("--groups", type=int, default=100_000)
    p.add_argument("--erasures", type=int, default=3)
    p.add_argument("--flavour", choices=["cauchy", "vandermonde"], default="cauchy")
    p.add_argument("--variant", type=int, default=0, help="0 perm tables (default), 1 LDS log/exp")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget (rank 0, N=1)")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--cpu-threads", type=int, default=None,
                   help="threads for the all-cores CPU baseline (default: the CPUs this process may use -- "
                        "affinity mask and cgroup quota, quicknet_amd.topology.cpu_share; 0 skips it)")
    p.add_argument("--no-side", action="store_true", help="skip the rank-0 side configurations")
    p.add_argument("--no-config4", action="store_true", help="skip the sharded RS(16,4) config 4 leg")
    p.add_argument("--config4-only", action="store_true",
                   help="run only the config 4 leg and print its record (tools/pmc_traffic.py --workload config4)")
    p.add_argument("--config4-groups", type=int, default=250_000, help="config 4 job size (tests shrink it)")
    p.add_argument("--no-host", action="store_true", help="skip the host-to-host legs (config 5)")
    p.add_argument("--protocol-check", action="store_true",
                   help="no GPU work: run the rank launch + barrier/max/sum protocol only (CPU tests)")
    p.add_argument("--launch-check", action="store_true",
                   help="launcher only: print the pre-spawn state (device count, NUMA plan, open GPU fds) and exit")
    p.add_argument("--deadline-s", type=float, default=1500.0,
                   help="launcher: ranks still running after this many seconds are killed (exit 124)")
    p.add_argument("--fail-grace-s", type=float, default=15.0,
                   help="launcher: after one rank fails, the others are ended this many seconds later")
    p.add_argument("--fail-rank", type=int, default=-1, help="--protocol-check only: this rank exits 3 (tests)")
    p.add_argument("--hang-rank", type=int, default=-1, help="--protocol-check only: this rank hangs (tests)")
    p.add_argument("--no-numa-bind", action="store_true", help="do not bind ranks to their GPU's NUMA node")
    p.add_argument("--force-dist", action="store_true",
                   help="init the process group even at one rank (exercises the RCCL path on a one-GPU box)")
    p.add_argument("--traffic", default=TRAFFIC_PATH,
                   help="PMC-derived HBM bytes per launch (tools/pmc_traffic.py), if present")
    return p.parse_args(argv)


# ---------------------------------------------------------------------------- rank launch
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _kill_group(p, sig):
    try:
        os.killpg(p.pid, sig)
    except (ProcessLookupError, PermissionError):
        pass


def launch_ranks(args, argv):
    """--gpus N > 1 with no WORLD_SIZE in the environment: start N fresh rank processes and
    return the worst of their exit codes.

    This process never imports torch and makes no HIP call: it counts devices from the KFD
    topology in sysfs (quicknet_amd.topology), and when sysfs does not say, each rank checks
    its own index (dist_setup).  Every rank runs in its own session, so ending it ends the
    processes it started too.  A rank that fails ends the others after --fail-grace-s (they
    would wait on a barrier forever); ranks still running at --deadline-s are killed and the
    launcher exits 124."""
    import signal
    n = args.gpus
    backend = os.environ.get("QFEC_BENCH_BACKEND", "nccl")
    count, source = (None, "not checked")
    if not args.protocol_check and backend == "nccl":
        count, source = topology.gpu_count()
        if count is not None and count < n:
            print(f"bench.py: --gpus {n} but only {count} GPU(s) visible ({source})", file=sys.stderr)
            return 2
    if args.launch_check:  # the pre-spawn state, for tests: no torch, no GPU file open
        print(json.dumps({"launch_check": True, "gpus_arg": n, "gpu_count": count, "gpu_count_source": source,
                          "torch_imported": "torch" in sys.modules, "gpu_fds": topology.open_gpu_fds(),
                          "plan": [topology.gpu_numa(r) and {kk: (len(v) if kk == "cpus" else v)
                                                              for kk, v in topology.gpu_numa(r).items()}
                                   for r in range(n)]}), flush=True)
        return 0
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env,
                                      start_new_session=True))
    rcs = [None] * n
    t_start = time.time()
    failed_at = first_bad = None
    timed_out = False
    try:
        while any(rc is None for rc in rcs):
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    rcs[i] = p.poll()
                    if rcs[i] not in (None, 0) and failed_at is None:
                        failed_at, first_bad = time.time(), rcs[i]
                        print(f"bench.py: rank {i} exited {rcs[i]}; ending the others in {args.fail_grace_s:g} s",
                              file=sys.stderr)
            now = time.time()
            over = now - t_start > args.deadline_s
            if over and not timed_out and any(rc is None for rc in rcs):
                timed_out = True
                print(f"bench.py: launch deadline {args.deadline_s:g} s passed; killing the ranks still running",
                      file=sys.stderr)
            if over or (failed_at is not None and now - failed_at > args.fail_grace_s):
                for i, p in enumerate(procs):
                    if rcs[i] is None:
                        _kill_group(p, signal.SIGTERM)
                for i, p in enumerate(procs):
                    if rcs[i] is None:
                        try:
                            rcs[i] = p.wait(timeout=10)
                        except subprocess.TimeoutExpired:
                            _kill_group(p, signal.SIGKILL)
                            rcs[i] = p.wait()
            time.sleep(0.05)
    finally:
        for p in procs:  # never leave a rank behind (e.g. the launcher itself interrupted)
            if p.poll() is None:
                _kill_group(p, signal.SIGKILL)
                p.wait()
    if timed_out:
        return 124
    if failed_at is None:
        return 0
    return first_bad if first_bad > 0 else 1  # the rank that failed first, not the ones ended after it


def dist_setup(args):
    """One rank per GPU over RCCL.  QFEC_BENCH_BACKEND=gloo (rehearsal only) runs the same
    rank protocol over gloo, with ranks sharing the visible GPUs round-robin.  Before anything
    imports torch, the rank binds itself to its GPU's NUMA node (quicknet_amd.topology)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
    backend = os.environ.get("QFEC_BENCH_BACKEND", "nccl")
    if args.protocol_check:
        backend = "gloo"
    numa = None
    if not args.protocol_check:
        dev_index = local
        if backend != "nccl":
            cnt, _ = topology.gpu_count()
            dev_index = local % cnt if cnt else 0
        numa = topology.bind_rank(dev_index) if not args.no_numa_bind else {"bound": False, "reason": "--no-numa-bind"}
    if args.protocol_check and args.fail_rank == rank:
        raise SystemExit(3)  # injected failure (tests/test_launch.py)
    if args.protocol_check and args.hang_rank == rank:
        time.sleep(3600)
    _load()
    if not args.protocol_check:
        have = torch.cuda.device_count()
        if backend != "nccl":
            local %= max(1, have)
        if local >= have:  # this rank's own check (the launcher may not have been able to count)
            print(f"bench.py: rank {rank} wants device {local} but {have} GPU(s) are visible", file=sys.stderr)
            raise SystemExit(2)
        torch.cuda.set_device(local)
        if isinstance(numa, dict) and not args.no_numa_bind:
            # the device HIP actually gave this rank: if sysfs ordering guessed another one,
            # move to the right node now (before any pinned host allocation)
            actual = topology.bdf_of_torch_device(torch.cuda.get_device_properties(local))
            numa["bdf_hip"] = actual
            if actual and numa.get("bdf") and actual != numa["bdf"]:
                numa["rebound"] = topology.bind_bdf(actual)
    if world > 1 or args.force_dist:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local, numa


def _dist_on():
    if torch is None:
        return False
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized()


def barrier(world):
    if _dist_on():
        import torch.distributed as dist
        dist.barrier()


def _all_reduce(x, world, op):
    """One float over all ranks.  The tensor lives where the backend wants it: on the GPU for
    RCCL, on the host for gloo (tests/test_multiproc.py drives these helpers over gloo)."""
    _load()
    if not _dist_on():
        return x
    import torch.distributed as dist
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=op)
    return float(t.item())


def all_max(x, world):
    import torch.distributed as dist
    return _all_reduce(x, world, dist.ReduceOp.MAX)


def all_sum(x, world):
    import torch.distributed as dist
    return _all_reduce(x, world, dist.ReduceOp.SUM)


def all_gather_float(x, world, rank):
    """Every rank's value of x, in rank order (a one-hot sum: one all-reduce of `world` floats)."""
    _load()
    if not _dist_on():
        return [x]
    import torch.distributed as dist
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.zeros(world, dtype=torch.float64, device=dev)
    t[rank] = x
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [float(v) for v in t.cpu().tolist()]


def protocol_check(args, rank, world):
    """The launch + timing protocol with no GPU work (CPU tests): each rank 'works' for a
    rank-dependent time; the line carries the same n_gpus / max-time / summed-units fields."""
    barrier(world)
    t0 = time.perf_counter()
    time.sleep(0.01 * (rank + 1))
    t1 = time.perf_counter()
    barrier(world)
    el = all_max(t1 - t0, world)
    units = all_sum(float(1000 * (rank + 1)), world)
    ranks = all_gather_float(float(os.getpid()), world, rank)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "protocol_check": True, "n_gpus": world, "gpus_arg": args.gpus,
                          "elapsed_max_s": el, "units": units, "distinct_rank_pids": len(set(ranks))}), flush=True)
    return 0


# ---------------------------------------------------------------------------- CPU baseline
def cpu_baseline(args, budget_s):
    """The reference's own rs.c (oracle/_ref, kind 'reference') -- or the CPU restatement
    (oracle/liboracle.so, kind 'port') when _ref is absent -- on a bounded sample of the same
    workload: encode + 3-erasure reconstruct of `sample` groups, 1 thread, repeated until the
    budget is spent."""
    from oracle.oracle import Oracle, RefCodec
    from quicknet_amd.synth import synth_bytes
    k, m, B = args.k, args.m, args.block
    sample = 10_000
    data = synth_bytes(SEED_ENCODE, sample * k * B).reshape(sample, k, B)
    par = np.zeros((sample, m, B), np.uint8)
    gm = erasure_marks(SEED_DECODE, sample, k + m, args.erasures)
    marks = marks_to_rs_layout(gm, k)
    dec_groups = int((gm[:, :k].sum(1) > 0).sum())
    if RefCodec.available() and args.flavour == "cauchy":
        ref = RefCodec()
        kind = "reference"
        h = ref.rs.reed_solomon_new(k, m)
        work = data.copy()
        ptrs = ref.shard_ptrs(work, par)
        n = sample * (k + m)

        def step():
            ref.rs_encode(h, ptrs, n, B)
            ref.rs_reconstruct(h, ptrs, marks, n, B)
    else:
        orc = Oracle()
        kind = "port"
        rows = orc.cauchy(k, m) if args.flavour == "cauchy" else orc.vandermonde(k, k + m)
        work = data.copy()

        def step():
            orc.rs_encode(rows, work, par, B)
            orc.rs_reconstruct(rows, work, par, marks, B)
    t0 = time.perf_counter()
    reps = 0
    while True:
        step()
        reps += 1
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    gib = reps * (sample + dec_groups) * k * B / GIB
    return {"value": round(gib / el, 4), "unit": "GiB/s", "cores": 1, "kind": kind, "cpu_model": cpu_model(),
            "sample": f"{reps} x (encode {sample} groups + reconstruct {dec_groups} groups with {args.erasures} "
                      f"random erasures/group), RS({k},{m}) B={B}, {el:.1f} s, 1 thread"}


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline_threads(args, budget_s, threads):
    """The same reference rs.c sample on `threads` host threads: groups split into contiguous
    slices (quicknet_amd.sharding's rule), one pointer array per slice, each thread looping
    encode + reconstruct on its slice until the budget is spent.  ctypes drops the GIL for
    the foreign call, so the threads run the C code in parallel; rs.c is reentrant after
    reed_solomon_init (its tables are read-only, the decode matrix lives on the stack)."""
    import threading
    from oracle.oracle import RefCodec
    from quicknet_amd.synth import synth_bytes
    if not RefCodec.available() or args.flavour != "cauchy":
        return None
    k, m, B = args.k, args.m, args.block
    sample = 10_000
    data = synth_bytes(SEED_ENCODE, sample * k * B).reshape(sample, k, B)
    par = np.zeros((sample, m, B), np.uint8)
    gm = erasure_marks(SEED_DECODE, sample, k + m, args.erasures)
    ref = RefCodec()
    h = ref.rs.reed_solomon_new(k, m)
    slices = []
    for t in range(threads):
        a, b = shard_range(sample, t, threads)
        if b > a:
            sl_marks = marks_to_rs_layout(gm[a:b], k)
            slices.append((ref.shard_ptrs(data[a:b], par[a:b]), sl_marks, (b - a) * (k + m),
                           (b - a + int((gm[a:b, :k].sum(1) > 0).sum())) * k * B))
    done = [0] * len(slices)
    spent = [0.0] * len(slices)
    start = threading.Barrier(len(slices) + 1)

    def run(i):
        ptrs, mk, n, _ = slices[i]
        start.wait()
        t0 = time.perf_counter()
        while True:
            ref.rs_encode(h, ptrs, n, B)
            ref.rs_reconstruct(h, ptrs, mk, n, B)
            done[i] += 1
            spent[i] = time.perf_counter() - t0
            if spent[i] >= budget_s:
                break

    ths = [threading.Thread(target=run, args=(i,)) for i in range(len(slices))]
    for t in ths:
        t.start()
    start.wait()
    for t in ths:
        t.join()
    el = max(spent)
    gib = sum(done[i] * slices[i][3] for i in range(len(slices))) / GIB
    return {"value": round(gib / el, 4), "unit": "GiB/s", "cores": len(slices), "kind": "reference",
            "sample": f"{sum(done)} slice passes over {sample} groups split {len(slices)} ways (encode + reconstruct with "
                      f"{args.erasures} random erasures/group), RS({k},{m}) B={B}, {el:.1f} s, {len(slices)} threads"}


def cpu_check_host_sample(samples):
    """The cpu_baseline leg's checker for config 5 (host_to_host_mixed): sampled groups of every
    pipe batch run through the reference's own module/rs.c (oracle/_ref) -- encode must give the
    parity the pipe wrote, and reconstruct of the same damaged groups must give the rows the pipe
    restored.  Without oracle/_ref, the C restatement (oracle/liboracle.so) is the checker."""
    from oracle.oracle import Oracle, RefCodec
    use_ref = RefCodec.available()
    ref = RefCodec() if use_ref else None
    orc = None if use_ref else Oracle()
    groups = bad = 0
    for s in samples:
        k, m, B = s["k"], s["m"], s["B"]
        G = len(s["idx"])
        data = np.ascontiguousarray(s["data"])
        par = np.zeros((G, m, B), np.uint8)
        dmg = data.copy()
        dmg[s["marks_data"].astype(bool)] = 0x5A
        marks = np.concatenate([s["marks_data"].reshape(-1), s["marks_parity"].reshape(-1)]).astype(np.uint8)
        if use_ref:
            h = ref.rs.reed_solomon_new(k, m)
            ref.rs_encode(h, ref.shard_ptrs(data, par), G * (k + m), B)
            rpar = par.copy()
            ref.rs_reconstruct(h, ref.shard_ptrs(dmg, rpar), marks, G * (k + m), B)
            ref.rs.reed_solomon_release(h)
        else:
            rows = orc.cauchy(k, m)
            orc.rs_encode(rows, data, par, B)
            orc.rs_reconstruct(rows, dmg, par.copy(), marks, B)
        good = (par == s["parity"]).all(axis=(1, 2)) & (dmg == s["restored"]).all(axis=(1, 2))
        groups += G
        bad += int((~good).sum())
    return {"match": bad == 0, "groups_checked": groups, "mismatched_groups": bad,
            "checker": "reference module/rs.c (oracle/_ref)" if use_ref else "oracle/liboracle.so (C restatement)"}


def cpu_check_rs_sample(sm):
    """The cpu_baseline leg's checker for rs_abi_host: the sampled groups through the reference's
    own module/rs.c (oracle/_ref; the C restatement oracle/liboracle.so without it) -- its encode
    must give the parity reed_solomon_encode wrote, and its reconstruct of the same damaged groups
    the rows reed_solomon_reconstruct restored."""
    from oracle.oracle import Oracle, RefCodec
    k, m, B = sm["k"], sm["m"], sm["B"]
    data, gm = np.ascontiguousarray(sm["data"]), sm["marks_gn"]
    S = data.shape[0]
    par = np.zeros((S, m, B), np.uint8)
    marks = marks_to_rs_layout(gm, k)
    dmg = data.copy()
    dmg[gm[:, :k].astype(bool)] = 0x5A
    if RefCodec.available():
        ref = RefCodec()
        h = ref.rs.reed_solomon_new(k, m)
        ptrs = ref.shard_ptrs(data, par)
        ref.rs_encode(h, ptrs, S * (k + m), B)
        ptrs = ref.shard_ptrs(dmg, par)
        rc = ref.rs_reconstruct(h, ptrs, marks, S * (k + m), B)
        ref.rs.reed_solomon_release(h)
        kind = "reference rs.c (oracle/_ref)"
    else:
        orc = Oracle()
        rows = orc.cauchy(k, m)
        orc.rs_encode(rows, data, par, B)
        rc = orc.rs_reconstruct(rows, dmg, par, marks, B)
        kind = "C restatement (oracle/liboracle.so)"
    par_ok = bool(np.array_equal(par, sm["par"]))
    rec_ok = bool(np.array_equal(dmg, sm["restored"]))
    return {"groups": int(S), "checker": kind, "parity_match": par_ok, "restored_match": rec_ok, "rc": int(rc),
            "match": par_ok and rec_ok and rc == 0}


def cpu_config0(budget_s):
    """BASELINE configs[0] literally: RS(10,3) encode of 10 000 x 1 KiB packets (1 000 groups)
    through the reference's own per-packet fec.c, as network/FecCodec.cpp drives it
    (fec_new(10, 13), then fec_encode(.., 10 + j, 1024) for j < 3 per group,
    FecCodecBuf.cpp:151), 1 thread, repeated until the budget is spent."""
    import ctypes as C
    from oracle.oracle import RefCodec
    from quicknet_amd.synth import SEED_CPU_ENCODE, synth_bytes
    if not RefCodec.available():
        return None
    ref = RefCodec()
    k, n, B, G = 10, 13, 1024, 1000
    data = synth_bytes(SEED_CPU_ENCODE, G * k * B).reshape(G, k, B)
    out = np.zeros((G, n - k, B), np.uint8)
    code = ref.fec.fec_new(k, n)
    srcs = [(C.c_void_p * k)(*[data[g, i].ctypes.data for i in range(k)]) for g in range(G)]
    t0 = time.perf_counter()
    reps = 0
    while True:
        for g in range(G):
            for j in range(n - k):
                ref.fec.fec_encode(code, srcs[g], C.c_void_p(out[g, j].ctypes.data), k + j, B)
        reps += 1
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    ref.fec.fec_free(code)
    return {"value": round(reps * G * k * B / el / GIB, 4), "unit": "GiB/s", "cores": 1, "kind": "reference",
            "sample": f"{reps} x {G * k} packets, RS(10,3) fec_encode per parity packet (system/fec.c), {el:.1f} s"}


# ---------------------------------------------------------------------------- GPU legs
# rank 0's side configurations (after the timed region): the Vandermonde flavour the network
# stack links (module/fec.c) at configs[1]+[2], and config 5's RS(4,2) shape device-resident
SIDE = (("vandermonde", 10, 3, 1024, 100_000, 3), ("cauchy", 4, 2, 1024, 100_000, 2))


def _make_batch(flavour, k, m, B, G, E, seed_data, marks_gm, dev):
    n, pitch = k + m, (B + 15) // 16 * 16
    code = qa.Code.cauchy(k, m) if flavour == "cauchy" else qa.Code.vandermonde(k, m)
    data = torch.empty((G, k, pitch), dtype=torch.uint8, device=dev)
    qa.synth_fill(data, seed_data)
    parity = torch.empty((G, m, pitch), dtype=torch.uint8, device=dev)
    gm = marks_gm
    marks = torch.from_numpy(marks_to_rs_layout(gm, k)).to(dev)
    work = data.clone()
    work[torch.from_numpy(gm[:, :k].astype(bool)).to(dev)] = 0x5A
    code.encode(data, parity, B)
    code.prepare_reconstruct()
    return code, data, parity, marks, work


def _spin(step, spinup_ms):
    t_spin = time.perf_counter()
    while (time.perf_counter() - t_spin) * 1e3 < spinup_ms:
        for _ in range(5):
            step()
        torch.cuda.synchronize()


def side_config(flavour, k, m, B, G, E, rank, steps=20, warmup=5, spinup_ms=25.0):
    """One encode + reconstruct step on G groups, device-resident, pitch = B rounded up to
    16 B (bytes counted at B); per-kernel HIP events; reconstruct must restore the data."""
    dev = torch.device("cuda", torch.cuda.current_device())
    gm = erasure_marks(rank_seed(SEED_DECODE ^ (k << 8 | m), rank), G, k + m, E)
    code, data, parity, marks, work = _make_batch(flavour, k, m, B, G, E, rank_seed(SEED_ENCODE ^ (k << 8 | m), rank),
                                                  gm, dev)
    dec_groups = int((gm[:, :k].sum(1) > 0).sum())
    erased = int(gm[:, :k].sum())
    s = torch.cuda.current_stream()

    def step():
        code.encode(data, parity, B)
        code.reconstruct(work, parity, marks, B)

    _spin(step, spinup_ms)
    for _ in range(warmup):
        step()
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
    for e in evs:
        for x in e:
            x.record(s)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for e in evs:
        e[0].record(s)
        code.encode(data, parity, B)
        e[1].record(s)
        code.reconstruct(work, parity, marks, B)
        e[2].record(s)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    enc_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
    dec_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in evs]))
    ok = bool(torch.equal(work[..., :B], data[..., :B]))
    enc_alg, dec_alg = (k + m) * B * G, (k * dec_groups + erased) * B
    out = {"config": f"RS({k},{m}) {flavour}, {G:,} groups x {B} B, {E} random erasures/group",
           "value": round((G + dec_groups) * k * B * steps / el / GIB, 2), "unit": "GiB/s",
           "encode_gibs": round(G * k * B / (enc_ms * 1e-3) / GIB, 2),
           "decode_gibs": round(dec_groups * k * B / (dec_ms * 1e-3) / GIB, 2),
           "encode_frac": round(enc_alg / (enc_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "reconstruct_frac": round(dec_alg / (dec_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "encode_avg_ms": round(enc_ms, 4), "reconstruct_avg_ms": round(dec_ms, 4), "verified": ok}
    del data, parity, work, marks
    torch.cuda.empty_cache()
    return out


CONFIG4 = dict(k=16, m=4, B=1400, E=4)


def skeleton_ratio(data, parity, marks, B, dec_ms, reps=10):
    """The reconstruct against its own memory skeleton (qfec_probe_reconstruct: the auto body's
    mapping, marks reads, survivor rows and erased-row writes, XOR in place of the decode; RS(10,3)
    and RS(16,4) only), timed on a copy of the batch right here: frac_of_skeleton = skeleton time /
    reconstruct time, i.e. how close the reconstruct runs to the ceiling of its access pattern."""
    try:
        skel = data.clone()
        s = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(3):
            qa.probe_reconstruct(skel, parity, marks, B)
        e0.record(s)
        for _ in range(reps):
            qa.probe_reconstruct(skel, parity, marks, B)
        e1.record(s)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        del skel
        return {"skeleton_avg_ms": round(ms, 4), "frac_of_skeleton": round(ms / dec_ms, 4)}
    except qa.QfecError as exc:  # a shape without a skeleton instance
        return {"skeleton_avg_ms": None, "skeleton_error": str(exc)}


def config4_sharded(rank, world, groups=250_000, steps=20, warmup=5, spinup_ms=25.0):
    """BASELINE configs[3]: RS(16,4) encode + decode of 4 000 000 x 1400 B packets = 250 000
    groups, split contiguously over the ranks (quicknet_amd.sharding.shard_range; groups are
    independent, rs.c:582-586, so there is no collective).  Erasures: 4 of 20 per group drawn
    over the whole job (seed 0x5EED0004), so every rank decodes its slice of the same pattern
    list at any N.  Timed on every rank between barriers; value = all ranks' data bytes /
    the slowest rank's time."""
    k, m, B, E = CONFIG4["k"], CONFIG4["m"], CONFIG4["B"], CONFIG4["E"]
    Gt = groups
    a, b = shard_range(Gt, rank, world)
    G = b - a
    dev = torch.device("cuda", torch.cuda.current_device())
    gm = erasure_marks(SEED_RS16, Gt, k + m, E)[a:b]
    code, data, parity, marks, work = _make_batch("cauchy", k, m, B, G, E, rank_seed(SEED_RS16, rank), gm, dev)
    dec_groups = int((gm[:, :k].sum(1) > 0).sum())
    erased = int(gm[:, :k].sum())
    s = torch.cuda.current_stream()

    def step():
        code.encode(data, parity, B)
        code.reconstruct(work, parity, marks, B)

    _spin(step, spinup_ms)
    for _ in range(warmup):
        step()
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
    for e in evs:
        for x in e:
            x.record(s)
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for e in evs:
        e[0].record(s)
        code.encode(data, parity, B)
        e[1].record(s)
        code.reconstruct(work, parity, marks, B)
        e[2].record(s)
    torch.cuda.synchronize()
    barrier(world)
    el_rank = time.perf_counter() - t0
    el = all_max(el_rank, world)
    enc_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
    dec_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in evs]))
    ok = bool(torch.equal(work[..., :B], data[..., :B]))
    ok = all_sum(0.0 if ok else 1.0, world) == 0.0
    skel = skeleton_ratio(data, parity, marks, B, dec_ms) if rank == 0 else {}
    bytes_rank = (G + dec_groups) * k * B * steps
    total = all_sum(float(bytes_rank), world)
    per_rank_ms = all_gather_float(el_rank / steps * 1e3, world, rank)
    enc_alg, dec_alg = (k + m) * B * G, (k * dec_groups + erased) * B
    out = {"config": f"RS({k},{m}) cauchy, {Gt:,} groups x {B} B ({Gt * k:,} packets) split over {world} rank(s), "
                     f"{E} random erasures/group (BASELINE configs[3])",
           "value": round(total / el / GIB, 2), "unit": "GiB/s", "scaling": "strong",
           "ms_per_step": round(el / steps * 1e3, 4), "per_rank_ms": [round(x, 4) for x in per_rank_ms],
           "groups_per_rank": [shard_range(Gt, r, world)[1] - shard_range(Gt, r, world)[0] for r in range(world)],
           "rank0_encode_frac": round(enc_alg / (enc_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "rank0_reconstruct_frac": round(dec_alg / (dec_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "rank0_encode_avg_ms": round(enc_ms, 4), "rank0_reconstruct_avg_ms": round(dec_ms, 4),
           "verified": ok}
    if rank == 0:
        out["rank0_reconstruct_skeleton"] = skel
        # PMC traffic of this rank's launches (tools/pmc_traffic.py --erasures 4, the same shape and
        # group count through bench.py's headline leg; keyed by the rank's group count)
        tr, src = config4_traffic(TRAFFIC_PATH, k, m, B, G, Gt, E)
        if isinstance(tr, dict):
            et, dt = tr.get("encode_bytes_per_launch"), tr.get("reconstruct_bytes_per_launch")
            out["rank0_traffic"] = {"encode_bytes_per_launch": et, "reconstruct_bytes_per_launch": dt,
                                    "encode_traffic_over_alg": round(et / enc_alg, 4) if et else None,
                                    "reconstruct_traffic_over_alg": round(dt / dec_alg, 4) if dt else None}
        out["rank0_traffic_source"] = src
    del data, parity, work, marks
    torch.cuda.empty_cache()
    return out


def config4_traffic(path, k, m, B, G, Gt, E):
    """PMC bytes per launch of config 4's encode and reconstruct at this rank's G groups: the entry
    for G itself, else (N > 1 shards the Gt groups) the whole batch's entry, taken at N = 1 in one
    launch, scaled by G / Gt -- a launch streams each group's rows once, so its bytes scale with
    the groups.  Returns (dict or None, source text)."""
    tr, src = load_traffic(path, f"rs{k}_{m}_b{B}_g{G}_e{E}")
    if tr is not None or G == Gt:
        return tr, src
    full, src0 = load_traffic(path, f"rs{k}_{m}_b{B}_g{Gt}_e{E}")
    if not isinstance(full, dict):
        return None, src
    f = G / Gt
    scaled = dict(full)
    for key in ("encode_bytes_per_launch", "reconstruct_bytes_per_launch"):
        if full.get(key):
            scaled[key] = full[key] * f
    return scaled, f"scaled by {G}/{Gt} groups from {src0}"


def wire_leg(rank, G=100_000, k=10, m=3, S=1024, steps=20, warmup=10, spinup_ms=25.0):
    """SURVEY 8(f) ranks 2-3 in the line: the FEC datagram batches of network/FecCodecBuf.cpp on
    the device, RS(10,13) with 1 KiB payloads (the fec.c matrix the network layer links), 3 of 13
    datagrams lost per group.  Send = qfec_pack_datagrams (shards, checksums, headers, check
    packets); receive = qfec_unpack_datagrams (header and datagram checksums, decode of the first
    k valid rows, dec_src_pkt_info).  Rates count payload bytes; the fractions count the minimal
    traffic (payload in + datagrams out; datagrams received in + data shard rows out) against
    8 TB/s.  Verified: every payload restored byte for byte with status 4 (checksummed)."""
    dev = torch.device("cuda", torch.cuda.current_device())
    n = k + m
    code = qa.Code.vandermonde(k, m)
    payload = torch.empty(G * k * S + 16, dtype=torch.uint8, device=dev)
    qa.synth_fill(payload, rank_seed(SEED_ENCODE ^ 0x77, rank))
    offsets = torch.arange(G * k, dtype=torch.int64, device=dev) * S
    sizes = torch.full((G * k,), S, dtype=torch.int32, device=dev)
    seq = torch.stack([torch.arange(G, dtype=torch.int32, device=dev) * n,
                       torch.arange(G, dtype=torch.int32, device=dev) * k], 1).contiguous()
    lost = torch.from_numpy(erasure_marks(rank_seed(SEED_DECODE ^ 0x77, rank), G, n, m).astype(bool)).to(dev)
    s = torch.cuda.current_stream()
    out = {}  # PMC traffic fields, merged into the leg's record

    def timed(fn):
        _spin(fn, spinup_ms)  # the same clock spin-up as the other legs
        for _ in range(warmup):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(steps):
            r = fn()
        e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / steps, r

    # preallocated outputs, launches straight through the C ABI (no per-call allocation)
    sp = (S + 4 + 15) // 16 * 16
    wp = (sp + 13 + 63) // 64 * 64  # 64-B multiple: the send writes whole lines
    L = qa.lib()
    shards = torch.empty((G, n, sp), dtype=torch.uint8, device=dev)
    wire = torch.empty((G, n, wp), dtype=torch.uint8, device=dev)
    wlen = torch.empty((G, n), dtype=torch.int32, device=dev)
    osh = torch.empty((G, n, sp), dtype=torch.uint8, device=dev)
    marks = torch.empty(G * n, dtype=torch.uint8, device=dev)
    rxs = torch.empty((G, n), dtype=torch.int32, device=dev)
    status = torch.empty((G, k), dtype=torch.int32, device=dev)
    psize = torch.empty((G, k), dtype=torch.int32, device=dev)
    st = s.cuda_stream

    def pack():
        rc = L.qfec_pack_datagrams(code._h, payload.data_ptr(), offsets.data_ptr(), sizes.data_ptr(), seq.data_ptr(), G,
                                   1, shards.data_ptr(), sp, wire.data_ptr(), wp, wlen.data_ptr(), st)
        assert rc == 0, rc

    def unpack():
        rc = L.qfec_unpack_datagrams(code._h, wire.data_ptr(), wp, rx_len.data_ptr(), G, 1, 2068, osh.data_ptr(), sp,
                                     marks.data_ptr(), rxs.data_ptr(), status.data_ptr(), psize.data_ptr(), st)
        assert rc == 0, rc

    pack_ms, _ = timed(pack)
    rx_len = torch.where(lost, torch.zeros_like(wlen), wlen).contiguous()
    unpack_ms, _ = timed(unpack)
    ok = bool((status == 4).all().item()) and bool((psize == S).all().item())
    ok = ok and bool(torch.equal(osh[:, :k, 4:4 + S].reshape(-1), payload[:G * k * S]))
    pay = G * k * S
    pack_traffic = pay + int(wlen.sum().item())
    unpack_traffic = int(rx_len.sum().item()) + G * k * ((S + 4 + 15) // 16 * 16)
    # the same batch straight to / from ProtocolUdp frames in one pass (qfec_pack_frames /
    # qfec_unpack_frames; SessionDesc.cpp:69-77 + ProtocolBasic.cpp:111-199 on every datagram)
    fp = (sp + 13 + 4 + 63) // 64 * 64
    masks = (torch.arange(G * n, dtype=torch.int32, device=dev) * 7 & 0xFF).to(torch.uint8)
    frames = torch.empty((G, n, fp), dtype=torch.uint8, device=dev)
    flen = torch.empty((G, n), dtype=torch.int32, device=dev)
    fst = torch.empty((G, n), dtype=torch.int32, device=dev)

    def pack_frames():
        rc = L.qfec_pack_frames(code._h, payload.data_ptr(), offsets.data_ptr(), sizes.data_ptr(), seq.data_ptr(), G, 1,
                                shards.data_ptr(), sp, masks.data_ptr(), None, 0x3C, 0x11, 0xFF, frames.data_ptr(), fp,
                                flen.data_ptr(), st)
        assert rc == 0, rc

    def unpack_frames():
        rc = L.qfec_unpack_frames(code._h, frames.data_ptr(), fp, rx_flen.data_ptr(), G, 0x3C, 0, 1, 2068,
                                  osh.data_ptr(), sp, marks.data_ptr(), rxs.data_ptr(), status.data_ptr(),
                                  psize.data_ptr(), fst.data_ptr(), None, st)
        assert rc == 0, rc

    pack_frames_ms, _ = timed(pack_frames)
    rx_flen = torch.where(lost, torch.zeros_like(flen), flen).contiguous()
    status.fill_(-9)
    unpack_frames_ms, _ = timed(unpack_frames)
    fok = bool((status == 4).all().item()) and bool((psize == S).all().item()) and bool((fst[~lost] == 0).all().item())
    fok = fok and bool(torch.equal(osh[:, :k, 4:4 + S].reshape(-1), payload[:G * k * S]))
    fok = fok and torch.equal(flen, wlen + 4)
    ok = ok and fok
    pack_frames_traffic = pay + int(flen.sum().item())
    unpack_frames_traffic = int(rx_flen.sum().item()) + G * k * sp
    framed = {"what": "the same batch to ProtocolUdp frames in one pass (qfec_pack_frames: 4-byte prefix, per-datagram "
                      "mask, FEC cmd/protocol) and back (qfec_unpack_frames: RecvPacket verdicts + unpack)",
              "frame_pitch": fp,
              "pack_frames_avg_ms": round(pack_frames_ms, 4), "unpack_frames_avg_ms": round(unpack_frames_ms, 4),
              "pack_frames_gibs": round(pay / (pack_frames_ms * 1e-3) / GIB, 2),
              "unpack_frames_gibs": round(pay / (unpack_frames_ms * 1e-3) / GIB, 2),
              "pack_frames_frac": round(pack_frames_traffic / (pack_frames_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
              "unpack_frames_frac": round(unpack_frames_traffic / (unpack_frames_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
              "pack_frames_min_traffic": pack_frames_traffic, "unpack_frames_min_traffic": unpack_frames_traffic,
              "traffic_basis": "min traffic: payload in + frames out / frames received in + data shard rows out",
              "parity": "framing bytes parity unpinned (ProtocolBasic.cpp does not build here; oracle restatement)",
              "verified": fok}
    wtr, wsrc = load_traffic(TRAFFIC_PATH, f"wire_rs{k}_{n}_s{S}_g{G}", WIRE_KERNEL_SOURCES)
    for key, alg in (("pack", pack_traffic), ("unpack", unpack_traffic), ("pack_frames", pack_frames_traffic),
                     ("unpack_frames", unpack_frames_traffic)):
        t = wtr.get(key) if isinstance(wtr, dict) else None
        tgt = framed if "frames" in key else out
        tgt[f"{key}_traffic"] = t
        tgt[f"{key}_traffic_over_min"] = round(t / alg, 4) if t else None
    out["traffic_source"] = wsrc
    return {"config": f"RS({k},{n}) fec_new (system/fec.c), {G:,} groups x {k} x {S} B payloads, checksums on, "
                     f"{m} of {n} datagrams lost per group",
           "pack_gibs": round(pay / (pack_ms * 1e-3) / GIB, 2), "unpack_gibs": round(pay / (unpack_ms * 1e-3) / GIB, 2),
           "pack_avg_ms": round(pack_ms, 4), "unpack_avg_ms": round(unpack_ms, 4),
           "pack_frac": round(pack_traffic / (pack_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "unpack_frac": round(unpack_traffic / (unpack_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "traffic_basis": "min traffic: payload in + datagrams out / datagrams received in + data shard rows out",
           "framed": framed, "verified": ok, **out}


def zfec_leg(timeout=240):
    """SURVEY 8(f) rank 1 in the line: the exact NetFecCodec layer (include/qfec_zfec.h) --
    64 sender sessions x 2 000 x 1 KiB payloads, RS(10,13), one send flush whose C callback hands
    every datagram it keeps to a receiving context (1 of 13 dropped per group), then one receive
    flush whose C callback folds every delivered payload; the best of reps 1-3 after a warm-up rep
    (tools/zfec_rate.py, its own process).  send_gibs / recv_gibs count payload bytes over each
    flush's wall time.  send_e2e_gibs / recv_e2e_gibs (interleaved reps, field `e2e`) also count the
    per-packet input calls, made from C loops: pack_input for every payload + the send flush, and
    unpack_input for every kept datagram + the receive flush -- the like-for-like figures beside
    the reference's own per-packet pipeline on one core (cpu_baseline.wire), which includes all of
    its per-packet work.  `verified`: delivery count, bytes and word sum, plus a byte-for-byte check
    of every 61st delivery against the payload sent under its source index.  Parity of the
    control flow is unpinned (NetFecCodec.cpp does not build here; tests/test_gpu_zfec.py)."""
    try:
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "zfec_rate.py"), "--json"], capture_output=True,
                           text=True, timeout=timeout)
        lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        if r.returncode != 0 or not lines:
            return {"error": (r.stderr or r.stdout)[-300:], "verified": False}
        out = json.loads(lines[-1])
        out["parity"] = "control flow parity unpinned (oracle/zfec_ref.py restatement); bytes pinned via FecCodecBuf.cpp"
        return out
    except Exception as exc:  # report, never fake
        return {"error": repr(exc), "verified": False}


def per_call_leg(reps=2000, ref_lib=None, batched=True):
    """The unchanged drop-in's per-call cost: what network/FecCodecBuf.cpp pays per
    packet when it links libqfec instead of system/fec.c.  RS(10,3) with 1 KiB payloads:
      fec_encode  one parity packet, sz = 1028 (get_fec_encoded_pkt, FecCodecBuf.cpp:151)
      fec_decode  3 data packets lost, slots in NetFecCodec order (fec_decode_pkts, :204)
    timed per call on the GPU path, plus the batched host-buffer encode (qfec_encode_host) at
    growing batch sizes; with ref_lib (the cpu_baseline leg only) the same calls on the
    reference's own system/fec.c (oracle/_ref, CPU, 1 thread)."""
    import ctypes as C
    k, n, sz = 10, 13, 1028
    rng = np.random.default_rng(11)
    data = rng.integers(0, 256, (n, sz), dtype=np.uint8)
    idx_t = [0, 1, 2, 4, 5, 7, 8, 10, 11, 12]  # data 3, 6, 9 lost; the first k valid rows
    # 64 distinct groups of inputs, cycled, so every group's first fec_encode meets new inputs
    # (libqfec keeps the last group's rows per handle: repeating one group would time its cache)
    groups = rng.integers(0, 256, (64, k, sz), dtype=np.uint8)
    out = {"shape": "RS(10,3), sz 1028 B per packet; encode inputs cycle over 64 distinct groups"}

    def run(lib, tag):
        h = C.c_void_p(lib.fec_new(k, n))
        srcs = [(C.c_void_p * k)(*[groups[g, i].ctypes.data for i in range(k)]) for g in range(64)]
        dst = np.zeros(sz, np.uint8)
        dptr = C.c_void_p(dst.ctypes.data)
        pk_t = (C.c_void_p * k)(*[data[i].ctypes.data for i in idx_t])
        pk = (C.c_void_p * k)()
        ix = (C.c_int * k)()
        ix_t = (C.c_int * k)(*idx_t)
        it = [0]

        def enc():  # one check packet of a new group
            lib.fec_encode(h, srcs[it[0] & 63], dptr, k, sz)
            it[0] += 1

        def grp():  # all n - k check packets of a new group, as get_fec_encoded_pkt asks for them
            s_ = srcs[it[0] & 63]
            for idx in range(k, n):
                lib.fec_encode(h, s_, dptr, idx, sz)
            it[0] += 1

        def dec():
            C.memmove(pk, pk_t, C.sizeof(pk))
            C.memmove(ix, ix_t, C.sizeof(ix))
            lib.fec_decode(h, pk, ix, sz)

        for f, name in ((enc, "fec_encode_us"), (grp, "fec_encode_group_us"), (dec, "fec_decode_us")):
            for _ in range(50):
                f()
            t0 = time.perf_counter()
            for _ in range(reps):
                f()
            out[f"{tag}{name}"] = round((time.perf_counter() - t0) / reps * 1e6, 2)
        lib.fec_free(h)

    if ref_lib is not None:  # the cpu_baseline leg's reference system/fec.c
        run(ref_lib, "ref_cpu_")
        return out
    st0 = qa.percall_stats()
    c0 = qa.percall_counters()
    run(qa.lib(), "gpu_")
    st = qa.percall_stats()
    c1 = qa.percall_counters()
    out["gpu_group_cache"] = {"hits": c1["group_hits"] - c0["group_hits"],
                              "misses": c1["group_misses"] - c0["group_misses"]}
    out["percall_idle_us"] = c1["idle_us"]
    out["gpu_path"] = ("resident server (percall_resident 1, qfec_percall.hpp)" if st["calls"] > st0["calls"]
                       else "one launch per call (qfec_percall.hpp k_percall)")
    out["gpu_server_launches"] = st["launches"] - st0["launches"]
    if not batched:
        return out
    # batched: qfec_encode_host (pinned host buffers in and out) per group vs 3 reference calls
    code = qa.Code.vandermonde(k, n - k)
    batch = []
    for G in (1, 4, 16, 64, 256, 1024):
        hd = torch.from_numpy(rng.integers(0, 256, (G, k, 1040), dtype=np.uint8)).pin_memory()
        hp = torch.empty((G, n - k, 1040), dtype=torch.uint8).pin_memory()
        for _ in range(5):
            code.encode_host(hd, hp, sz)
        r = max(3, min(200, 2000 // G))
        t0 = time.perf_counter()
        for _ in range(r):
            code.encode_host(hd, hp, sz)
        batch.append({"groups": G, "us_per_group": round((time.perf_counter() - t0) / r / G * 1e6, 3)})
    out["batched_encode_host"] = batch
    return out


def load_traffic(path, workload_key, sources=KERNEL_SOURCES):
    """PMC bytes per launch for this workload from profiles/traffic.json, or None when absent
    or measured on other kernel sources (the file records their sha256)."""
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None, "absent"
    ent = t.get(workload_key)
    if not isinstance(ent, dict):
        return None, "no entry for this workload"
    want = kernel_sources_hash(sources)
    if ent.get("kernel_sources_sha256") != want:
        return None, f"stale: measured on kernel sources {ent.get('kernel_sources_sha256')}, now {want}"
    run = ent.get("run", "PMC run")
    # the counter CSVs behind the entry, as tracked in the repository (the entry names them; they
    # are not shipped to the GPU box, so their presence here says nothing)
    csv = ent.get("csv") or f"profiles/{run}/pmc"
    return ent, f"{os.path.relpath(path, ROOT)} ({run}, kernel sources {want}; counter CSVs {csv}/)"


def kernel_sources_hash(sources=KERNEL_SOURCES):
    h = hashlib.sha256()
    for f in sources:
        with open(os.path.join(ROOT, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if (args.gpus > 1 or args.launch_check) and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args, argv)
    rank, world, local, numa = dist_setup(args)
    if args.protocol_check:
        rc = protocol_check(args, rank, world)
        if _dist_on():
            import torch.distributed as dist
            dist.destroy_process_group()
        return rc
    qa.set_kernel_variant(args.variant)
    if args.config4_only:  # measurement helper: the config 4 leg's launches alone, under a profiler
        c4 = config4_sharded(rank, world, args.config4_groups, steps=args.steps, warmup=args.warmup)
        if rank == 0:
            print(json.dumps({"config4": c4}), flush=True)
        return 0 if c4["verified"] else 1
    dev = torch.device("cuda", local)
    k, m, B, G, E = args.k, args.m, args.block, args.groups, args.erasures
    n = k + m
    code = qa.Code.cauchy(k, m) if args.flavour == "cauchy" else qa.Code.vandermonde(k, m)
    stream = torch.cuda.current_stream()

    data = torch.empty((G, k, B), dtype=torch.uint8, device=dev)
    qa.synth_fill(data, rank_seed(SEED_ENCODE, rank))
    parity = torch.empty((G, m, B), dtype=torch.uint8, device=dev)
    gm = erasure_marks(rank_seed(SEED_DECODE, rank), G, n, E)
    marks = torch.from_numpy(marks_to_rs_layout(gm, k)).to(dev)
    dec_groups = int((gm[:, :k].sum(1) > 0).sum())
    erased_data = int(gm[:, :k].sum())
    work = data.clone()  # the damaged copy reconstruct rewrites
    work[torch.from_numpy(gm[:, :k].astype(bool)).to(dev)] = 0x5A
    code.encode(data, parity)
    code.prepare_reconstruct()
    torch.cuda.synchronize()

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        code.encode(data, parity)
        if ev is not None:
            ev[1].record(stream)
        code.reconstruct(work, parity, marks)
        if ev is not None:
            ev[2].record(stream)

    # setup, untimed: a fresh GPU runs the first ~20 steps (~10 ms) 5-8 % slower while its
    # clocks leave the idle state (profiles/r01t_sustain.txt); spin it up before the W
    # warmup steps so the timed region sees the steady state whatever W the caller picks
    _spin(step, args.spinup_ms)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # timed region: K steps between barrier + synchronize on both sides
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    for e in evs:  # torch creates the HIP event at its first record: do that outside the timed region
        for x in e:
            x.record(stream)
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(evs[i])
    torch.cuda.synchronize()
    barrier(world)
    t1 = time.perf_counter()
    el = all_max(t1 - t0, world)
    per_rank_ms = all_gather_float((t1 - t0) / args.steps * 1e3, world, rank)
    enc_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
    dec_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in evs]))

    # correctness guard on the measured buffers: reconstruct restored the data exactly
    ok = bool(torch.equal(work, data))
    ok = all_sum(0.0 if ok else 1.0, world) == 0.0

    data_bytes_rank = (G + dec_groups) * k * B * args.steps
    total_bytes = all_sum(float(data_bytes_rank), world)
    value = total_bytes / el / GIB

    enc_alg = (k + m) * B * G                      # read k shards, write m
    dec_alg = (k * dec_groups + erased_data) * B   # read k survivors, write e erased
    enc_gbs = enc_alg / (enc_ms * 1e-3) / 1e9
    dec_gbs = dec_alg / (dec_ms * 1e-3) / 1e9
    traffic, traffic_src = load_traffic(args.traffic, f"rs{k}_{m}_b{B}_g{G}")

    def roof(kernel, ach, alg, ms, tkey):
        tr = traffic.get(tkey) if isinstance(traffic, dict) else None
        return {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": tr, "traffic_source": traffic_src,
                "kernel": kernel, "algorithmic_bytes": alg, "avg_ms": round(ms, 4),
                "read_frac": round((alg - (m * B * G if kernel == "encode" else erased_data * B)) / (ms * 1e-3) / 1e9
                                   / HBM_PEAK_GBS, 4)}

    r_enc = roof("encode", enc_gbs, enc_alg, enc_ms, "encode_bytes_per_launch")
    r_dec = roof("reconstruct", dec_gbs, dec_alg, dec_ms, "reconstruct_bytes_per_launch")
    dominant, other = (r_enc, r_dec) if enc_ms >= dec_ms else (r_dec, r_enc)

    # calibration probe: the encode's traffic with XOR only (not a codec)
    probe_ms = copy_gbs = None
    if rank == 0:
        pe0, pe1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        scratch = torch.empty_like(parity)
        for _ in range(3):
            qa.probe_stream(data, scratch, B)
        pe0.record(stream)
        for _ in range(10):
            qa.probe_stream(data, scratch, B)
        pe1.record(stream)
        torch.cuda.synchronize()
        probe_ms = pe0.elapsed_time(pe1) / 10
        del scratch
        # achievable-peak references: the XOR probe above moves the encode's
        # exact traffic; a plain device-to-device copy of the data batch is the other one
        probe_gbs = enc_alg / (probe_ms * 1e-3) / 1e9
        for r in (r_enc, r_dec):
            r["frac_of_probe"] = round(r["achieved"] / probe_gbs, 4)
        r_dec.update(skeleton_ratio(data, parity, marks, B, dec_ms))
        cdst = torch.empty_like(data)
        for _ in range(3):
            cdst.copy_(data)
        pe0.record(stream)
        for _ in range(10):
            cdst.copy_(data)
        pe1.record(stream)
        torch.cuda.synchronize()
        copy_gbs = 2 * data.numel() / (pe0.elapsed_time(pe1) / 10 * 1e-3) / 1e9
        del cdst
    del work, marks
    torch.cuda.empty_cache()

    # BASELINE configs[3] on every rank (strong scaling over the ranks)
    config4 = None
    if not args.no_config4:
        config4 = config4_sharded(rank, world, args.config4_groups)
        ok = ok and config4["verified"]

    # BASELINE configs[4] (host -> device -> host) on every rank, and the single-shape
    # host-inclusive encode on rank 0; both verified byte for byte
    host_mixed = host_line = host_sample = None
    if not args.no_host:
        from quicknet_amd.hoststream import host_encode_leg, host_mixed_leg
        host_mixed = host_mixed_leg(rank, world, barrier, all_max, all_sum, all_gather_float,
                                    sample_groups=64 if rank == 0 and world == 1 and not args.no_cpu else 0)
        host_sample = host_mixed.pop("_sample", None)
        ok = ok and bool(host_mixed.get("verified"))
        # the same stream through the staged copies, for comparison (not the field's value)
        staged = host_mixed_leg(rank, world, barrier, all_max, all_sum, all_gather_float, passes=2, zero_copy=False)
        ok = ok and bool(staged.get("verified"))
        host_mixed["staged"] = {x: staged.get(x) for x in ("value", "verified", "pcie_gbs_per_rank", "h2d_gbs_per_rank",
                                                          "d2h_gbs_per_rank", "error") if x in staged}
        if rank == 0:
            host_line = host_encode_leg(code, data, parity, B)
            ok = ok and bool(host_line.get("verified"))

    # module/rs.h unchanged on host shard pointers (the reference's own batched interface), rank 0
    rs_host = rs_host_sample = None
    if rank == 0 and not args.no_host:
        from quicknet_amd.hoststream import rs_abi_host_leg
        try:
            rs_host = rs_abi_host_leg()
            rs_host_sample = rs_host.pop("_sample", None)
        except Exception as exc:  # report, never fake
            rs_host = {"error": repr(exc), "verified": False}
        ok = ok and bool(rs_host.get("verified"))

    per_call = None
    if rank == 0 and not args.no_host:
        try:
            per_call = per_call_leg()
        except Exception as exc:  # report, never fake
            per_call = {"error": repr(exc)}

    side = wire = zfec = None
    if rank == 0 and not args.no_side:
        side = [side_config(fl, sk, sm, sB, sG, sE, rank) for fl, sk, sm, sB, sG, sE in SIDE]
        try:
            wire = wire_leg(rank)
        except Exception as exc:  # report, never fake
            wire = {"error": repr(exc), "verified": False}
        ok = ok and bool(wire.get("verified"))
        ok = ok and all(x["verified"] for x in side)
        zfec = zfec_leg()
        ok = ok and bool(zfec.get("verified"))

    cpu = cpu_mt = None
    if rank == 0 and world == 1 and not args.no_cpu:
        try:
            cpu = cpu_baseline(args, args.cpu_seconds)
        except Exception as exc:  # report, never fake
            cpu = {"value": None, "error": repr(exc)}
        threads = topology.cpu_share()["usable"] if args.cpu_threads is None else args.cpu_threads
        if threads > 0:
            try:
                cpu_mt = cpu_baseline_threads(args, args.cpu_seconds / 2, threads)
            except Exception as exc:
                cpu_mt = {"value": None, "error": repr(exc)}
        try:
            cpu["config0"] = cpu_config0(args.cpu_seconds / 5)
        except Exception as exc:
            cpu["config0"] = {"error": repr(exc)}
        try:  # the reference's per-packet calls, beside the GPU drop-in's (per_call)
            from oracle.oracle import RefCodec
            if RefCodec.available():
                cpu["per_call"] = per_call_leg(ref_lib=RefCodec().fec)
                if isinstance(per_call, dict) and "batched_encode_host" in per_call:
                    ref3 = 3 * cpu["per_call"]["ref_cpu_fec_encode_us"]
                    beat = [b["groups"] for b in per_call["batched_encode_host"] if b["us_per_group"] < ref3]
                    per_call["batch_beats_reference_encode_at_groups"] = beat[0] if beat else None
                if isinstance(per_call, dict) and "gpu_fec_encode_group_us" in per_call:
                    # the unchanged caller's group of n - k fec_encode calls, GPU over CPU reference
                    ref_g = cpu["per_call"].get("ref_cpu_fec_encode_group_us")
                    if ref_g:
                        per_call["group_vs_reference"] = round(per_call["gpu_fec_encode_group_us"] / ref_g, 3)
        except Exception as exc:
            cpu["per_call"] = {"error": repr(exc)}
        if rs_host_sample is not None:  # the checker role: the rs.h host path against the reference rs.c
            try:
                rs_host["reference_check"] = cpu_check_rs_sample(rs_host_sample)
                ok = ok and bool(rs_host["reference_check"].get("match"))
            except Exception as exc:
                rs_host["reference_check"] = {"error": repr(exc)}
                rs_host["verified"] = False
                ok = False
            for tag, base in (("vs_cpu_1thread", cpu), ("vs_cpu_threads", cpu_mt)):
                if isinstance(base, dict) and base.get("value") and rs_host.get("value"):
                    rs_host[tag] = round(rs_host["value"] / base["value"], 2)
        if host_sample is not None:  # the checker role: config 5's output against the reference rs.c
            try:
                host_mixed["reference_check"] = cpu_check_host_sample(host_sample)
                ok = ok and bool(host_mixed["reference_check"].get("match"))
            except Exception as exc:  # a checker that could not run verifies nothing
                host_mixed["reference_check"] = {"error": repr(exc)}
                host_mixed["verified"] = False
                ok = False
        # the reference's datagram pipeline (FecCodecBuf.cpp + system/fec.c, oracle/_ref),
        # RS(10,13) 1 KiB payloads, send + receive, 1 thread: the CPU side of DESIGN 3.5
        ref_wire = os.path.join(ROOT, "oracle", "_ref", "ref_wire_bench")
        if cpu is not None and os.path.exists(ref_wire):
            try:
                r = subprocess.run([ref_wire, "10", "13", "1024", "2000", str(args.cpu_seconds / 5)],
                                   capture_output=True, text=True, timeout=120)
                cpu["wire"] = json.loads(r.stdout) if r.returncode == 0 else {"error": r.stderr[-200:]}
            except Exception as exc:
                cpu["wire"] = {"error": repr(exc)}

    host_cpus = topology.cpu_share()
    nn = numa.get("numa_node") if isinstance(numa, dict) else None
    per_rank_numa = [int(x) for x in all_gather_float(float(-1 if nn is None else nn), world, rank)]
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 4),
            "per_rank_ms": [round(x, 4) for x in per_rank_ms],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (splitmix64 bytes, device-generated), seeds 0x5EED0002/0x5EED0003 per rank",
            "config": {
                "workload": f"RS({k},{m}) encode of {G * k:,} x {B} B packets ({G:,} groups) + reconstruct with "
                            f"{E} random erasures/group, per GPU (BASELINE configs[1]+[2])",
                "k": k, "m": m, "block_size": B, "groups_per_gpu": G, "erasures_per_group": E,
                "flavour": "cauchy (module/rs.c)" if args.flavour == "cauchy" else "vandermonde (module/fec.c)",
                "kernel_variant": ["perm", "ldslog"][args.variant],
                "parallelism": f"groups sharded, {world} rank(s), no collective on the data path",
            },
            "encode_gibs": round(G * k * B / (enc_ms * 1e-3) / GIB, 2),
            "decode_gibs": round(dec_groups * k * B / (dec_ms * 1e-3) / GIB, 2),
            "roofline": dominant,
            "roofline_other": other,
            "probe_stream_gbs": round(enc_alg / (probe_ms * 1e-3) / 1e9, 1) if probe_ms else None,
            "copy_d2d_gbs": round(copy_gbs, 1) if copy_gbs else None,
            "config4": config4,
            "host_to_host_mixed": host_mixed,
            "host_to_host_encode": host_line,
            "rs_abi_host": rs_host,
            "per_call": per_call,
            "verified": ok,
            "cpu_baseline": cpu,
            "cpu_baseline_threads": cpu_mt,
            "host_cpus": host_cpus,
            "per_rank_numa": per_rank_numa,
            "numa_binding_rank0": numa,
            "process_group": torch.distributed.get_backend() if _dist_on() else None,
            "side_configs": side,
            "wire": wire,
            "zfec": zfec,
        }
        print(json.dumps(out), flush=True)
    if _dist_on():
        import torch.distributed as dist
        barrier(world)  # the other ranks wait for rank 0's side configurations, then all tear down
        dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
