"""Multi-rank path on CPU (gloo, world_size 2): groups shard contiguously across ranks with
no data-path collective, the sharded result equals the single-rank result, and the job
throughput is all ranks' units over the slowest rank's time (bench.py's protocol)."""
import hashlib
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from quicknet_amd.sharding import aggregate_rate, rank_seed, shard_range
from quicknet_amd.synth import synth_bytes


def test_shard_range_covers_exactly():
    for G in (0, 1, 7, 100_000, 250_000):
        for D in (1, 2, 3, 4, 8):
            spans = [shard_range(G, r, D) for r in range(D)]
            assert spans[0][0] == 0 and spans[-1][1] == G
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b == c
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


def test_rank_seeds_distinct():
    seeds = {rank_seed(0x5EED0002, r) for r in range(8)}
    assert len(seeds) == 8


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, G, k, m, B, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle.oracle import Oracle
    orc = Oracle()
    rows = orc.cauchy(k, m)
    a, b = shard_range(G, rank, world)
    data = synth_bytes(99, G * k * B).reshape(G, k, B)[a:b].copy()  # each rank owns its groups
    par = np.zeros((b - a, m, B), np.uint8)
    dist.barrier()
    import time
    t0 = time.perf_counter()
    orc.rs_encode(rows, data, par, B)
    el = time.perf_counter() - t0
    dist.barrier()
    t = torch.tensor([el], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    units = torch.tensor([float(b - a)], dtype=torch.float64)
    dist.all_reduce(units, op=dist.ReduceOp.SUM)
    # gather parity only to check the result (not part of the data path)
    gathered = [None] * world
    dist.all_gather_object(gathered, par.tobytes())
    if rank == 0:
        out.put((float(t.item()), float(units.item()), b"".join(gathered)))
    dist.destroy_process_group()


def test_gloo_two_ranks_match_single():
    G, k, m, B, world = 64, 10, 3, 256, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, G, k, m, B, q)) for r in range(world)]
    for p in procs:
        p.start()
    tmax, units, blob = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from oracle.oracle import Oracle
    orc = Oracle()
    data = synth_bytes(99, G * k * B).reshape(G, k, B)
    par = np.zeros((G, m, B), np.uint8)
    orc.rs_encode(orc.cauchy(k, m), data, par, B)
    assert hashlib.sha256(blob).digest() == hashlib.sha256(par.tobytes()).digest()
    assert units == G and tmax > 0
    assert aggregate_rate([32, 32], [1.0, 2.0]) == 32.0


def _bench_helpers_worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench  # the same helpers bench.py's timed region uses (gloo: host tensors)
    bench.barrier(world)
    el = bench.all_max(0.5 + rank, world)                 # the slowest rank's time
    ok = bench.all_sum(0.0 if rank != 1 else 1.0, world)  # one rank failed verification
    total = bench.all_sum(float(100 * (rank + 1)), world)  # all ranks' bytes
    if rank == 0:
        out.put((el, ok, total))
    dist.destroy_process_group()


def test_bench_reductions_over_gloo():
    """bench.py's barrier / max-over-ranks time / summed bytes, run as two gloo ranks: the
    job value is all ranks' bytes over the slowest rank's time, and one rank's failed check
    makes the whole line fail."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_helpers_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    el, ok, total = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert (el, ok, total) == (1.5, 1.0, 300.0)
