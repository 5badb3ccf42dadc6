"""Group partitioning across GPUs.

(k+m)-shard groups are independent in both reference codecs (module/rs.c:582-586 loops
groups with no shared state; fec_encode/fec_decode work per group), so G groups split into
contiguous per-device ranges with no collective on the data path.  The only cross-rank
traffic is the timing protocol of bench.py (a barrier and a max over ranks).
"""


def shard_range(groups: int, rank: int, world: int):
    """[start, stop) of rank's contiguous share: floor(G/D), +1 for the first G mod D ranks."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(groups, world)
    start = rank * base + min(rank, extra)
    stop = start + base + (1 if rank < extra else 0)
    return start, stop


def rank_seed(seed: int, rank: int) -> int:
    """Per-rank synthetic stream for weak scaling (each rank owns distinct groups)."""
    return (seed + 0x1000_0000 * rank) & 0xFFFFFFFFFFFFFFFF


def aggregate_rate(units_per_rank, seconds_per_rank):
    """Whole-job throughput: all units over the slowest rank's time."""
    return sum(units_per_rank) / max(seconds_per_rank)
