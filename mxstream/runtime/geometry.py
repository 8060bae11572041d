"""Keyed-state geometry: how many LDS-sized hash sub-tables and how large.

A sub-table is owned by one workgroup per step (window_agg) and is the unit of the keyBy
partition buckets, so the count sets both the aggregation parallelism (>= ~256 workgroups fill
the 256 CUs) and the number of scatter buckets (the write-combined partition handles <= 512 per
rank x destination). The slot count per sub-table is sized to its share of keys at <= 0.7 load
(linear probing in LDS: ~2.2 probes per hit), between 64 and 4096 slots (32 KB of keys in LDS).
"""
from __future__ import annotations

import math

MIN_SUBTABLES_NODE = 256   # across all ranks of the node
MAX_CAP_LOG2 = 12
MIN_CAP_LOG2 = 6


def _next_pow2(x: int) -> int:
    return 1 << max(0, int(x - 1).bit_length())


def state_geometry(max_keys: int, world: int, cap_log2: int | None = None) -> tuple[int, int]:
    """Return (nsub, cap_log2) for one rank."""
    per_rank = int(max_keys / world * (1.3 if world > 1 else 1.0)) + 64
    if cap_log2 is not None and cap_log2 < 9:
        # Explicit small tables (tests): fixed capacity, load <= 0.5.
        nsub = _next_pow2(max(1, math.ceil(per_rank / ((1 << cap_log2) * 0.5))))
        return nsub, cap_log2
    load = 0.7
    nsub = _next_pow2(max(1, math.ceil(per_rank / ((1 << MAX_CAP_LOG2) * load))))
    nsub = max(nsub, _next_pow2(max(1, MIN_SUBTABLES_NODE // world)))
    need = per_rank / nsub / load
    cl = max(MIN_CAP_LOG2, min(MAX_CAP_LOG2, int(math.ceil(math.log2(max(need, 2))))))
    # Binomial spread between sub-tables: keep >= 4 sigma of headroom at small shares.
    mean = per_rank / nsub
    while cl < MAX_CAP_LOG2 and mean + 4 * math.sqrt(mean) + 8 > (1 << cl) * 0.85:
        cl += 1
    return nsub, cl


def fixed_geometry(max_keys: int, world: int, cap_log2: int) -> tuple[int, int]:
    """(nsub, cap_log2) for a fixed sub-table size: as many sub-tables as that size needs at
    <= 0.7 load (at least MIN_SUBTABLES_NODE over the node)."""
    per_rank = int(max_keys / world * (1.3 if world > 1 else 1.0)) + 64
    cl = max(MIN_CAP_LOG2, min(MAX_CAP_LOG2, int(cap_log2)))
    nsub = _next_pow2(max(1, math.ceil(per_rank / ((1 << cl) * 0.7))))
    return max(nsub, _next_pow2(max(1, MIN_SUBTABLES_NODE // world))), cl
