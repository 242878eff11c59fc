"""Source sharding over GPUs.

Every source's travel-time field is independent (the reference's process pool hands out whole
sources: parallel_TTF / parallel_TTF_rays, Anis_TTF_rays.py:3560-3733), so sources are dealt
to devices or ranks with no data-path exchange; rays (i, j) run where receiver j's field lives
(parallel_TTF_rays :3715-3733).
"""
import numpy as np


def deal(items, n_parts):
    """Block-cyclic deal of `items` over n_parts (part k gets items[k::n_parts])."""
    items = list(items)
    n_parts = max(1, int(n_parts))
    return [items[k::n_parts] for k in range(n_parts)]


def bench_sources(rank, n_sources, n, dnx):
    """C4 sources of one bench rank (weak scaling: every rank runs n_sources top-surface sources).

    x = 16 + 32 k + 4 (rank mod 8), z = 0, k = 0 .. n_sources-1 (wrapped over the n/32 columns);
    rank 0 gets exactly BASELINE C4's sources; ranks 0..7 never share a source.
    """
    k = np.arange(n_sources) % (n // 32)
    scx = dnx * (16 + 32 * k + 4 * (rank % 8)).astype(np.float64)
    scz = np.zeros(n_sources)
    return scx, scz


def gather_plan(n_sources, world):
    """Where bench.py's strong deal puts every source after the RCCL gather to rank 0: rank r holds
    sources deal(range(n_sources), world)[r] in its slots 0, 1, ...; alifmm_gather_fields stacks
    them on the root rank after rank (slot offset sum(count[:r]) + k, _alifmm.gather_layout).
    Returns (counts, root_slot_of_source)."""
    parts = deal(range(n_sources), world)
    counts = [len(p) for p in parts]
    off = np.concatenate(([0], np.cumsum(counts)))[:-1]
    slot = np.empty(n_sources, dtype=np.int64)
    for r, p in enumerate(parts):
        slot[p] = off[r] + np.arange(len(p))
    return counts, slot
