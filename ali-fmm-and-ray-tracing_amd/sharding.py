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


def max_over_ranks(value, dist=None):
    """Max of a float over all ranks of the default process group (identity without one)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(value)
    import torch

    t = torch.tensor([float(value)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
