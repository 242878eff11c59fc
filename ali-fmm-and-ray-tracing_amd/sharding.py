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


def gather_fields(ctx, n_local, fnz, fnx, rank, world, device, first_slot=0):
    """RCCL gather of every rank's resident fields to rank 0 (the result-return leg of bench.py).

    Each rank copies its n_local fields device-to-device into one contiguous buffer
    (alifmm_copy_fields, kind 2) and joins one dist.gather over an RCCL ("nccl") group onto rank
    0's device; ranks with fewer fields pad to the largest count.  torch is imported before the
    library is loaded (bench.py), so both share one HIP runtime and device pointers are valid
    in both.  Returns the timings (max over ranks) and rates of the two parts."""
    import time

    import torch
    import torch.distributed as dist

    torch.cuda.set_device(device)
    g = dist.new_group(backend="nccl")
    counts = torch.tensor([n_local], dtype=torch.int64)
    cmax = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(cmax, counts)
    nmax = int(max(int(c) for c in cmax))
    buf = torch.empty((nmax, fnz, fnx), dtype=torch.float64, device="cuda")
    recv = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
    dist.barrier(group=g)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    d2d_gbps = ctx.copy_fields_to_device(first_slot, n_local, buf.data_ptr()) if n_local else 0.0
    t1 = time.perf_counter()
    dist.gather(buf, recv, dst=0, group=g)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    copy_s = max_over_ranks(t1 - t0, dist)
    gather_s = max_over_ranks(t2 - t1, dist)
    total = int(sum(int(c) for c in cmax)) * fnz * fnx * 8
    remote = total - n_local * fnz * fnx * 8 if rank == 0 else 0
    remote = int(max_over_ranks(remote, dist))
    del recv, buf
    dist.destroy_process_group(g)
    return {"pack_d2d_ms": copy_s * 1e3, "pack_d2d_GBps": d2d_gbps, "rccl_gather_ms": gather_s * 1e3,
            "rccl_gather_bytes_into_rank0": remote,
            "rccl_gather_GBps_into_rank0": remote / gather_s / 1e9 if gather_s > 0 else None}


def max_over_ranks(value, dist=None):
    """Max of a float over all ranks of the default process group (identity without one)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(value)
    import torch

    t = torch.tensor([float(value)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
