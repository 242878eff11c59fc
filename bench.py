"""Benchmark: grid-cell updates/s + sources/s on the 4096^2 anisotropic weld-like grid (BASELINE.json).

One process per GPU (python -m torch.distributed.run ... bench.py --gpus N).  A "step" is one
pass of the hot path over one batch: first-arrival travel-time fields for the rank's sources
(BASELINE C4: 128 sources on the top surface per GPU, subgrid 1), inputs resident in HBM, fields
left resident in HBM (the ray tracer reads them there).  Sources are independent: each rank
computes its own shard (weak scaling), no data-path collective; torch.distributed (gloo) only
provides the barrier and the max-over-ranks of the step time.

Reported: value = all ranks' (cells x sources) / max-over-ranks wall time of the timed steps;
roofline of the dominant kernel (the band kernel: fmm_band_pair_kernel, two workgroups per source,
when the batch fits the device, else fmm_band_kernel) from in-library HIP events on its stream; cpu_baseline = the
CPU restatement of the reference (oracle/, one source per thread) on a bounded sample, rank 0, N=1.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "ali-fmm-and-ray-tracing_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s
# algorithmic bytes per cell-sweep (one local-operator evaluation on the band front), DESIGN.md §5:
# T f64 read+write 16, status int32 read+write 8, material (veln f64, vel_map f64, velpn i32, stiffness idx i32) 24
BYTES_PER_SWEEP = 48


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n", type=int, default=4096, help="grid side (4096 = BASELINE C4)")
    ap.add_argument("--sources", type=int, default=128, help="sources per GPU (BASELINE C4: 128)")
    ap.add_argument("--cpu-sample", type=int, default=16, help="sources in the CPU-baseline sample (0: skip)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cdelta", type=float, default=None)
    ap.add_argument("--exact-r", type=float, default=None)
    ap.add_argument("--no-cpu", action="store_true")
    return ap.parse_args()


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("gloo", rank=rank, world_size=world)

    import _alifmm
    import sharding
    import workloads as W

    n = args.n
    veln, velpn, vel_map, stif = W.weldlike_model(n)
    dnx = W.weldlike_dnx()
    vt = W.default_table()
    # one GPU per rank (LOCAL_RANK); ALIFMM_BENCH_DEVICE pins every rank to one device, only to
    # rehearse the multi-process path on a one-GPU box
    dev = int(os.environ.get("ALIFMM_BENCH_DEVICE", local))
    ctx = _alifmm.Context(dev)
    if args.cdelta is not None:
        ctx.set_option("cdelta", args.cdelta)
    if args.exact_r is not None:
        ctx.set_option("exact_r", args.exact_r)
    ctx.set_model(veln, velpn, vel_map, stif, vt, vt, dnx)
    scx, scz = sharding.bench_sources(rank, args.sources, n, dnx)

    def barrier():
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        ctx.travel(scx, scz, subgrid=1, first_slot=0, copy_out=False)
    barrier()
    t0 = time.perf_counter()
    band_ms = init_ms = 0.0
    for _ in range(args.steps):
        ctx.travel(scx, scz, subgrid=1, first_slot=0, copy_out=False)
        ti, tb, _ = ctx.last_timing()
        init_ms += ti
        band_ms += tb
    barrier()
    dt = time.perf_counter() - t0
    sweeps = sum(ctx.source_stats(i)[1] for i in range(args.sources))
    band_kernel = "fmm_band_pair_kernel" if int(ctx.get_option("last_pair")) else "fmm_band_kernel"
    steps_main = [int(ctx.source_stats(i)[0][3]) for i in range(args.sources)]
    dt = sharding.max_over_ranks(dt, dist)
    cells = float(n) * n
    total_src = args.sources * world
    value = cells * total_src * args.steps / dt
    band_avg_s = band_ms / args.steps / 1e3
    achieved = BYTES_PER_SWEEP * sweeps / band_avg_s / 1e9 if band_avg_s > 0 else None

    config = {"workload": "C4: %dx%d weld-like, %d top-surface Tx sources per GPU, subgrid 1" % (n, n, args.sources),
              "sources_per_gpu": args.sources, "total_sources": args.sources * world, "grid": [n, n], "subgrid": 1,
              "cdelta": args.cdelta, "exact_r": args.exact_r}
    # HBM-side bytes per launch: PMC passes of tools/profile.sh on this library AND this workload
    traffic = traffic_bytes = None
    try:
        import glob
        import hashlib

        lib_sha = hashlib.sha256(open(_alifmm.LIB_PATH, "rb").read()).hexdigest()
        for f in sorted(glob.glob(os.path.join(REPO, "profiles", "*_traffic.json"))):
            t = json.load(open(f))
            if (t.get("libalifmm_sha256") == lib_sha and t.get("traffic_bytes_per_launch")
                    and t.get("bench_config") == {k: v for k, v in config.items() if k != "total_sources"}):
                traffic_bytes = t["traffic_bytes_per_launch"]
                traffic = traffic_bytes / band_avg_s / 1e9  # GB/s over the same launch time as achieved
    except OSError:
        pass

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu and args.cpu_sample > 0:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle as O

        ns = args.cpu_sample
        th = min(args.cpu_threads, ns)
        t1 = time.perf_counter()
        O.travel_batch(scx[:ns], scz[:ns], veln, velpn, vel_map, stif, vt, vt, dnx=dnx, n_threads=th)
        tc = time.perf_counter() - t1
        model = ""
        try:
            model = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
        except (OSError, StopIteration):
            pass
        cpu = {"value": cells * ns / tc, "unit": "grid-cell updates/s", "cores": th, "kind": "port",
               "host_cpu": model, "host_cpus_visible": os.cpu_count(), "seconds_per_source_per_core": tc * th / ns,
               "sample": "%d C4 sources (4096^2, z=0) on %d threads, one source per thread, oracle/alifmm_oracle.c "
                         "(bit-exact restatement of the reference's heap FMM); %.1f s wall" % (ns, th, tc)}
    if rank == 0:
        out = {
            "metric": "grid-cell updates/sec + sources/sec on 4096^2 anisotropic grid",
            "value": value,
            "unit": "grid-cell updates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: weld-like model built from the reference's weld_*.npy (edge-padded, 8x nearest), "
                    "stiffness row of the notebook",
            "config": config,
            "sources_per_s": total_src * args.steps / dt,
            "kernel_ms_per_step": {"fmm_init_kernel": init_ms / args.steps, band_kernel: band_ms / args.steps},
            "band_steps_main_mean": float(np.mean(steps_main)),
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": (achieved / HBM_PEAK_GBS) if achieved else None, "traffic": traffic,
                         "kernel": band_kernel, "bytes_per_cell_sweep": BYTES_PER_SWEEP,
                         "cell_sweeps_per_launch": int(sweeps),
                         "algorithmic_bytes_per_launch": BYTES_PER_SWEEP * int(sweeps),
                         "traffic_bytes_per_launch": traffic_bytes},
            "cpu_baseline": cpu,
        }
        if cpu:
            out["speedup_vs_cpu_baseline"] = value / cpu["value"]
        print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main()
