"""Benchmark: grid-cell updates/s + sources/s on the 4096^2 anisotropic weld-like grid (BASELINE.json,
config 4: "4096x4096 weld-like grid, 128 Tx sources sharded across 1/2/4/8 MI355X").

One process per GPU: `python bench.py --gpus N` spawns its N ranks itself (launch_ranks; it refuses
when fewer than N GPUs are visible), or runs as one rank of an outside launcher (python -m
torch.distributed.run ... bench.py --gpus N, WORLD_SIZE set).  n_gpus = the ranks that ran.  The 128 C4 sources
(z = 0, x = 16 + 32 k) are dealt block-cyclically over the N ranks, as the
reference's update_parallel hands whole sources to its workers (Anis_TTF_rays.py:3938-4051), so
the total work is fixed and the curve over N is STRONG scaling; --weak gives every rank its own
128 sources instead.  A "step" is one pass of the hot path over the rank's sources: their
first-arrival travel-time fields (inputs resident in HBM, fields left resident in HBM, where the
ray tracer reads them).  Sources are independent: no data-path collective; torch.distributed
(gloo) only provides the barrier and the max over ranks of the step time.

value = 128 x 4096^2 cell-updates x steps / max-over-ranks wall time of the timed steps.
roofline: the band kernel (fmm_band_k_kernel), SURVEY §8(d)'s 18.1 algorithmic bytes per
cell-sweep (one evaluation of the local operator, counted by the kernel) over the kernel's
in-library HIP-event time on its stream; traffic = HBM bytes per launch from rocprofv3 PMC
passes of the same library build (profiles/*_traffic.json), with traffic / algorithmic.
result_return: after the timed steps, the fields' way back (not in value): D2H into pageable
host memory through the library's pinned staging ring, every rank at once; with --gather (N > 1)
also an RCCL gather of every rank's fields to rank 0 over xGMI.
cpu_baseline: the CPU restatement of the reference (oracle/, one source per thread) on a bounded
sample, rank 0, N = 1.
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
VALU_SIMDS = 256 * 4  # 256 CUs x 4 SIMDs
CLOCK_HZ = 2.4e9      # peak engine clock
# algorithmic bytes per cell-sweep (T f32 read + write 8, orientation 4,
# vel_map 4, material id 1, halo 1.06)
BYTES_PER_SWEEP = 18.1
# per-core speed of the C restatement over the numba reference on C3 (2048^2, one source), both
# measured in the build container: 8.69 s (numba) / 3.73 s (oracle/alifmm_oracle.c)
PORT_VS_REFERENCE_PER_CORE = 8.69 / 3.73


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n", type=int, default=4096, help="grid side (4096 = BASELINE C4)")
    ap.add_argument("--sources", type=int, default=128, help="total sources (strong) or per GPU (--weak)")
    ap.add_argument("--weak", action="store_true", help="every rank runs --sources sources of its own")
    ap.add_argument("--cpu-sample", type=int, default=0, help="sources in the CPU sample (0: one per thread)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: the CPUs this job is granted (affinity, cgroup quota)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-return", action="store_true", help="skip the result-return measurement")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end ALI_FMM.update() measurement")
    ap.add_argument("--no-c3", action="store_true", help="skip the BASELINE config 3 line (N = 1)")
    ap.add_argument("--gather", action="store_true", help="N > 1: also time an RCCL gather of all fields to rank 0")
    ap.add_argument("--members", type=int, default=None, help="band-kernel workgroups per source (0: auto)")
    ap.add_argument("--cdelta", type=float, default=None)
    ap.add_argument("--no-c5", action="store_true", help="skip the BASELINE config 5 leg (receiver fields + rays)")
    return ap.parse_args()


_COUNT_GPUS = r"""
import ctypes, sys
try:
    h = ctypes.CDLL("libamdhip64.so")
except OSError:
    try:
        h = ctypes.CDLL("/opt/rocm/lib/libamdhip64.so")
    except OSError:
        print(0); sys.exit(0)
n = ctypes.c_int(0)
print(n.value if h.hipGetDeviceCount(ctypes.byref(n)) == 0 else 0)
"""


def visible_gpus():
    """HIP devices this job sees, counted in a child process: the launching parent never
    initialises the GPU (its children are the ranks)."""
    import subprocess

    try:
        r = subprocess.run([sys.executable, "-c", _COUNT_GPUS], capture_output=True, text=True, timeout=120)
        return int(r.stdout.strip().splitlines()[-1])
    except (subprocess.SubprocessError, ValueError, IndexError):
        return 0


def _free_port():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n):
    """`bench.py --gpus N` run directly (no WORLD_SIZE in the environment, N > 1): one process per
    GPU, LOCAL_RANK = RANK = 0 .. N-1 over a gloo group on 127.0.0.1, as the reference's
    find_all_TTF_rays_parallel / update_parallel spawn their own n_threads workers
    (Anis_TTF_rays.py:4550-4685, :3938-4051).  Refuses (exit 2) when fewer than N GPUs are visible,
    unless ALIFMM_BENCH_DEVICE pins every rank to one device (rehearsal) or ALIFMM_BENCH_STUB asks
    for the GPU-free stub ranks of the CPU tests.  Rank 0 prints the JSON line; the exit status is
    the first failing rank's (the others are then stopped)."""
    import signal
    import subprocess

    if "ALIFMM_BENCH_DEVICE" not in os.environ and "ALIFMM_BENCH_STUB" not in os.environ:
        have = visible_gpus()
        if have < n:
            print("bench.py: --gpus %d but %d GPU(s) visible (set ALIFMM_BENCH_DEVICE=<dev> to rehearse "
                  "every rank on one device)" % (n, have), file=sys.stderr, flush=True)
            return 2
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port, ALIFMM_BENCH_LAUNCHED="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c
                for q in live:  # a failed rank leaves the others blocked in the group: stop them
                    q.send_signal(signal.SIGTERM)
        time.sleep(0.2)
    return rc


def max_over_ranks(value, dist=None):
    """Max of a float over all ranks of the default process group (identity without one)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(value)
    import torch

    t = torch.tensor([float(value)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _sum_over_ranks(value, dist=None):
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return int(value)
    import torch

    t = torch.tensor([int(value)], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())


def rccl_gather_fields(ctx, n_local, subgrid, rank, world, dist, first_slot=0):
    """RCCL gather of every rank's resident fields to rank 0 through the library's C-ABI
    (alifmm_comm_init_rank + alifmm_gather_fields: one ncclSend / ncclRecv per field over xGMI,
    no padding), the result-return leg for N > 1.  torch.distributed (gloo, CPU) only carries the
    128-byte RCCL id and the per-rank counts.  Returns the timings (max over ranks)."""
    import _alifmm

    uid = [_alifmm.Comm.unique_id() if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    counts = [None] * world
    dist.all_gather_object(counts, int(n_local))
    t0 = time.perf_counter()
    comm = _alifmm.Comm.rank(ctx, world, rank, uid[0])
    init_s = max_over_ranks(time.perf_counter() - t0, dist)
    try:
        dist.barrier()
        ms = comm.gather(0, subgrid, [first_slot] * world, counts, dst_slot=first_slot)
    finally:
        comm.close()
    gather_s = max_over_ranks(ms / 1e3, dist)
    fz, fx = ctx.field_shape(subgrid)
    remote = (sum(counts) - counts[0]) * fz * fx * 8
    return {"rccl_init_ms": init_s * 1e3, "rccl_gather_ms": gather_s * 1e3, "rccl_gather_bytes_into_rank0": remote,
            "rccl_gather_GBps_into_rank0": remote / gather_s / 1e9 if gather_s > 0 else None,
            "rccl_gather": "alifmm_gather_fields (library C-ABI, librccl), one message per field"}


def rank_sources(args, rank, world, dnx):
    import sharding

    if args.weak:
        scx, scz = sharding.bench_sources(rank, args.sources, args.n, dnx)
        return scx, scz, np.arange(args.sources)
    k = np.array(sharding.deal(range(args.sources), world)[rank], dtype=np.int64)
    kk = k % (args.n // 32)
    return dnx * (16 + 32 * kk).astype(np.float64), np.zeros(len(k)), k


def _host_cpus():
    """(usable, quota, physical, logical): CPUs this process may run on (affinity), the job's CPU
    share in whole CPUs (cgroup quota / OMP_NUM_THREADS; None: unlimited), physical cores and
    logical CPUs of the host."""
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count()
    quota = None
    try:  # cgroup v2, else v1
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            if q > 0:
                quota = max(1, q // int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read()))
        except (OSError, ValueError):
            pass
    # the GPU boxes state a job's CPU share in OMP_NUM_THREADS (16 per GPU)
    share = os.environ.get("OMP_NUM_THREADS", "")
    if share.isdigit() and int(share) > 0:
        quota = min(quota or int(share), int(share))
    cores, phys, core = set(), None, None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("physical id"):
                phys = line.split(":")[1].strip()
            elif line.startswith("core id"):
                core = line.split(":")[1].strip()
                cores.add((phys, core))
    except OSError:
        pass
    return usable, quota, len(cores) or os.cpu_count(), os.cpu_count()


def c3_line(ctx, W):
    """BASELINE config 3 (2048^2 Voronoi grains, anisotropic, one interior source; all CUs on the
    one source: K band members) after the timed C4 steps: init / band kernel times (in-library HIP
    events, best of 3 after a warm-up), cell-sweeps and the band kernel's roofline at SURVEY
    §8(d)'s 18.1 B per sweep; the field against the reference's own (tests/golden/c3_2048,
    decimated x8) as a sanity figure (tests/test_gpu_parity.py holds the parity check)."""
    ctx.release_fields()
    vt = W.default_table()
    ctx.set_model(*W.c3_model(), vt, vt, 1e-3)
    x, z = W.c3_source()
    ctx.travel([x], [z], copy_out=False)
    best = None
    for _ in range(3):
        ctx.travel([x], [z], copy_out=False)
        t = ctx.last_timing()
        best = t if best is None or t[2] < best[2] else best
    st = ctx.source_stats(0)
    sweeps = int(st[1])
    out = {"workload": "C3: 2048x2048 Voronoi grains (rng 1234, 128 seeds), velpn 0, one source (x=%d, z=%d)"
                       % (round(x / 1e-3), round(z / 1e-3)),
           "init_ms": best[0], "band_ms": best[1], "total_ms": best[2], "band_workgroups": int(ctx.get_option("last_k")),
           "band_steps": int(st[0][3]), "cell_sweeps": sweeps,
           "roofline": {"bound": "hbm", "kernel": "fmm_band_k_kernel", "bytes_per_cell_sweep": BYTES_PER_SWEEP,
                        "achieved": BYTES_PER_SWEEP * sweeps / (best[1] * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                        "unit": "GB/s"}}
    out["roofline"]["frac"] = out["roofline"]["achieved"] / HBM_PEAK_GBS
    try:
        R = np.load(os.path.join(REPO, "tests", "golden", "c3_2048.npz"))["field_dec8"]
        D = ctx.get_field(0, 1)[::8, ::8]
        zz, xx = np.mgrid[0:D.shape[0], 0:D.shape[1]]
        m = np.hypot(zz - z / 1e-3 / 8, xx - x / 1e-3 / 8) > 1
        rel = np.abs(D[m] - R[m]) / R[m]
        out.update({"field_vs_reference_rel_max_dec8": float(rel.max()), "field_vs_reference_rel_mean_dec8": float(rel.mean())})
    except OSError:
        pass
    ctx.release_fields()
    return out


C5_PER_SIDE = 256


def c5_receivers(rank, world):
    """BASELINE config 5's receivers of this rank: the 256 bottom transducers (x = 8 + 16 k,
    z = 4095) dealt block-cyclically (sharding.deal), as find_all_TTF_rays_parallel hands each
    worker whole receivers and traces a receiver's rays in the process that built its field
    (parallel_TTF_rays, Anis_TTF_rays.py:3715-3733, :4550-4685)."""
    import sharding

    return np.array(sharding.deal(range(C5_PER_SIDE), world)[rank], dtype=np.int64)


def c5_leg(ctx, rank, world, dist, n, dnx, barrier):
    """BASELINE config 5 after the C4 steps: 256 top transducers (z = 0) firing into 256 bottom
    receivers (trans_pairs[i, 256 + j] = 1, the pattern of Weld_rays.py:52-55): each rank builds its
    receivers' fields (resident) and traces their 256 rays each (times only), then the (256, 256)
    times matrix is gathered to rank 0 (gloo: 512 KB).  Timed: fields + rays, max over ranks."""
    ctx.release_fields()
    xs = (8 + 16 * np.arange(C5_PER_SIDE)).astype(np.float64)
    mine = c5_receivers(rank, world)
    rx = xs[mine]
    src = np.stack([xs, np.zeros(C5_PER_SIDE)], 1)
    # warm-up: the travel arena and the ray buffers at the timed call's size (kept by the context)
    ctx.travel(dnx * rx[:2], np.full(min(2, len(rx)), dnx * (n - 1)), first_slot=0, copy_out=False)
    nr = len(rx) * C5_PER_SIDE
    ctx.find_rays(np.zeros(nr, dtype=np.int32), np.tile(src, (len(rx), 1)),
                  np.tile([rx[0], float(n - 1)], (nr, 1)), with_points=False)
    barrier()
    t0 = time.perf_counter()
    ctx.travel(dnx * rx, np.full(len(rx), dnx * (n - 1)), first_slot=0, copy_out=False)
    t1 = time.perf_counter()
    slots = np.repeat(np.arange(len(rx)), C5_PER_SIDE)
    s_xy = np.tile(src, (len(rx), 1))
    r_xy = np.repeat(np.stack([rx, np.full(len(rx), float(n - 1))], 1), C5_PER_SIDE, axis=0)
    times, lens, flags, _ = ctx.find_rays(slots, s_xy, r_xy, with_points=False)
    t2 = time.perf_counter()
    barrier()
    total = max_over_ranks(t2 - t0, dist)
    fields_s = max_over_ranks(t1 - t0, dist)
    rays_s = max_over_ranks(t2 - t1, dist)
    part = (mine.tolist(), times.reshape(len(rx), C5_PER_SIDE).tolist(), int(lens.sum()))
    parts = [part]
    if dist is not None:
        parts = [None] * world
        dist.all_gather_object(parts, part)
    ctx.release_fields()
    if rank != 0:
        return None
    tm = np.full((C5_PER_SIDE, C5_PER_SIDE), np.nan)  # [source i, receiver j]
    for js, tj, _ in parts:
        for j, row in zip(js, tj):
            tm[:, j] = row
    rays = C5_PER_SIDE * C5_PER_SIDE
    return {"workload": "C5: 4096x4096 weld-like grid, 256 top Tx (z=0) -> 256 bottom Rx (z=4095), x = 8 + 16 k: "
                        "256 receiver fields (subgrid 1) dealt over the GPUs + 65 536 rays on the receiver's GPU",
            "total_s": total, "fields_s": fields_s, "rays_s": rays_s, "rays": rays, "rays_per_s": rays / total,
            "fields_per_s": C5_PER_SIDE / total, "receivers_per_gpu": [len(p[0]) for p in parts],
            "points": int(sum(p[2] for p in parts)),
            "times_complete": bool(np.all(np.isfinite(tm)) and np.all(tm > 0)),
            "times_checksum": float(np.sum(tm)),
            "times": "gathered to rank 0 as the (256, 256) matrix (gloo)"}


def cpu_baseline(args, scx, scz, model, vt, dnx, cells):
    """the C restatement of the reference's solver, one source per thread on the
    CPUs this job is granted (affinity and cgroup quota), plus one source on one core; the
    all-core figure of the host is the 1-core rate times its physical cores (stated as such)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O

    veln, velpn, vel_map, stif = model
    usable, quota, phys, logical = _host_cpus()
    th = args.cpu_threads or min(usable, quota or usable)
    ns = args.cpu_sample or th
    xs, zs = np.resize(scx, ns), np.resize(scz, ns)
    t1 = time.perf_counter()
    O.travel_batch(xs[:1], zs[:1], veln, velpn, vel_map, stif, vt, vt, dnx=dnx, n_threads=1)
    one = time.perf_counter() - t1
    t1 = time.perf_counter()
    O.travel_batch(xs, zs, veln, velpn, vel_map, stif, vt, vt, dnx=dnx, n_threads=th)
    tc = time.perf_counter() - t1
    model_name = ""
    try:
        model_name = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
    except (OSError, StopIteration):
        pass
    per_core = cells / one  # cell-updates/s of one core
    return {"value": cells * ns / tc, "unit": "grid-cell updates/s", "cores": th, "kind": "port",
            "sample": "%d C4 sources (4096^2, z=0) on %d threads (this job's CPUs: affinity %d, share %s), "
                      "one source per thread, oracle/alifmm_oracle.c (bit-exact restatement of the reference's "
                      "heap FMM); %.1f s wall; plus 1 source on 1 core: %.2f s"
                      % (ns, th, usable, quota, tc, one),
            "host_cpu": model_name, "host_physical_cores": phys, "host_logical_cpus": logical,
            "seconds_per_source_1core": one,
            "value_1core": per_core,
            "value_all_physical_cores_extrapolated": per_core * phys,
            "port_vs_numba_reference_per_core": PORT_VS_REFERENCE_PER_CORE}


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print("bench.py: --gpus %d but WORLD_SIZE %d" % (args.gpus, world), file=sys.stderr, flush=True)
        sys.exit(2)
    dist = None
    if world > 1:
        import torch  # noqa: F401  (before the library: one HIP runtime for both, see rccl_gather_fields)
        import torch.distributed as dist

        dist.init_process_group("gloo", rank=rank, world_size=world)
    stub = "ALIFMM_BENCH_STUB" in os.environ
    # ranks that reached this point (the group's size is what was asked; this is what ran)
    ran = _sum_over_ranks(1, dist)
    if stub:  # CPU tests of the launcher: the source deal without a GPU
        scx, _, ids = rank_sources(args, rank, world, 1.0)
        got = [None] * world
        if dist is not None:
            dist.all_gather_object(got, [int(i) for i in ids])
        else:
            got = [[int(i) for i in ids]]
        rec = [None] * world
        if dist is not None:
            dist.all_gather_object(rec, c5_receivers(rank, world).tolist())
        else:
            rec = [c5_receivers(0, 1).tolist()]
        if rank == 0:
            print(json.dumps({"stub": True, "n_gpus": ran, "sources_per_rank": got, "c5_receivers_per_rank": rec}),
                  flush=True)
        if dist is not None:
            dist.destroy_process_group()
        return

    import _alifmm
    import sharding
    import workloads as W

    # one GPU per rank (LOCAL_RANK); ALIFMM_BENCH_DEVICE pins every rank to one device, only to
    # rehearse the multi-process path on a one-GPU box
    dev = int(os.environ.get("ALIFMM_BENCH_DEVICE", local))
    have = _alifmm.device_count()
    if dev >= have:
        print("bench.py: rank %d needs device %d, %d visible" % (rank, dev, have), file=sys.stderr, flush=True)
        sys.exit(3)
    n = args.n
    model = W.weldlike_model(n)
    dnx = W.weldlike_dnx()
    vt = W.default_table()
    ctx = _alifmm.Context(dev)
    devices = [dev]
    if dist is not None:
        devices = [None] * world
        dist.all_gather_object(devices, dev)
    if args.cdelta is not None:
        ctx.set_option("cdelta", args.cdelta)
    if args.members is not None:
        ctx.set_option("members", args.members)
    ctx.set_model(*model, vt, vt, dnx)
    scx, scz, _ = rank_sources(args, rank, world, dnx)
    ns = len(scx)

    def barrier():
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        ctx.travel(scx, scz, subgrid=1, first_slot=0, copy_out=False)
    barrier()
    t0 = time.perf_counter()
    band_ms = init_ms = 0.0
    for _ in range(args.steps):
        ctx.travel(scx, scz, subgrid=1, first_slot=0, copy_out=False)  # synchronous: returns when done
        ti, tb, _ = ctx.last_timing()
        init_ms += ti
        band_ms += tb
    barrier()
    dt = max_over_ranks(time.perf_counter() - t0, dist)
    sweeps = sum(ctx.source_stats(i)[1] for i in range(ns))
    steps_main = [int(ctx.source_stats(i)[0][3]) for i in range(ns)]
    members = int(ctx.get_option("last_k"))
    cells = float(n) * n
    total_src = args.sources * (world if args.weak else 1)
    value = cells * total_src * args.steps / dt
    band_avg_s = band_ms / args.steps / 1e3
    achieved = BYTES_PER_SWEEP * sweeps / band_avg_s / 1e9 if band_avg_s > 0 else None

    config = {"workload": "C4: %dx%d weld-like grid, %d top-surface Tx sources %s, subgrid 1"
                          % (n, n, total_src, "per GPU (weak)" if args.weak else "dealt over the GPUs (strong)"),
              "total_sources": total_src, "sources_per_gpu": ns, "grid": [n, n], "subgrid": 1,
              "band_workgroups_per_source": members, "cdelta": args.cdelta}
    # HBM-side bytes per launch: rocprofv3 PMC passes (tools/profile.sh) on this library and workload
    traffic_bytes = None
    valu = None
    try:
        import glob
        import hashlib

        lib_sha = hashlib.sha256(open(_alifmm.LIB_PATH, "rb").read()).hexdigest()
        for f in sorted(glob.glob(os.path.join(REPO, "profiles", "*_traffic.json"))):
            t = json.load(open(f))
            if (t.get("libalifmm_sha256") == lib_sha and t.get("traffic_bytes_per_launch")
                    and t.get("kernel", "fmm_band_k_kernel") == "fmm_band_k_kernel"
                    and t.get("sources_per_gpu") == ns and t.get("grid") == [n, n]):
                traffic_bytes = t["traffic_bytes_per_launch"]
                if t.get("valu_insts_per_launch"):
                    valu = t
    except OSError:
        pass

    # result-return leg (not in value): D2H of this rank's fields; RCCL gather to rank 0 (N > 1)
    ret = None
    if not args.no_return:
        ret = {}
        barrier()
        t1 = time.perf_counter()
        _, gbps = ctx.copy_fields(0, ns, 1)
        d2h = max_over_ranks(time.perf_counter() - t1, dist)
        ret.update({"d2h_ms": d2h * 1e3, "d2h_GBps_per_gpu": gbps, "bytes_per_gpu": int(cells * 8 * ns),
                    "d2h": "pageable host memory through the library's pinned staging ring, every GPU at once"})
        # the same copy DMA'd straight into the pageable destination, registered for the copy
        dst = np.empty((ns, n, n))
        barrier()
        t1 = time.perf_counter()
        ctx.copy_fields_into(0, dst, range(ns), 1, dst_kind=3)
        d2h_reg = max_over_ranks(time.perf_counter() - t1, dist)
        del dst
        ret.update({"d2h_registered_ms": d2h_reg * 1e3, "d2h_registered_GBps_per_gpu": cells * 8 * ns / d2h_reg / 1e9})
        if world > 1 and "ALIFMM_BENCH_DEVICE" in os.environ:
            ret["rccl_gather"] = "skipped: every rank on one device (RCCL needs one GPU per rank)"
        elif world > 1 and args.gather:
            ret.update(rccl_gather_fields(ctx, ns, 1, rank, world, dist))
    # end to end through the drop-in (N = 1): ALI_FMM.update() on the C4 sources — model digest,
    # fields, and their single copy into the caller's (nsrc, 4096, 4096) stack; the second call is
    # timed (the first uploads the model into the object's own context)
    e2e = None
    if world == 1 and not args.no_e2e:
        import Anis_TTF_rays as A

        ctx.release_fields()
        M = A.ALI_FMM(model[0], model[1], model[2], scx, scz, stif_den=model[3], dnx=dnx)
        M.update(model[0], model[1], model[2], model[3])
        runs = []
        for _ in range(2):  # steady state: the better of two calls (each returns a fresh 17 GB stack)
            t1 = time.perf_counter()
            F = M.update(model[0], model[1], model[2], model[3])
            runs.append(time.perf_counter() - t1)
            if _ == 0:
                del F
        te = min(runs)
        e2e = {"update_s": te, "update_s_runs": runs, "cell_updates_per_s": cells * ns / te, "sources_per_s": ns / te,
               "stack_bytes": int(F.nbytes), "fields_ms": M._ctx(0).last_timing()[2],
               "stream_tail_ms": M._ctx(0).get_option("stream_tail_ms"),
               "stream_fallback_fields": M._ctx(0).get_option("stream_fallback"),
               "what": "ALI_FMM.update() at C4: model digest (xxh3 of every array) + fields on the GPU, each "
                       "streamed tile by tile out of the band kernel into the returned stack while it runs "
                       "(alifmm_travel_into; stream_tail_ms = kernel end to last tile copied)"}
        del F
        for c in M._ctxs.values():
            c.close()
    c5 = None
    if not args.no_c5:
        c5 = c5_leg(ctx, rank, world, dist, n, dnx, barrier)
    c3 = None
    if world == 1 and not args.no_c3:
        c3 = c3_line(ctx, W)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(args, scx, scz, model, vt, dnx, cells)
    if rank == 0:
        out = {
            "metric": "grid-cell updates/sec + sources/sec on 4096^2 anisotropic grid",
            "value": value,
            "unit": "grid-cell updates/s",
            "n_gpus": ran,
            "devices": devices,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak" if args.weak else "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: weld-like model built from the reference's weld_*.npy (edge-padded, 8x nearest), "
                    "stiffness row of the notebook",
            "config": config,
            "sources_per_s": total_src * args.steps / dt,
            "kernel_ms_per_step": {"fmm_init_kernel": init_ms / args.steps, "fmm_band_k_kernel": band_ms / args.steps},
            "band_steps_main_mean": float(np.mean(steps_main)),
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
                         "traffic": traffic_bytes,
                         "kernel": "fmm_band_k_kernel", "bytes_per_cell_sweep": BYTES_PER_SWEEP,
                         "cell_sweeps_per_launch": int(sweeps),
                         "algorithmic_bytes_per_launch": BYTES_PER_SWEEP * int(sweeps),
                         "traffic_over_algorithmic": (traffic_bytes / (BYTES_PER_SWEEP * sweeps))
                         if traffic_bytes else None,
                         # what does bound it: f64 VALU issue (a wave64 VALU op occupies a SIMD for
                         # >= 4 cycles), from the SQ pass of the same build: VALU cycles / SIMD cycles
                         "valu_issue": ({"insts_per_launch": valu["valu_insts_per_launch"],
                                         "floor_ms": valu["valu_insts_per_launch"] * 4 / VALU_SIMDS / CLOCK_HZ * 1e3,
                                         "frac": valu["valu_insts_per_launch"] * 4 / VALU_SIMDS / CLOCK_HZ / band_avg_s,
                                         "sq_wait_any_frac": valu.get("sq_wait_any_frac")}
                                        if valu and band_avg_s > 0 else None)},
            "result_return": ret,
            "update_end_to_end": e2e,
            "c3": c3,
            "c5": c5,
            "cpu_baseline": cpu,
        }
        if cpu:
            out["speedup_vs_cpu_baseline"] = value / cpu["value"]
            out["speedup_vs_cpu_all_physical_cores_extrapolated"] = value / cpu["value_all_physical_cores_extrapolated"]
            # the numba reference itself, by the measured per-core calibration of the port
            out["speedup_vs_numba_reference_same_cores"] = value / (cpu["value"] / PORT_VS_REFERENCE_PER_CORE)
            out["speedup_vs_numba_reference_all_physical_cores"] = value / (
                cpu["value_all_physical_cores_extrapolated"] / PORT_VS_REFERENCE_PER_CORE)
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main()
