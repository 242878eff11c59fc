"""CPU-side checks of the boundary and the host logic (no GPU needed):
the C-ABI library loads and exports every entry point include/alifmm.h declares, the drop-in
module's host-only behaviour (errors, velocity tables) matches the reference, and the N>1 source
sharding is disjoint and complete across a world_size-2 gloo process group."""
import os
import re
import socket

import numpy as np
import pytest

import workloads as W

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def _declared():
    h = open(os.path.join(REPO, "include", "alifmm.h")).read()
    h = re.sub(r"/\*.*?\*/", "", h, flags=re.S)
    return sorted(set(re.findall(r"\b(alifmm_[a-z_0-9]+)\s*\(", h)))


def test_cabi_exports_every_declared_symbol():
    import ctypes

    import _alifmm

    assert os.path.exists(_alifmm.LIB_PATH), "build first: __graft_entry__.build()"
    lib = ctypes.CDLL(_alifmm.LIB_PATH)
    names = _declared()
    assert len(names) >= 15, names
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    lib.alifmm_version.restype = ctypes.c_char_p
    assert b"gfx950" in lib.alifmm_version()
    # the ctypes binding declares a signature for every exported entry point
    src = open(os.path.join(REPO, "ali-fmm-and-ray-tracing_amd", "_alifmm.py")).read()
    unbound = [n for n in names if '"%s"' % n not in src]
    assert not unbound, unbound


def test_library_is_gfx950_only():
    import _alifmm

    blob = open(_alifmm.LIB_PATH, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa-[-a-z]*gfx[0-9a-z]+", blob))
    assert targets == {b"amdgcn-amd-amdhsa--gfx950"}, targets


def test_dropin_errors_match_reference():
    import Anis_TTF_rays as A

    n = 11
    veln = np.zeros((n, n))
    velpn = np.ones((n, n), dtype=np.int64)
    vm = np.ones((n, n))
    with pytest.raises(TypeError):  # :3820-3826 stiffness must be int64
        A.ALI_FMM(veln, velpn, vm, [0.0], [0.0], stif_den=np.ones((n, n, 5), dtype=np.int32))
    with pytest.raises(TypeError):  # :3831-3838 velpn must be integer
        A.ALI_FMM(veln, np.ones((n, n)), vm, [0.0], [0.0])
    M = A.ALI_FMM(veln, velpn, vm, [1e-3 * 2, 1e-3 * 7.5], [0.0, 1e-3 * 4.5])
    assert list(M.isx) == [2, 8] and list(M.isz) == [0, 4]  # Python round(): half-even (:3851-3853)
    with pytest.raises(ValueError):  # :4573-4574
        M.find_all_TTF_rays_parallel(veln, velpn, vm, n_threads=1)


def test_velocity_tables_match_reference(golden):
    """add_materials / generate_{group,phase}_vel (host-side, :4112-4256) vs the reference's K2 tables."""
    import Anis_TTF_rays as A

    g = golden("kat_notebook")
    dnx = 1e-3
    veln = np.zeros((201, 201))
    velpn = np.ones((201, 201), dtype=int)
    vm1 = np.ones((201, 201))
    c22, c23, c33, c44, sigma = 249.0e9, 133.0e9, 205.0e9, 125.0e9, 7850
    M1 = A.ALI_FMM(veln, velpn, vm1, dnx * np.array([1, 199]), dnx * np.array([100, 140]), dnx=1e-3)
    M1.add_materials(np.array([[c22, c23, c33, c44, 2 * sigma], [c22, c23, c33, c44, 3 * sigma]]), True)
    M1.add_materials(np.array([c22, c23, c33, c44, sigma]))
    assert np.array_equal(M1.velocity_dat, g["k2_group"]) and np.array_equal(M1.phase_vel, g["k2_phase"])


def test_group_vel_function_matches_reference(golden):
    """Module-level group_vel() (host-side, :3520-3558) vs the reference's own outputs."""
    import Anis_TTF_rays as A

    g = golden("group_vel")
    a = np.array([A.group_vel(x, 249000, 133000, 205000, 125000, 7850, 1.0) for x in g["angles"]])
    b = np.array([A.group_vel(x, 203600, 129800, 203600, 133500, 7874, 1.3) for x in g["angles"]])
    assert np.array_equal(a, g["set1"]) and np.array_equal(b, g["iron_scaled"])


def test_deal_partitions_sources():
    import sharding

    for n_src in (0, 1, 7, 128, 131):
        for parts in (1, 2, 3, 8):
            d = sharding.deal(range(n_src), parts)
            flat = sorted(i for p in d for i in p)
            assert flat == list(range(n_src)) and len(d) == parts
            assert max(len(p) for p in d) - min(len(p) for p in d) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, q):
    import sys
    import types

    sys.path.insert(0, os.path.join(REPO, "ali-fmm-and-ray-tracing_amd"))
    sys.path.insert(0, REPO)
    import torch.distributed as dist

    import bench
    import sharding

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = {}
    for weak in (True, False):  # --weak (every rank 128 sources) and the default strong deal
        args = types.SimpleNamespace(weak=weak, sources=128, n=4096)
        scx, scz, ids = bench.rank_sources(args, rank, world, 2.5e-5)
        allx, allid = [None] * world, [None] * world  # ragged shards: object gathers over gloo
        dist.all_gather_object(allx, np.round(scx / 2.5e-5).astype(np.int64))
        dist.all_gather_object(allid, np.asarray(ids, dtype=np.int64))
        out[weak] = (allx, allid, scz.tolist())
    # the counts every rank passes to alifmm_gather_fields (bench.rccl_gather_fields), exchanged as there
    counts = [None] * world
    dist.all_gather_object(counts, len(out[False][0][rank]))
    m = bench.max_over_ranks(float(rank) + 0.5, dist)
    if rank == 0:
        q.put((out, counts, m))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharding_gloo(world):
    """bench.py's N>1 path on CPU with gloo ranks: --weak gives disjoint complete 128-source sets
    (rank 0 = BASELINE C4's); the default strong deal splits C4's 128 sources block-cyclically with
    nothing lost or doubled; the RCCL gather's layout (counts exchanged over gloo, rank after rank
    on the root: sharding.gather_plan / _alifmm.gather_layout) puts every source in its own root
    slot; the max-over-ranks reduction picks the slowest rank."""
    import torch.multiprocessing as mp

    import sharding
    import _alifmm

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out, counts, m = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    xw, _, szw = out[True]
    for a in xw:
        assert len(set(a.tolist())) == 128
    assert not set(xw[0].tolist()) & set(xw[1].tolist())
    assert xw[0].tolist() == [16 + 32 * k for k in range(128)]  # rank 0 = BASELINE C4 sources
    xs, ids, szs = out[False]
    allids = np.concatenate(ids)
    assert sorted(allids.tolist()) == list(range(128))  # strong: every C4 source exactly once
    assert np.array_equal(np.concatenate(xs), 16 + 32 * allids)
    assert [len(a) for a in ids] == counts and sum(counts) == 128 and max(counts) - min(counts) <= 1
    cnt, slot = sharding.gather_plan(128, world)
    assert cnt == counts
    assert sorted(slot.tolist()) == list(range(128))  # one root slot per source
    off = _alifmm.gather_layout(counts)
    for r in range(world):
        assert np.array_equal(slot[ids[r]], off[r] + np.arange(counts[r]))
    assert m == world - 0.5 and set(szw) == {0.0} and set(szs) == {0.0}


def test_ray_store_matches_dense_layout(tmp_path):
    """Compact ray storage: PackedRayPaths reads like the reference's dense
    (n, n, 5(nnz+nnx)) ray arrays (:4286-4289) for the indexing callers use (Weld_rays.py:64-66
    trims [:, :, 0:max_len]; ray_path :4687-4705 reads [i, j, 0:len]), and save/load round-trips."""
    from raystore import PackedRayPaths, RayStore

    rng = np.random.default_rng(5)
    n, cap = 7, 40
    st = RayStore(n, cap)
    dense = np.zeros((2, n, n, cap))
    pairs = [(i, j) for i in range(n) for j in range(n) if rng.random() < 0.6]
    for chunk in (pairs[: len(pairs) // 2], pairs[len(pairs) // 2:]):
        lens = rng.integers(1, cap + 1, len(chunk))
        pts = rng.normal(size=(int(lens.sum()), 2))
        st.add([p[0] for p in chunk], [p[1] for p in chunk], lens, pts)
        o = 0
        for (i, j), L in zip(chunk, lens):
            dense[:, i, j, :L] = pts[o:o + L].T
            o += L
    for ax in (0, 1):
        P = PackedRayPaths(st, ax)
        D = dense[ax]
        assert P.shape == D.shape and len(P) == n
        np.testing.assert_array_equal(np.asarray(P), D)
        ml = int(st.ray_len.max())
        for key in [(slice(None), slice(None), slice(0, ml)), (3,), (2, 5), (2, 5, slice(0, 9)), (1, 4, 7),
                    (slice(1, 5), 2), (Ellipsis, 3), (np.array([0, 2, 6]), np.array([1, 1, 3])),
                    (slice(None), np.array([4, 0]), slice(2, 30, 3)), (-1, -2, -3)]:
            np.testing.assert_array_equal(P[key], D[key], err_msg=str(key))
    for i, j in pairs:
        x, z = st.path(i, j)
        L = st.ray_len[i, j]
        np.testing.assert_array_equal(x, dense[0, i, j, :L])
        np.testing.assert_array_equal(z, dense[1, i, j, :L])
    f = str(tmp_path / "rays.npz")
    st.save(f)
    st2 = RayStore.load(f)
    np.testing.assert_array_equal(st2.ray_len, st.ray_len)
    np.testing.assert_array_equal(st2.dense(0), dense[0])
    np.testing.assert_array_equal(st2.dense(1), dense[1])


def test_ray_flags_raise():
    """a ray cut short at the reference's point capacity (the reference raises
    IndexError there) or on an empty search plane is an error, not a plausible time; the
    reference's early exit (bit 0) is normal output."""
    import _alifmm

    _alifmm.check_ray_flags(np.array([0, 1, 0, 1], dtype=np.int32))
    with pytest.raises(IndexError):
        _alifmm.check_ray_flags(np.array([0, 2], dtype=np.int32))
    with pytest.raises(_alifmm.AlifmmError):
        _alifmm.check_ray_flags(np.array([4, 0], dtype=np.int32))


def test_model_key_tracks_every_cell():
    """ADVICE r2 / VERDICT r2: the resident-model key is a digest of the full content, so an
    in-place edit of ANY cell of a C4-size array (interior, unsampled) changes it, as does new
    data at a recycled address; trust_model_identity=True opts into the identity cache (which then
    keeps the key, by contract)."""
    import Anis_TTF_rays as A

    n = 4096
    veln = np.zeros((n, n))
    velpn = np.zeros((n, n), dtype=np.int64)
    vm = np.ones((n, n))
    sd = W.stif_field(n, n)
    vt = W.default_table()
    args = [veln, velpn, vm, sd, vt, vt]
    k0 = A._model_digest(args)
    assert A._model_digest(args) == k0
    veln[100, 100] += 5.0
    k1 = A._model_digest(args)
    assert k1 != k0
    sd[2001, 3003, 2] += 1
    k2 = A._model_digest(args)
    assert k2 not in (k0, k1)
    vm[4095, 17] *= 1.5
    assert A._model_digest(args) not in (k0, k1, k2)
    assert A._model_digest([veln.copy(), velpn, vm, sd.copy(), vt, vt]) == A._model_digest(args)
    try:
        A.trust_model_identity = True
        k3 = A._model_digest(args)
        veln[7, 7] += 1.0
        assert A._model_digest(args) == k3  # identity cache: the caller promised no in-place edits
    finally:
        A.trust_model_identity = False
        A._identity_cache.clear()
    assert A._model_digest(args) != k3


def test_shutdown_keeps_library_mapped(monkeypatch):
    """The atexit teardown (_alifmm.shutdown) destroys contexts but leaves libalifmm.so mapped, so
    the process maps name the HIP library to the end; only under rocprofv3 (ROCPROF* variables) is
    it unloaded early (the profiler's finalisation runs before the module destructor otherwise)."""
    import _alifmm

    for k in list(os.environ):
        if k.startswith(("ROCPROF", "ROCP_")):
            monkeypatch.delenv(k)
    _alifmm.lib()
    _alifmm.shutdown()
    maps = open("/proc/self/maps").read()
    assert os.path.realpath(_alifmm.LIB_PATH) in maps
    assert _alifmm.lib() is not None  # still usable after the teardown
    monkeypatch.setenv("ROCPROFILER_TEST_MARKER", "1")
    assert _alifmm._profiler_attached()


@pytest.mark.parametrize("args", [
    "3 2 6 300 333 1",       # K = 2, W = 64, ragged last stripe and tile row
    "2 16 4 257 500 2",      # K = 16, W = 16: members with no stripe of their own at the edge
    "1 1 6 64 64 3",         # one member
    "4 4 6 1000 130 4",
    "2 2 6 4096 4096 5",     # the C4 geometry (64 x 128 tiles, 1024 own tiles per member)
])
def test_stream_protocol_model(args, tmp_path):
    """The host side of the band kernel's field streaming (csrc/tile_stream.h: tile plan, queue
    drain, slot hand-back) against a CPU model of the kernel's side (tests/stream_sim.cpp: bursts
    of completed tiles past a step's list, the end flush): every field arrives intact in reversed,
    non-consecutive rows, and a ring one list too small is reported as a deadlock."""
    import subprocess

    here = os.path.dirname(os.path.abspath(__file__))
    exe = str(tmp_path / "stream_sim")
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread",
                    "-I" + os.path.join(here, "..", "ali-fmm-and-ray-tracing_amd", "csrc"),
                    os.path.join(here, "stream_sim.cpp"), "-o", exe], check=True)
    r = subprocess.run([exe] + args.split(), capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.startswith("ok"), r.stdout + r.stderr
    if args.startswith("3 2"):
        r = subprocess.run([exe] + args.split() + ["40", "2"], capture_output=True, text=True, timeout=120)
        assert r.returncode == 1 and "deadlock=1" in r.stdout, r.stdout


def _bench(args, env_extra, timeout=240):
    import subprocess
    import sys

    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "ALIFMM_BENCH_DEVICE",
                                                            "ALIFMM_BENCH_STUB")}
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=timeout)


@pytest.mark.parametrize("world", [2, 3])
def test_bench_launches_its_own_ranks(world):
    """`python bench.py --gpus N` without an outside launcher spawns N ranks itself (gloo on
    127.0.0.1), deals C4's 128 sources block-cyclically over them and reports n_gpus = the ranks
    that ran (stub ranks: the launcher and the deal, no GPU)."""
    import json

    r = _bench(["--gpus", str(world)], {"ALIFMM_BENCH_STUB": "1"})
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == world
    per = line["sources_per_rank"]
    assert len(per) == world and sorted(sum(per, [])) == list(range(128))
    assert max(map(len, per)) - min(map(len, per)) <= 1
    # the C5 leg's deal: every one of the 256 bottom receivers on exactly one rank (its rays with it)
    rec = line["c5_receivers_per_rank"]
    assert len(rec) == world and sorted(sum(rec, [])) == list(range(256))
    assert max(map(len, rec)) - min(map(len, rec)) <= 1


def test_bench_refuses_more_gpus_than_visible():
    """--gpus N with fewer than N visible GPUs (none in this container) exits non-zero before any
    rank starts, unless ALIFMM_BENCH_DEVICE pins the ranks to one device for a rehearsal."""
    r = _bench(["--gpus", "2", "--steps", "1"], {})
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "GPU(s) visible" in r.stderr

