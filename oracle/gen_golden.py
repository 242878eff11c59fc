"""Generate tests/golden/*.npz by running the REFERENCE itself (TEST INFRASTRUCTURE ONLY).

Runs only in the build container, where /root/reference exists:
    cd /tmp && NUMBA_CACHE_DIR=/tmp/numba_cache /opt/conda/bin/python3.9 -W ignore \
        /root/repo/oracle/gen_golden.py [names...]
The reference module is exec'd from its own file with the 'padded' stage-1 arrays
(oracle/numba_boot.py).  No reference source is copied into the repo:
only the inputs/outputs written here (data) are committed.
"""
import hashlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(REPO, "tests"))

import numba_boot  # noqa: E402
import numpy as np  # noqa: E402

import workloads as W  # noqa: E402

OUT = os.path.join(REPO, "tests", "golden")
R = None


def ref():
    global R
    if R is None:
        R = numba_boot.load_reference()
    return R


def tr(scx, scz, veln, velpn, vel_map, stif, av, ph, dnx):
    nnz, nnx = veln.shape
    if stif is None:  # the class passes float zeros when stif_den is None (:3890-3891)
        stif = np.zeros((nnz, nnx, 5))
    T = ref().travel(scx, scz, np.zeros((nnx, nnz), dtype=int), np.zeros((round(0.5 * nnx * nnz) + 4, 2), dtype=int),
                     0, np.zeros((nnz, nnx)), veln, velpn, vel_map, stif, av, ph, 0, 0, dnx, dnx, nnx, nnz)
    return T.copy()


def save(name, **arrs):
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **arrs)
    print("wrote", path, os.path.getsize(path), "bytes", flush=True)


def mat_table(c22, c23, c33, c44, rho):
    """Material table via the reference's own ALI_FMM.generate_group_vel / generate_phase_vel."""
    n = 5
    m = ref().ALI_FMM(np.zeros((n, n)), np.ones((n, n), dtype=int), np.ones((n, n)), np.array([0.0]), np.array([0.0]))
    g = m.generate_group_vel(c22, c23, c33, c44, rho, plot=False)
    p = m.generate_phase_vel(c22, c23, c33, c44, rho, plot=False)
    return g, p


def gen_fmm_small():
    cases = {}
    k = 0

    def add(veln, velpn, vel_map, stif, av, ph, dnx, srcs, sg=1):
        nonlocal k
        for (x, z) in srcs:
            if sg == 1:
                T = tr(dnx * x, dnx * z, veln, velpn, vel_map, stif, av, ph, dnx)
            else:
                T = ref().travel_finer_grid(dnx * x, dnx * z, veln, velpn, vel_map, stif, sg, av, ph, 0, 0, dnx,
                                            dnx).copy()
            p = "c%d_" % k
            cases[p + "veln"] = veln
            cases[p + "velpn"] = velpn
            cases[p + "vel_map"] = vel_map
            if stif is not None:
                cases[p + "stif"] = stif
            cases[p + "av"] = av
            cases[p + "ph"] = ph
            cases[p + "meta"] = np.array([dnx, x, z, sg], dtype=np.float64)
            cases[p + "out"] = T
            k += 1

    vt = W.default_table()
    # (a) isotropic, non-square, sources at centre/corners/edges (top rows exercise SURVEY B-D2)
    nz, nx = 41, 53
    add(np.zeros((nz, nx)), np.ones((nz, nx), dtype=np.int64), 5790.0 * np.ones((nz, nx)), None, vt, vt, 1e-3,
        [(26, 20), (0, 0), (52, 40), (10, 0), (0, 15), (52, 1)])
    # (b) anisotropic Voronoi grains, per-cell stiffness
    n = 61
    veln = W.voronoi_small(n, 3)
    add(veln, np.zeros((n, n), dtype=np.int64), np.ones((n, n)), W.stif_field(n, n), vt, vt, 1e-3,
        [(30, 20), (30, 0), (1, 60), (60, 1), (45, 59)])
    # (c) table-defined anisotropic material (notebook constants, first set), velpn = 1
    g, p = mat_table(249.0e9, 133.0e9, 205.0e9, 125.0e9, 7850)
    av = np.zeros((361, 2)); av[:, 0] = np.arange(361); av[:, 1] = g
    ph = np.zeros((361, 2)); ph[:, 0] = np.arange(361); ph[:, 1] = p
    nz, nx = 48, 40
    add(W.voronoi_orientations(48, 5, 11)[:, :40].copy(), np.ones((nz, nx), dtype=np.int64), np.ones((nz, nx)),
        np.zeros((nz, nx, 5), dtype=np.int64), av, ph, 1e-3, [(10, 10), (39, 47), (20, 0)])
    # (d) weld patch: mixed stiffness / isotropic cells, fractional orientations (int32 truncation in stages)
    wv, wp, wm, ws = W.weld_model()
    sl = (slice(0, 60), slice(200, 280))
    add(wv[sl].copy(), wp[sl].copy(), wm[sl].copy(), ws[sl].copy(), vt, vt, 2e-4, [(40, 0), (10, 59), (79, 30)])
    # (e) travel_finer_grid, sg = 1 (SURVEY B-D4), 3, 5
    n = 21
    veln = W.voronoi_small(25, 5)[:21, :].copy()
    add(veln, np.zeros((21, 25), dtype=np.int64), np.ones((21, 25)), W.stif_field(21, 25), vt, vt, 1e-3,
        [(10, 0), (12, 10)], sg=3)
    add(veln, np.zeros((21, 25), dtype=np.int64), np.ones((21, 25)), W.stif_field(21, 25), vt, vt, 1e-3,
        [(3, 20)], sg=5)
    add(veln, np.zeros((21, 25), dtype=np.int64), np.ones((21, 25)), W.stif_field(21, 25), vt, vt, 1e-3,
        [(12, 10)], sg=1)
    # (f) velocity-gradient isotropic (notebook K1 model, smaller)
    n = 31
    vm = np.zeros((n, n))
    for j in range(n):
        vm[:, j] = 3000 + 21 * j * 6
    add(np.zeros((n, n)), np.ones((n, n), dtype=np.int64), vm, None, vt, vt, 1e-3, [(1, 5), (29, 25)])
    cases["ncases"] = np.array(k)
    save("fmm_small", **cases)


def gen_c1():
    veln, velpn, vm, _ = W.c1_model()
    vt = W.default_table()
    srcs = [(100, 100), (0, 0), (37, 150)]
    out = np.stack([tr(1e-3 * x, 1e-3 * z, veln, velpn, vm, np.zeros((201, 201, 5)), vt, vt, 1e-3) for x, z in srcs])
    save("c1_fields", src=np.array(srcs), out=out)


def gen_kat():
    RR = ref()
    res = {}
    # K1 (notebook cells 4-16): velocity gradient, default sg = 9
    dnx = 1e-3
    veln = 0 * np.ones((201, 201))
    velpn = 1 * np.ones((201, 201), dtype=int)
    vm = np.zeros((201, 201))
    for j in range(201):
        vm[:, j] = 3000 + 21 * j
    M = RR.ALI_FMM(veln, velpn, vm, dnx * np.array([1, 199]), dnx * np.array([30, 180]), dnx=1e-3)
    t0 = time.time()
    res["k1_times"] = M.find_all_TTF_rays(veln, velpn, vm)
    res["k1_ray_x"], res["k1_ray_y"] = [np.asarray(a) for a in M.ray_path(0, 1)]
    print("K1", res["k1_times"][0, 1], "%.1fs" % (time.time() - t0), flush=True)
    # K2 (cells 20-30): table material, first constant set (SURVEY B-D12)
    c22, c23, c33, c44, sigma = 249.0e9, 133.0e9, 205.0e9, 125.0e9, 7850
    veln = 0 * np.ones((201, 201))
    velpn = 1 * np.ones(veln.shape, dtype=int)
    vm = 1 * np.ones(veln.shape)
    M1 = RR.ALI_FMM(veln, velpn, vm, dnx * np.array([1, 199]), dnx * np.array([100, 140]), dnx=1e-3)
    M1.add_materials(np.array([[c22, c23, c33, c44, 2 * sigma], [c22, c23, c33, c44, 3 * sigma]]), True)
    M1.add_materials(np.array([c22, c23, c33, c44, sigma]))
    res["k2_group"] = M1.velocity_dat.copy()
    res["k2_phase"] = M1.phase_vel.copy()
    trans = np.zeros((2, 2)); trans[1, 0] = 1; trans[0, 1] = 1
    t0 = time.time()
    res["k2_times"] = M1.find_all_TTF_rays(veln, velpn, vm, trans_pairs=trans)
    for (i, j) in [(0, 1), (1, 0)]:
        rx, ry = M1.ray_path(i, j)
        res["k2_ray_x_%d%d" % (i, j)], res["k2_ray_y_%d%d" % (i, j)] = np.asarray(rx), np.asarray(ry)
    print("K2", res["k2_times"], "%.1fs" % (time.time() - t0), flush=True)
    # K3 (cells 34-40): per-cell stiffness, veln = 20 deg
    sd = np.zeros((201, 201, 5), dtype=np.int64)
    sd[:, :, 0] = 249000; sd[:, :, 1] = 133000; sd[:, :, 2] = 205000; sd[:, :, 3] = 125000; sd[:, :, 4] = 7850
    veln = 20 * np.ones((201, 201))
    velpn = 0 * np.ones((201, 201), dtype=int)
    vm = 1 * np.ones((201, 201))
    M2 = RR.ALI_FMM(veln, velpn, vm, dnx * np.array([1, 199, 100]), dnx * np.array([100, 140, 1]), stif_den=sd,
                    dnx=1e-3)
    t0 = time.time()
    res["k3_times"] = M2.find_all_TTF_rays(veln, velpn, vm, stif_den=sd)
    for (i, j) in [(0, 1), (0, 2), (1, 2)]:
        rx, ry = M2.ray_path(i, j)
        res["k3_ray_x_%d%d" % (i, j)], res["k3_ray_y_%d%d" % (i, j)] = np.asarray(rx), np.asarray(ry)
    print("K3", res["k3_times"], "%.1fs" % (time.time() - t0), flush=True)
    # the two material tables of notebook cell 20 (both constant sets)
    for tag, cs in (("set1", (249.0e9, 133.0e9, 205.0e9, 125.0e9, 7850)),
                    ("iron", (2.036e11, 1.298e11, 2.036e11, 1.335e11, 7874))):
        res["gen_group_" + tag], res["gen_phase_" + tag] = mat_table(*cs)
    save("kat_notebook", **res)


def _rays(T, sg, pairs, veln, velpn, vm, sd, vt, dnx, isx, isz):
    res = {}
    for (i, j) in pairs:
        src = np.array([sg * isx[i], sg * isz[i]])
        rec = np.array([sg * isx[j], sg * isz[j]])
        rx, ry, t = ref().find_ray(dnx, vt, src, rec, T, veln, velpn, vm, sd, sg)
        res["ray_x_%d" % i], res["ray_y_%d" % i], res["time_%d" % i] = rx.copy(), ry.copy(), np.array(t)
        print("  ray", i, "->", j, "time %.10e npts %d" % (t, len(rx)), flush=True)
    return res


def gen_weld(sg):
    veln, velpn, vm, sd = W.weld_model()
    vt = W.default_table()
    dnx = 2e-4
    scx, scz = W.weld_transducers()
    isx = np.round(scx / dnx)
    isz = np.round(scz / dnx)
    j = 46
    t0 = time.time()
    if sg == 1:
        T = tr(scx[j], scz[j], veln, velpn, vm, sd, vt, vt, dnx)
    else:
        T = ref().travel_finer_grid(scx[j], scz[j], veln, velpn, vm, sd, sg, vt, vt, 0, 0, dnx, dnx).copy()
    print("weld sg=%d TTF %.1fs" % (sg, time.time() - t0), flush=True)
    res = _rays(T, sg, [(0, j), (15, j), (30, j)], veln, velpn, vm, sd, vt, dnx, isx, isz)
    if sg == 1:
        res["field"] = T
    else:
        res["field_dec"] = T[::sg, ::sg].copy()
        res["row_mid"] = T[T.shape[0] // 2].copy()
        res["col_mid"] = T[:, T.shape[1] // 2].copy()
        res["fine_shape"] = np.array(T.shape)
    save("weld_sg%d" % sg, **res)


def gen_c3():
    veln, velpn, vm, sd = W.c3_model()
    vt = W.default_table()
    x, z = W.c3_source()
    t0 = time.time()
    T = tr(x, z, veln, velpn, vm, sd, vt, vt, 1e-3)
    print("C3 %.1fs" % (time.time() - t0), flush=True)
    save("c3_2048", field_dec8=T[::8, ::8].copy(), row_src=T[int(round(z / 1e-3))].copy(),
         elapsed=np.array(time.time() - t0))


def gen_c4():
    veln, velpn, vm, sd = W.weldlike_model()
    vt = W.default_table()
    dnx = W.weldlike_dnx()
    scx, scz = W.c4_sources(128)
    k = 64
    t0 = time.time()
    T = tr(scx[k], scz[k], veln, velpn, vm, sd, vt, vt, dnx)
    el = time.time() - t0
    print("C4 src %d %.1fs" % (k, el), flush=True)
    res = {"field_dec8": T[::8, ::8].copy(), "row_top": T[0].copy(), "src_index": np.array(k),
           "elapsed": np.array(el)}
    # F7: rays at 4096^2 sg=1 through a bottom receiver's TTF
    rec = (2056, 4095)
    t0 = time.time()
    TR = tr(dnx * rec[0], dnx * rec[1], veln, velpn, vm, sd, vt, vt, dnx)
    print("C4 receiver TTF %.1fs" % (time.time() - t0), flush=True)
    res["rec_field_dec8"] = TR[::8, ::8].copy()
    xs = [8, 1032, 2056, 3080, 4088]
    for x in xs:
        t0 = time.time()
        rx, ry, t = ref().find_ray(dnx, vt, np.array([float(x), 0.0]), np.array([float(rec[0]), float(rec[1])]), TR,
                                   veln, velpn, vm, sd, 1)
        res["ray_x_%d" % x], res["ray_y_%d" % x], res["time_%d" % x] = rx.copy(), ry.copy(), np.array(t)
        print("  ray x=%d time %.10e npts %d %.2fs" % (x, t, len(rx), time.time() - t0), flush=True)
    save("c4_weldlike", **res)


C4_WIN = 48  # half-width (nodes) of the full-resolution windows kept around the C4 source and receiver


def gen_c4_window():
    """The reference's C4 fields at full resolution in a (2 C4_WIN + 1)^2 window around source 64
    and around the F7 receiver (2056, 4095): pins the exact heap-ordered prefix cell by cell (the
    decimated c4_weldlike fields hold only a dozen cells inside it)."""
    veln, velpn, vm, sd = W.weldlike_model()
    vt = W.default_table()
    dnx = W.weldlike_dnx()
    scx, scz = W.c4_sources(128)
    res = {"half": np.array(C4_WIN)}
    for name, (x, z) in (("src", (int(round(scx[64] / dnx)), int(round(scz[64] / dnx)))), ("rec", (2056, 4095))):
        t0 = time.time()
        T = tr(dnx * x, dnx * z, veln, velpn, vm, sd, vt, vt, dnx)
        z0, z1 = max(0, z - C4_WIN), min(T.shape[0], z + C4_WIN + 1)
        x0, x1 = max(0, x - C4_WIN), min(T.shape[1], x + C4_WIN + 1)
        res[name + "_xz"] = np.array([x, z])
        res[name + "_box"] = np.array([z0, z1, x0, x1])
        res[name + "_win"] = T[z0:z1, x0:x1].copy()
        print("C4 %s window %.1fs" % (name, time.time() - t0), flush=True)
    save("c4_window", **res)


CORRIDOR_R = 6  # Chebyshev radius (fine nodes) kept around each rounded ray point at subgrid 1


def gen_c4_corridor():
    """F7 rays pinned on the reference's OWN 4096^2 receiver field: the field is kept only in a
    corridor of CORRIDOR_R nodes around each reference ray's points (find_ray :3104-3465 reads the
    plane sg ahead of round(last point), +-(3 sg + 1) candidates along it), NaN elsewhere.  The
    reference's find_ray is re-run on the corridor field and must return the identical ray and
    time, which proves the corridor holds every node the reference reads."""
    veln, velpn, vm, sd = W.weldlike_model()
    vt = W.default_table()
    dnx = W.weldlike_dnx()
    rec = (2056, 4095)
    t0 = time.time()
    TR = tr(dnx * rec[0], dnx * rec[1], veln, velpn, vm, sd, vt, vt, dnx)
    print("C4 receiver TTF %.1fs" % (time.time() - t0), flush=True)
    nz, nx = TR.shape
    keep = np.zeros(TR.shape, dtype=bool)
    res = {"receiver": np.array(rec, dtype=np.float64), "radius": np.array(CORRIDOR_R)}
    xs = [8, 1032, 2056, 3080, 4088]
    rays = {}
    for x in xs:
        rx, ry, t = ref().find_ray(dnx, vt, np.array([float(x), 0.0]), np.array([float(rec[0]), float(rec[1])]), TR,
                                   veln, velpn, vm, sd, 1)
        rays[x] = (rx.copy(), ry.copy(), float(t))
        for px, pz in zip(np.round(rx).astype(int), np.round(ry).astype(int)):
            keep[max(0, pz - CORRIDOR_R):pz + CORRIDOR_R + 1, max(0, px - CORRIDOR_R):px + CORRIDOR_R + 1] = True
        res["ray_x_%d" % x], res["ray_y_%d" % x], res["time_%d" % x] = rx.copy(), ry.copy(), np.array(t)
        print("  ray x=%d time %.10e npts %d" % (x, t, len(rx)), flush=True)
    TC = np.full(TR.shape, np.nan)
    TC[keep] = TR[keep]
    for x in xs:  # the corridor suffices: the reference on it == the reference on the whole field
        rx, ry, t = ref().find_ray(dnx, vt, np.array([float(x), 0.0]), np.array([float(rec[0]), float(rec[1])]), TC,
                                   veln, velpn, vm, sd, 1)
        assert t == rays[x][2] and np.array_equal(rx, rays[x][0]) and np.array_equal(ry, rays[x][1]), x
    idx = np.flatnonzero(keep).astype(np.int32)
    res["corridor_idx"] = idx
    res["corridor_val"] = TR.reshape(-1)[idx]
    res["shape"] = np.array([nz, nx])
    print("corridor %d nodes (%.2f %% of the field)" % (len(idx), 100.0 * len(idx) / TR.size), flush=True)
    save("c4_ray_corridor", **res)


def gen_local_ops():
    """update()/fouds18_A() on random 7x7 neighbourhoods.  Both read material only at (iz, ix)
    (:1368-1406, :286-315), so each case stores its centre material and fills the patch with it."""
    RR = ref()
    rng = np.random.default_rng(7)
    n = 7
    pad = 16
    g, p = mat_table(249.0e9, 133.0e9, 205.0e9, 125.0e9, 7850)
    tab_g = np.zeros((361, 3)); tab_g[:, 0] = np.arange(361); tab_g[:, 1] = 1.0; tab_g[:, 2] = g
    tab_p = np.zeros((361, 3)); tab_p[:, 0] = np.arange(361); tab_p[:, 1] = 1.0; tab_p[:, 2] = p
    NU, NF = 2500, 1500
    rec = {k: [] for k in ("u_ttn", "u_nsts", "u_mat", "u_stif", "u_args", "u_out",
                           "f_ttn", "f_nsts", "f_mat", "f_stif", "f_args", "f_out")}

    def rand_case():
        zz, xx = np.mgrid[0:n, 0:n]
        sz, sx = rng.uniform(-20, 30, 2)
        T = np.hypot(zz - sz, xx - sx) * rng.uniform(1e-7, 3e-7)
        T = T + rng.uniform(0, 2e-7) + rng.normal(0, 1, (n, n)) * 10 ** rng.uniform(-11, -8)
        if rng.random() < 0.15:
            T = np.round(T / 1e-8) * 1e-8  # exact ties
        T = np.abs(T)
        st = rng.choice([-1, 0, 3], size=(n, n), p=[0.35, 0.45, 0.2]).astype(np.int32)
        veln = rng.uniform(-50, 400) if rng.random() < 0.8 else float(np.round(rng.uniform(0, 180)))
        velpn = int(rng.integers(0, 3))
        vm = rng.uniform(0.5, 2.0) if rng.random() < 0.5 else 1.0
        stif = np.array([rng.integers(200000, 300000), rng.integers(100000, 150000), rng.integers(150000, 240000),
                         rng.integers(80000, 130000), rng.integers(7000, 9000)], dtype=np.int64)
        return T, st, veln, velpn, vm, stif

    def fill(veln, velpn, vm, stif):
        sd = np.empty((n, n, 5), dtype=np.int64)
        sd[:, :] = stif
        return (np.full((n, n), veln), np.full((n, n), velpn, dtype=np.int64), np.full((n, n), vm), sd)

    for it in range(NU):
        T, st, veln, velpn, vm, stif = rand_case()
        iz, ix = rng.integers(0, n, 2)
        quirk = rng.random() < 0.15
        nnz_arg = n + int(rng.integers(1, 5)) if quirk else n
        Tp = np.zeros((n + pad, n)); Tp[:n] = T
        Sp = -np.ones((n + pad, n), dtype=np.int32); Sp[:n] = st
        dnx = 10 ** rng.uniform(-5, -3)
        A = fill(veln, velpn, vm, stif)
        v = RR.update(A[0], A[1], A[2], Sp[:n], Tp[:n], int(iz), int(ix), dnx, nnz_arg, n, tab_p, A[3])
        rec["u_ttn"].append(T); rec["u_nsts"].append(st.astype(np.int8))
        rec["u_mat"].append([veln, velpn, vm]); rec["u_stif"].append(stif)
        rec["u_args"].append([iz, ix, dnx, nnz_arg, n])
        rec["u_out"].append(v)
    for it in range(NF):
        T, st, veln, velpn, vm, stif = rand_case()
        st[st > 0] = 1
        iz, ix = rng.integers(0, n, 2)
        dnx = 10 ** rng.uniform(-5, -3)
        if rng.random() < 0.5:
            T[iz, ix] = 0.0
        A = fill(veln, velpn, vm, stif)
        v = RR.fouds18_A(int(iz), int(ix), st, T, dnx, dnx, n, n, A[0], A[1], A[2], tab_g, A[3])
        rec["f_ttn"].append(T); rec["f_nsts"].append(st.astype(np.int8))
        rec["f_mat"].append([veln, velpn, vm]); rec["f_stif"].append(stif)
        rec["f_args"].append([iz, ix, dnx])
        rec["f_out"].append(v)
    out = {k: np.array(v) for k, v in rec.items()}
    out["tab_g"] = tab_g
    out["tab_p"] = tab_p
    nfb = int(np.sum(out["u_out"] == -1.0))
    print("update cases %d (returned -1: %d), fouds18 cases %d" % (NU, nfb, NF), flush=True)
    save("local_ops", **out)


def gen_tbp():
    RR = ref()
    veln, velpn, vm, sd = W.weld_model()
    vt = W.default_table()
    rng = np.random.default_rng(11)
    rows = []
    for sg in (1, 3, 9):
        fz, fx = sg * (veln.shape[0] - 1) + 1, sg * (veln.shape[1] - 1) + 1
        for it in range(700):
            x1 = float(rng.integers(0, fx)) if rng.random() < 0.5 else rng.uniform(0, fx - 1)
            y1 = float(rng.integers(0, fz)) if rng.random() < 0.5 else rng.uniform(0, fz - 1)
            L = rng.uniform(0, 4 * sg)
            kind = rng.random()
            if kind < 0.1:
                x2, y2 = x1, min(fz - 1, max(0, y1 + rng.choice([-1, 1]) * L))
            elif kind < 0.2:
                x2, y2 = min(fx - 1, max(0, x1 + rng.choice([-1, 1]) * L)), y1
            elif kind < 0.3:
                d = rng.choice([-1, 1]) * round(L)
                x2, y2 = min(fx - 1, max(0, x1 + d)), min(fz - 1, max(0, y1 + d))
            else:
                a = rng.uniform(0, 2 * np.pi)
                x2 = min(fx - 1, max(0, x1 + L * np.cos(a)))
                y2 = min(fz - 1, max(0, y1 + L * np.sin(a)))
            t = RR.time_between_points(x1, x2, y1, y2, 2e-4, sg, vt, veln, velpn, vm, sd)
            rows.append([x1, x2, y1, y2, sg, t])
    save("tbp_weld", rows=np.array(rows))


def gen_group_vel():
    RR = ref()
    ang = np.concatenate([np.linspace(0, 180, 1801), [0.005, 89.995, 90.005, 179.995, 45, 135, 30.5]])
    out = np.array([RR.group_vel(a, 249000, 133000, 205000, 125000, 7850, 1.0) for a in ang])
    out2 = np.array([RR.group_vel(a, 203600, 129800, 203600, 133500, 7874, 1.3) for a in ang])
    save("group_vel", angles=ang, set1=out, iron_scaled=out2)


GENS = {"fmm_small": gen_fmm_small, "c1": gen_c1, "kat": gen_kat, "weld1": lambda: gen_weld(1),
        "weld9": lambda: gen_weld(9), "c3": gen_c3, "c4": gen_c4, "c4_corridor": gen_c4_corridor, "c4_window": gen_c4_window, "local_ops": gen_local_ops, "tbp": gen_tbp,
        "group_vel": gen_group_vel}

if __name__ == "__main__":
    names = sys.argv[1:] or list(GENS)
    for nm in names:
        t0 = time.time()
        GENS[nm]()
        print("== %s done in %.1fs" % (nm, time.time() - t0), flush=True)
    man_path = os.path.join(OUT, "MANIFEST.json")
    man = json.load(open(man_path)) if os.path.exists(man_path) else {}
    with open("/root/reference/Anis_TTF_rays.py", "rb") as fh:
        man["reference_sha256"] = hashlib.sha256(fh.read()).hexdigest()
    man["generator"] = "oracle/gen_golden.py (numba %s, numpy %s, padded stage-1 semantics)" % (
        numba_boot.numba.__version__, np.__version__)
    man.setdefault("generated", {})
    for nm in names:
        man["generated"][nm] = time.strftime("%Y-%m-%d %H:%M:%S")
    json.dump(man, open(man_path, "w"), indent=1, sort_keys=True)
