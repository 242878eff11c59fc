"""GPU parity: the MI355X path (libalifmm.so through the drop-in module) against the oracle and the
reference's own golden vectors.  Run on the GPU box: pytest -m gpu.

Tolerances (justified by SURVEY.md §7 hard part 2 and Appendix C; every measured
error is also written to gpurun_out/parity_envelope.json, profiles/r2_parity_envelope.json keeps
the run the thresholds are set against, about 2x above it):
  * local operators, time_between_points, rays on a given field: bit-exact except where ocml's
    f64 atan/tan/sin/cos differ from glibc by an ulp -> rel <= 1e-12 per value, >= 99 % exact;
  * the exact prefix (every cell with T <= exact_r * dnx / vmax, heap order of the reference,
    :94-237 and :1512-1993): rel <= 1e-12;
  * travel-time fields (band-synchronous reformulation of the heap FMM), cells > 5 nodes from
    the source: rel L-inf <= 3e-3, rel mean <= 5e-5 on the C3, C4 and weld grids (FIELD_*), and
    SMALL_* on the 41..201-node cases, whose errors are larger relative to their small T;
  * ray travel times end-to-end (GPU fields + GPU rays): rel <= 5e-4 (RAY_END2END; C4's 4096-node
    rays 2.5e-3, K1-K3 against the notebook's 9 printed digits 1e-4).
"""
import numpy as np
import pytest

import oracle as O
import workloads as W

pytestmark = pytest.mark.gpu

# measured (profiles/r2_parity_envelope.json): C3 5.8e-4 / 1.9e-5, C4 9.0e-4 / 2.1e-5, weld sg1
# 1.3e-3 / 2.1e-5, weld sg9 6.0e-4 / 1.6e-5; small cases 2.9e-3 / 8.1e-5; rays: weld 6.2e-5, C4
# 1.2e-3 (through the GPU receiver field, whose own error is 3.5e-4), K1-K3 4.6e-5
FIELD_MAX, FIELD_MEAN = 3e-3, 5e-5
SMALL_MAX, SMALL_MEAN = 6e-3, 2e-4
RAY_END2END = 5e-4
RAY_C4 = 2.5e-3
KAT_END2END = 1e-4  # K1-K3: the notebook prints 9 significant digits of its numba run
EXACT = 1e-12


@pytest.fixture(scope="module")
def A():
    import Anis_TTF_rays as A

    return A


@pytest.fixture(scope="module")
def ctx():
    import _alifmm

    c = _alifmm.Context(0)
    yield c
    c.close()


def _field_err(T, Tref, src, excl=5):
    zz, xx = np.mgrid[0:T.shape[0], 0:T.shape[1]]
    m = np.hypot(zz - src[1], xx - src[0]) > excl
    r = np.abs(T[m] - Tref[m]) / Tref[m]
    return float(r.max()), float(r.mean())


def _check_field(envelope, name, T, Tref, src, excl=5, tol=(FIELD_MAX, FIELD_MEAN)):
    mx, mean = _field_err(T, Tref, src, excl)
    envelope[name] = {"rel_max": mx, "rel_mean": mean}
    assert mx <= tol[0] and mean <= tol[1], (name, mx, mean)


def _exact_pin(envelope, name, T, Tref, tstop, min_cells):
    """Every cell the exact heap walk finalises (T <= tstop, the walk's stop) equals the reference's
    value to 1e-12 relative (device transcendental ulps), the source cell exactly."""
    m = Tref <= 0.999 * tstop
    n = int(m.sum())
    rel = np.abs(T[m] - Tref[m]) / np.maximum(Tref[m], 1e-300)
    envelope[name] = {"cells": n, "rel_max": float(rel.max()) if n else None, "exact_frac": float(np.mean(T[m] == Tref[m]))}
    assert n >= min_cells, (name, n)
    assert rel.max() <= EXACT, (name, float(rel.max()))


def _ray_err(envelope, name, t, ref, tol=RAY_END2END):
    r = abs(t - ref) / ref
    envelope.setdefault(name, []).append(float(r))
    assert r <= tol, (name, t, ref)


def test_library_is_the_hip_build():
    import _alifmm

    assert _alifmm.device_count() >= 1
    assert b"gfx950" in _alifmm.lib().alifmm_version()


def test_local_ops_vs_reference_vectors(golden, ctx, envelope):
    g = golden("local_ops")
    n = len(g["u_out"])
    a = g["u_args"]
    out = ctx.local_ops(0, g["u_ttn"], g["u_nsts"].astype(np.int32), a[:, 0], a[:, 1], a[:, 2], a[:, 2], a[:, 3],
                        a[:, 4], g["u_mat"][:, 0], g["u_mat"][:, 1].astype(np.int64), g["u_mat"][:, 2], g["u_stif"],
                        g["tab_p"])
    ref = g["u_out"]
    exact = np.sum(out == ref)
    rel = np.abs(out - ref) / np.maximum(np.abs(ref), 1e-300)
    envelope["local_ops_update"] = {"exact_frac": float(exact / n), "rel_max": float(rel.max())}
    assert exact >= 0.99 * n and rel.max() <= 1e-12, (exact, n, rel.max())
    f = g["f_args"]
    m = len(g["f_out"])
    outf = ctx.local_ops(1, g["f_ttn"], g["f_nsts"].astype(np.int32), f[:, 0], f[:, 1], f[:, 2], f[:, 2],
                         np.full(m, 7), np.full(m, 7), g["f_mat"][:, 0], g["f_mat"][:, 1].astype(np.int64),
                         g["f_mat"][:, 2], g["f_stif"], g["tab_g"])
    reff = g["f_out"]
    exact = np.sum(outf == reff)
    rel = np.abs(outf - reff) / np.maximum(np.abs(reff), 1e-300)
    envelope["local_ops_fouds18"] = {"exact_frac": float(exact / m), "rel_max": float(rel.max())}
    assert exact >= 0.99 * m and rel.max() <= 1e-12, (exact, m, rel.max())


def test_time_between_points_vs_reference_vectors(golden, ctx, envelope):
    rows = golden("tbp_weld")["rows"]
    veln, velpn, vm, sd = W.weld_model()
    vt = W.default_table()
    ctx.set_model(veln, velpn, vm, sd, vt, vt, 2e-4)
    for sg in (1, 3, 9):
        r = rows[rows[:, 4] == sg]
        out = ctx.time_between_points(r[:, 0], r[:, 1], r[:, 2], r[:, 3], sg)
        rel = np.abs(out - r[:, 5]) / np.maximum(r[:, 5], 1e-300)
        envelope["tbp_sg%d" % sg] = {"exact_frac": float(np.mean(out == r[:, 5])), "rel_max": float(rel.max())}
        # every piece of the DDA evaluates atan/tan/cos (ocml vs glibc ulps): most values bit-exact
        assert np.mean(out == r[:, 5]) >= 0.9 and rel.max() <= 1e-12, (sg, np.mean(out == r[:, 5]), rel.max())


def test_fmm_small_fields(golden, A, envelope):
    g = golden("fmm_small")
    for k in range(int(g["ncases"])):
        p = "c%d_" % k
        dnx, x, z, sg = g[p + "meta"]
        stif = g[p + "stif"] if (p + "stif") in g else None
        veln = g[p + "veln"]
        if int(sg) == 1:
            T = A.travel(dnx * x, dnx * z, None, None, 0, np.zeros(veln.shape), veln, g[p + "velpn"], g[p + "vel_map"],
                         stif, g[p + "av"], g[p + "ph"], 0, 0, dnx, dnx, veln.shape[1], veln.shape[0])
            src = (x, z)
        else:
            T = A.travel_finer_grid(dnx * x, dnx * z, veln, g[p + "velpn"], g[p + "vel_map"], stif, int(sg),
                                    g[p + "av"], g[p + "ph"], 0, 0, dnx, dnx)
            src = (sg * x, sg * z)
        ref = g[p + "out"]
        assert T.shape == ref.shape
        _check_field(envelope, "fmm_small_%d_sg%d" % (k, int(sg)), T, ref, src, excl=5 * int(sg),
                     tol=(SMALL_MAX, SMALL_MEAN))


def test_c1_fields_analytic_and_exact_prefix(golden, A, envelope):
    g = golden("c1_fields")
    veln, velpn, vm, _ = W.c1_model()
    M = A.ALI_FMM(veln, velpn, vm, 1e-3 * g["src"][:, 0].astype(float), 1e-3 * g["src"][:, 1].astype(float))
    T = M.update(veln, velpn, vm)
    c = M._ctx(0)
    tstop = c.get_option("exact_r") * 1e-3 / c.get_option("vmax")
    zz, xx = np.mgrid[0:201, 0:201]
    for k, (x, z) in enumerate(g["src"]):
        _check_field(envelope, "c1_%d" % k, T[k], g["out"][k], (x, z), tol=(SMALL_MAX, SMALL_MEAN))
        _exact_pin(envelope, "exact_c1_%d" % k, T[k], g["out"][k], tstop, 200)
        r = np.hypot(zz - z, xx - x)
        m = r > 20
        rel = np.abs(T[k][m] - 1e-3 * r[m] / 5790.0) / (1e-3 * r[m] / 5790.0)
        assert rel.max() < 2.0e-2 and rel.mean() < 9e-3


def test_weld_sg1_field_rays_and_exact_prefix(golden, A, ctx, envelope):
    g = golden("weld_sg1")
    veln, velpn, vm, sd = W.weld_model()
    vt = W.default_table()
    scx, scz = W.weld_transducers()
    T = A.travel(scx[46], scz[46], None, None, 0, np.zeros(veln.shape), veln, velpn, vm, sd, vt, vt, 0, 0, 2e-4, 2e-4,
                 500, 424)
    _check_field(envelope, "weld_sg1", T, g["field"], (250, 423))
    ctx.set_model(veln, velpn, vm, sd, vt, vt, 2e-4)
    T2 = ctx.travel([scx[46]], [scz[46]])[0]
    assert np.array_equal(T2, T)
    _exact_pin(envelope, "exact_weld_sg1", T, g["field"], ctx.get_option("exact_r") * 2e-4 / ctx.get_option("vmax"),
               100)
    # ray tracer in isolation: the reference's own field in, the reference's rays out
    isx, isz = np.round(scx / 2e-4), np.round(scz / 2e-4)
    for i in (0, 15, 30):
        rx, ry, t = A.find_ray(2e-4, vt, [isx[i], isz[i]], [isx[46], isz[46]], g["field"], veln, velpn, vm, sd, 1)
        ref_t = float(g["time_%d" % i])
        assert abs(t - ref_t) / ref_t <= EXACT, (i, t, ref_t)
        assert len(rx) == len(g["ray_x_%d" % i])
        assert np.max(np.abs(rx - g["ray_x_%d" % i])) <= 1e-9 and np.max(np.abs(ry - g["ray_y_%d" % i])) <= 1e-9


def test_weld_sg9_field_and_rays(golden, A, envelope):
    """travel_finer_grid, subgrid 9 (the reference's weld example): 3808 x 4492 fine field, then
    rays 0/15/30 -> 46 on the GPU field vs the reference's rays on its own field."""
    g = golden("weld_sg9")
    veln, velpn, vm, sd = W.weld_model()
    vt = W.default_table()
    scx, scz = W.weld_transducers()
    T = A.travel_finer_grid(scx[46], scz[46], veln, velpn, vm, sd, 9, vt, vt, 0, 0, 2e-4, 2e-4)
    assert T.shape == tuple(g["fine_shape"])
    _check_field(envelope, "weld_sg9_dec9", T[::9, ::9], g["field_dec"], (250, 423))
    for nm, line, ref in (("row", T[T.shape[0] // 2], g["row_mid"]), ("col", T[:, T.shape[1] // 2], g["col_mid"])):
        r = np.abs(line - ref) / np.maximum(ref, 1e-300)
        envelope["weld_sg9_" + nm] = float(r.max())
        assert r.max() <= FIELD_MAX, r.max()
    isx, isz = np.round(scx / 2e-4), np.round(scz / 2e-4)
    for i in (0, 15, 30):
        rx, ry, t = A.find_ray(2e-4, vt, [9 * isx[i], 9 * isz[i]], [9 * isx[46], 9 * isz[46]], T, veln, velpn, vm,
                               sd, 9)
        _ray_err(envelope, "ray_weld_sg9", t, float(g["time_%d" % i]))


def test_notebook_kats_end_to_end(golden, A, envelope):
    """K1-K3 through the unchanged ALI_FMM surface (GPU fields + GPU rays) vs the published outputs."""
    g = golden("kat_notebook")
    dnx = 1e-3
    veln = 0 * np.ones((201, 201))
    velpn = 1 * np.ones((201, 201), dtype=int)
    vm = np.zeros((201, 201))
    for j in range(201):
        vm[:, j] = 3000 + 21 * j
    M = A.ALI_FMM(veln, velpn, vm, dnx * np.array([1, 199]), dnx * np.array([30, 180]), dnx=1e-3)
    t = M.find_all_TTF_rays(veln, velpn, vm)
    _ray_err(envelope, "kat_k1", t[0, 1], 5.08845096e-05, KAT_END2END)
    c22, c23, c33, c44, sigma = 249.0e9, 133.0e9, 205.0e9, 125.0e9, 7850
    vm1 = np.ones((201, 201))
    M1 = A.ALI_FMM(veln, velpn, vm1, dnx * np.array([1, 199]), dnx * np.array([100, 140]), dnx=1e-3)
    M1.add_materials(np.array([[c22, c23, c33, c44, 2 * sigma], [c22, c23, c33, c44, 3 * sigma]]), True)
    M1.add_materials(np.array([c22, c23, c33, c44, sigma]))
    assert np.array_equal(M1.velocity_dat, g["k2_group"]) and np.array_equal(M1.phase_vel, g["k2_phase"])
    trans = np.zeros((2, 2))
    trans[1, 0] = 1
    trans[0, 1] = 1
    t = M1.find_all_TTF_rays(veln, velpn, vm1, trans_pairs=trans)
    for (i, j), tp in {(0, 1): 3.54124066e-05, (1, 0): 3.54107926e-05}.items():
        _ray_err(envelope, "kat_k2", t[i, j], tp, KAT_END2END)
    sd = W.stif_field(201, 201)
    veln3 = 20 * np.ones((201, 201))
    velpn3 = 0 * np.ones((201, 201), dtype=int)
    M2 = A.ALI_FMM(veln3, velpn3, vm1, dnx * np.array([1, 199, 100]), dnx * np.array([100, 140, 1]), stif_den=sd,
                   dnx=1e-3)
    t = M2.find_all_TTF_rays(veln3, velpn3, vm1, stif_den=sd)
    for (i, j), tp in {(0, 1): 3.56081540e-05, (0, 2): 2.53646805e-05, (1, 2): 2.76255662e-05}.items():
        _ray_err(envelope, "kat_k3", t[i, j], tp, KAT_END2END)


def test_c3_2048_field_and_exact_prefix(golden, ctx, envelope):
    """BASELINE C3: 2048^2 Voronoi grains, stiffness everywhere, source (1024, 682), vs the reference
    field (every 8th node + the source row); the source row's exact-prefix cells to 1e-12."""
    g = golden("c3_2048")
    vt = W.default_table()
    ctx.set_model(*W.c3_model(), vt, vt, 1e-3)
    x, z = W.c3_source()
    T = ctx.travel([x], [z])[0]
    _check_field(envelope, "c3_dec8", T[::8, ::8], g["field_dec8"], (1024 / 8, 682 / 8), excl=1)
    r = np.abs(T[682] - g["row_src"]) / np.maximum(g["row_src"], 1e-300)
    r[1019:1030] = 0  # within 5 nodes of the source
    envelope["c3_row_src"] = float(r.max())
    assert r.max() <= FIELD_MAX, r.max()
    tstop = ctx.get_option("exact_r") * 1e-3 / ctx.get_option("vmax")
    _exact_pin(envelope, "exact_c3_row", T[682], g["row_src"], tstop, 10)


def test_c4_4096_fields_rays_and_batch_consistency(golden, ctx, envelope):
    """BASELINE C4/C5 grid (4096^2 weld-like): a top-surface source field and a bottom receiver
    field vs the reference (every 8th node, exact prefix included), the 5 reference rays end to
    end, and per-source fields that do not depend on the batch they were computed in (a 4-source
    batch vs single-source calls: bit-identical)."""
    g = golden("c4_weldlike")
    vt = W.default_table()
    dnx = W.weldlike_dnx()
    veln, velpn, vm, sd = W.weldlike_model()
    ctx.set_model(veln, velpn, vm, sd, vt, vt, dnx)
    tstop = ctx.get_option("exact_r") * dnx / ctx.get_option("vmax")
    sx, sz = W.c4_sources(128)
    k = int(g["src_index"])
    T = ctx.travel([sx[k]], [sz[k]])[0]
    _check_field(envelope, "c4_src%d_dec8" % k, T[::8, ::8], g["field_dec8"], ((16 + 32 * k) / 8, 0), excl=1)
    _exact_pin(envelope, "exact_c4_src", T[::8, ::8], g["field_dec8"], tstop, 3)
    TR = ctx.travel([dnx * 2056], [dnx * 4095])[0]
    _check_field(envelope, "c4_rec_dec8", TR[::8, ::8], g["rec_field_dec8"], (2056 / 8, 4095 / 8), excl=1)
    _exact_pin(envelope, "exact_c4_rec", TR[::8, ::8], g["rec_field_dec8"], tstop, 3)
    # the same fields at full resolution around the source and the receiver (c4_window: the
    # reference's own values in a 97 x 97 window): every cell of the exact heap-ordered prefix
    # cell by cell, the rest of the window within the field tolerance
    w = golden("c4_window")
    for name, F in (("src", T), ("rec", TR)):
        z0, z1, x0, x1 = (int(v) for v in w[name + "_box"])
        x, z = (int(v) for v in w[name + "_xz"])
        Fw, Rw = F[z0:z1, x0:x1], w[name + "_win"]
        _exact_pin(envelope, "exact_c4_%s_window" % name, Fw, Rw, tstop, 300)
        _check_field(envelope, "c4_%s_window" % name, Fw, Rw, (x - x0, z - z0))
    # batch independence: sources 0..3 together == each alone (sources never share state)
    B = ctx.travel(sx[:4], sz[:4])
    for i in (0, 3):
        assert np.array_equal(B[i], ctx.travel([sx[i]], [sz[i]])[0])
    assert np.array_equal(B[k], T) if k < 4 else True
    del B
    # rays through the reference's own receiver field are not available at full resolution in the
    # fixture (decimated), so trace through the GPU receiver field and compare end to end
    xs = (8, 1032, 2056, 3080, 4088)
    ctx.put_field(0, 1, TR)
    t, lens, flags, rays = ctx.find_rays([0] * 5, [[x, 0.0] for x in xs], [[2056.0, 4095.0]] * 5)
    for i, x in enumerate(xs):
        _ray_err(envelope, "ray_c4", t[i], float(g["time_%d" % x]), RAY_C4)
        rx = g["ray_x_%d" % x]
        assert abs(len(rays[i][0]) - len(rx)) <= 0.02 * len(rx), (x, len(rays[i][0]), len(rx))


def test_c4_full_128_source_batch(golden, ctx, envelope):
    """The benchmarked configuration itself: all 128 C4 sources in one call (auto members per
    source), fields left resident; the golden source's field vs the reference, and a few slots
    bit-identical to single-source calls (which run with 16 members per source)."""
    g = golden("c4_weldlike")
    vt = W.default_table()
    dnx = W.weldlike_dnx()
    ctx.set_model(*W.weldlike_model(), vt, vt, dnx)
    sx, sz = W.c4_sources(128)
    k = int(g["src_index"])
    ctx.travel(sx, sz, copy_out=False)
    kb = int(ctx.get_option("last_k"))
    Tk = ctx.get_field(k, 1)
    _check_field(envelope, "c4_batch128_src%d_dec8" % k, Tk[::8, ::8], g["field_dec8"], ((16 + 32 * k) / 8, 0),
                 excl=1)
    others = {i: ctx.get_field(i, 1) for i in (0, 127)}
    steps = [int(ctx.source_stats(i)[0][3]) for i in range(128)]
    envelope["c4_batch128"] = {"members": kb, "steps_mean": float(np.mean(steps))}
    assert all(s > 0 for s in steps)
    # the resident fields come back through copy_fields exactly as get_field returns them
    C, gbps = ctx.copy_fields(0, 2, 1)
    assert np.array_equal(C[0], others[0]) and gbps > 0
    for i, Ti in list(others.items()) + [(k, Tk)]:
        S = ctx.travel([sx[i]], [sz[i]])[0]
        assert int(ctx.get_option("last_k")) != kb or kb == 16
        assert np.array_equal(S, Ti), i
    # the whole batch streamed out of the band kernel tile by tile (alifmm_travel_into) into
    # non-consecutive rows of a larger stack, in reverse order: every field equals the resident one
    # and no row outside the destinations is touched
    fz, fx = ctx.field_shape(1)
    D = np.zeros((130, fz, fx))
    rows = list(range(129, 1, -1))
    ctx.travel_into(sx, sz, D, rows)
    envelope["c4_batch128_stream"] = {"tail_ms": ctx.get_option("stream_tail_ms"),
                                      "fallback_fields": ctx.get_option("stream_fallback")}
    assert ctx.get_option("stream_fallback") == 0
    for i in (0, 1, k, 126, 127):
        assert np.array_equal(D[rows[i]], ctx.get_field(i, 1)), i
        if i in others:
            assert np.array_equal(D[rows[i]], others[i]), i
    assert not D[0].any() and not D[1].any()
    del D
    ctx.release_fields()


def test_members_bit_identical(ctx, envelope):
    """One source over K = 2, 3, 4, 6, 16 workgroups (column stripes, one exchange per band step) gives
    the same bits as K = 1: C4 sources on stripe boundaries, the grid corners and the interior;
    the weld model at subgrid 3 (stage grids + fine-grid main loop)."""
    vt = W.default_table()
    dnx = W.weldlike_dnx()
    ctx.set_model(*W.weldlike_model(), vt, vt, dnx)
    xs = dnx * np.array([0.0, 63.0, 64.0, 2047.0, 4095.0, 1000.0])
    zs = dnx * np.array([0.0, 0.0, 100.0, 4095.0, 4095.0, 2000.0])
    try:
        ctx.set_option("members", 1)
        ref = ctx.travel(xs, zs)
        assert ctx.get_option("last_k") == 1.0
        for K in (2, 3, 4, 6, 16):
            ctx.set_option("members", K)
            F = ctx.travel(xs, zs)
            assert ctx.get_option("last_k") == K
            assert np.array_equal(F, ref), (K, [float(np.nanmax(np.abs(F[i] - ref[i]))) for i in range(len(xs))])
        del ref, F
        veln, velpn, vm, sd = W.weld_model()
        ctx.set_model(veln, velpn, vm, sd, vt, vt, 2e-4)
        scx, scz = W.weld_transducers()
        ctx.set_option("members", 1)
        ref = ctx.travel(scx[[0, 46]], scz[[0, 46]], subgrid=3)
        for K in (2, 5, 8):
            ctx.set_option("members", K)
            assert np.array_equal(ctx.travel(scx[[0, 46]], scz[[0, 46]], subgrid=3), ref), K
    finally:
        ctx.set_option("members", 0)
    ctx.release_fields()


def test_exact_walk_lds_equals_hbm(ctx, envelope):
    """travel_finer_grid()'s exact heap walk in LDS (fmm_exact_lds.hip: statuses, heap indices and
    speculative stencils in LDS) gives the same bits as the HBM walk (fmm_exact.hip) it replaces:
    weld sources on the bottom edge and in the interior (the whole 397 x 397 stage-1 grid) at
    subgrid 9, edge sources at subgrid 3 and 5 (Anis_TTF_rays.py:2187-2504, :2775-2817)."""
    vt = W.default_table()
    veln, velpn, vm, sd = W.weld_model()
    ctx.set_model(veln, velpn, vm, sd, vt, vt, 2e-4)
    scx, scz = W.weld_transducers()
    cases = [(np.array([scx[46], 250 * 2e-4]), np.array([scz[46], 212 * 2e-4]), 9),
             (scx[[0, 15, 46]], scz[[0, 15, 46]], 3), (scx[[30, 61]], scz[[30, 61]], 5)]
    try:
        for x, z, sg in cases:
            ctx.set_option("exact_lds", 0)
            ref = ctx.travel(x, z, subgrid=sg)
            ctx.set_option("exact_lds", 1)
            F = ctx.travel(x, z, subgrid=sg)
            same = [bool(np.array_equal(F[i], ref[i], equal_nan=True)) for i in range(len(x))]
            envelope.setdefault("exact_walk_lds_vs_hbm", []).append({"subgrid": sg, "bit_identical": same})
            assert all(same), (sg, same)
    finally:
        ctx.set_option("exact_lds", 1)
    ctx.release_fields()


def test_band_fouds18_path_vs_oracle(golden, ctx, envelope):
    """fouds18_A() as the band kernel runs it (the material record + the per-material slownesses
    precomputed by mat_slowness_kernel, fouds18<true>) against the oracle's fouds18_A with the
    same cell's material, on the reference's own neighbourhoods, for both material views (subgrid
    1 as is; subgrid > 1 with finer_grid_n's int32 orientation / float32 vel_map)."""
    g = golden("local_ops")
    vt = W.default_table()
    n = len(g["f_out"])
    f = g["f_args"]
    iz, ix, dnx = f[:, 0].astype(np.int32), f[:, 1].astype(np.int32), f[:, 2]
    nsts = g["f_nsts"].astype(np.int32)
    rng = np.random.default_rng(7)
    # weld: orientation columns; C3: per-cell stiffness (velpn 0) in every grain
    for name, (veln, velpn, vm, sd), dx in (("weld", W.weld_model(), 2e-4), ("c3", W.c3_model(512), 1e-3)):
        ctx.set_model(veln, velpn, vm, sd, vt, vt, dx)
        mz = rng.integers(0, veln.shape[0], n)
        mx = rng.integers(0, veln.shape[1], n)
        for quant in (0, 1):
            out = ctx.fouds18_band(g["f_ttn"], nsts, iz, ix, dnx, dnx, np.full(n, 7), np.full(n, 7), mz, mx, quant)
            ref = np.empty(n)
            for c in range(n):
                a, b = veln[mz[c], mx[c]], vm[mz[c], mx[c]]
                if quant:
                    a, b = float(int(a)), float(np.float32(b))
                st = None if sd is None else np.ascontiguousarray(np.broadcast_to(sd[mz[c], mx[c]], (7, 7, 5)))
                ref[c] = O.fouds18_A(int(iz[c]), int(ix[c]), nsts[c], g["f_ttn"][c], dnx[c], dnx[c], 7, 7,
                                     np.full((7, 7), a), np.full((7, 7), int(velpn[mz[c], mx[c]]), dtype=np.int64),
                                     np.full((7, 7), b), vt, st)
            rel = np.abs(out - ref) / np.maximum(np.abs(ref), 1e-300)
            envelope["fouds18_band_%s_q%d" % (name, quant)] = {"exact_frac": float(np.mean(out == ref)),
                                                               "rel_max": float(rel.max())}
            assert np.mean(out == ref) >= 0.99 and rel.max() <= EXACT, (name, quant, np.mean(out == ref), rel.max())


def test_weld_example_end_to_end(golden, A, envelope, tmp_path):
    """Weld_rays.py (the reference's example) through the unchanged ALI_FMM surface, minus plots:
    31 bottom receiver fields at subgrid 9 + 961 top->bottom rays (find_all_TTF_rays_parallel),
    the trimmed ray arrays the script saves, and rays 0/15/30 -> 46 vs the reference's times."""
    import raystore

    veln, velpn, vel_map, stif = W.weld_model()
    velpn = velpn.astype(int)
    sx, sy = W.weld_transducers()
    n = len(sx) // 2
    pairs = np.zeros((2 * n, 2 * n))
    pairs[:n, n:] = 1
    M = A.ALI_FMM(veln, velpn, vel_map, sx, sy, stif_den=stif, dnx=0.0002)
    t = M.find_all_TTF_rays_parallel(veln, velpn, vel_map, stif_den=stif, n_threads=8, trans_pairs=pairs)
    g = golden("weld_sg9")
    for i in (0, 15, 30):
        _ray_err(envelope, "ray_weld_example", t[i, 46], float(g["time_%d" % i]))
    assert np.all(t[:n, n:] > 0) and np.all(t[n:, :] == 0) and np.all(t[:n, :n] == 0)
    max_len = int(np.max(M.ray_len))
    assert 2 < max_len <= M.ray_paths_x.shape[2]
    k = int(M.ray_len[15, 46])
    rx, ry = M.ray_path(15, 46)
    assert len(rx) == k and abs(rx[0] - sx[15] / 0.0002) < 1e-9
    assert abs(ry[0] - 0) < 1e-12 and abs(ry[-1] - 423) < 1e-12 and abs(rx[-1] - 250) < 1e-12
    # compact ray storage: the same call with the dense arrays disabled gives the same
    # times, and the packed views read exactly like the dense arrays (Weld_rays.py:64-66 trimming)
    lim = A.ray_dense_limit_bytes
    try:
        A.ray_dense_limit_bytes = 0
        M2 = A.ALI_FMM(veln, velpn, vel_map, sx, sy, stif_den=stif, dnx=0.0002)
        t2 = M2.find_all_TTF_rays_parallel(veln, velpn, vel_map, stif_den=stif, n_threads=8, trans_pairs=pairs)
    finally:
        A.ray_dense_limit_bytes = lim
    assert isinstance(M2.ray_paths_x, A.PackedRayPaths)
    np.testing.assert_array_equal(t2, t)
    np.testing.assert_array_equal(M2.ray_len, M.ray_len)
    np.testing.assert_array_equal(M2.ray_paths_x[:, :, 0:max_len], M.ray_paths_x[:, :, 0:max_len])
    np.testing.assert_array_equal(M2.ray_paths_y[:, :, 0:max_len], M.ray_paths_y[:, :, 0:max_len])
    rx2, ry2 = M2.ray_path(15, 46)
    np.testing.assert_array_equal(rx2, rx)
    np.testing.assert_array_equal(ry2, ry)
    # save_ray_store round trip: the .npz reads back (np.load, no pickles) to the same rays
    path = str(tmp_path / "rays.npz")
    M2.save_ray_store(path)
    S = raystore.RayStore.load(path)
    np.testing.assert_array_equal(S.ray_len, M.ray_len)
    for i, j in ((0, 46), (15, 46), (30, 61)):
        x, z = S.path(i, j)
        np.testing.assert_array_equal(x, M.ray_paths_x[i, j, 0:M.ray_len[i, j]])
        np.testing.assert_array_equal(z, M.ray_paths_y[i, j, 0:M.ray_len[i, j]])


def test_update_parallel_low_mem_and_update_i(golden, A, envelope, tmp_path, monkeypatch):
    """update_parallel(low_mem=True) writes temp_TTF_<i>.npy per selected source into the working
    directory and returns None (:3938-4051, spill :3614/:3668), the files bit-equal to update();
    update_i (:4053-4088) at subgrid 1 and 9 equals the batch call's field, and at subgrid 9 the
    reference's weld field."""
    veln, velpn, vm, sd = W.weld_model()
    velpn = velpn.astype(int)
    sx, sy = W.weld_transducers()
    M = A.ALI_FMM(veln, velpn, vm, sx, sy, stif_den=sd, dnx=0.0002)
    sel = np.zeros(len(sx), dtype=int)
    sel[[3, 46, 60]] = 1
    F = M.update(veln, velpn, vm, stif_den=sd, subgrid_size=1, sources=sel)
    monkeypatch.chdir(tmp_path)
    assert M.update_parallel(veln, velpn, vm, stif_den=sd, subgrid_size=1, sources=sel, n_threads=2,
                             low_mem=True) is None
    assert sorted(p.name for p in tmp_path.iterdir()) == ["temp_TTF_3.npy", "temp_TTF_46.npy", "temp_TTF_60.npy"]
    for i in (3, 46, 60):
        np.testing.assert_array_equal(np.load(tmp_path / ("temp_TTF_%d.npy" % i)), F[i])
    np.testing.assert_array_equal(M.update_i(46, veln, velpn, vm, stif_den=sd, subgrid_size=1), F[46])
    T9 = M.update_i(46, veln, velpn, vm, stif_den=sd, subgrid_size=9)
    g = golden("weld_sg9")
    assert T9.shape == tuple(g["fine_shape"])
    _check_field(envelope, "update_i_sg9_dec9", T9[::9, ::9], g["field_dec"], (250, 423))
    sel9 = np.zeros(len(sx), dtype=int)
    sel9[46] = 1
    np.testing.assert_array_equal(M.update(veln, velpn, vm, stif_den=sd, subgrid_size=9, sources=sel9)[46], T9)


def test_sharded_contexts_bit_identical(A, monkeypatch):
    """per-source outputs are bit-identical whatever the number of GPUs the sources
    are dealt over.  ALIFMM_DEVICE_MAP=0,0,0 gives the *_parallel methods three independent
    contexts (streams, resident fields, host threads) on the box's one GPU, i.e. the multi-GPU
    sharding path (sharding.deal, rays traced where the receiver's field lives)."""
    veln, velpn, vm, sd = W.weld_model()
    velpn = velpn.astype(int)
    sx, sy = W.weld_transducers()
    sel = [0, 7, 20, 31, 40, 46, 55, 61]
    sx, sy = sx[sel], sy[sel]
    M1 = A.ALI_FMM(veln, velpn, vm, sx, sy, stif_den=sd, dnx=0.0002)
    F1 = M1.update(veln, velpn, vm, stif_den=sd, subgrid_size=1)
    monkeypatch.setenv("ALIFMM_DEVICE_MAP", "0,0,0")
    M3 = A.ALI_FMM(veln, velpn, vm, sx, sy, stif_den=sd, dnx=0.0002)
    assert M3._devices(8) == [0, 1, 2]
    F3 = M3.update_parallel(veln, velpn, vm, stif_den=sd, subgrid_size=1, n_threads=3)
    np.testing.assert_array_equal(F3, F1)
    n = len(sel)
    pairs = np.zeros((n, n))
    pairs[:4, 4:] = 1  # top transducers -> bottom receivers (Weld_rays.py:52-55)
    t1 = M1.find_all_TTF_rays(veln, velpn, vm, subgrid_size=1, trans_pairs=pairs, stif_den=sd)
    t3 = M3.find_all_TTF_rays_parallel(veln, velpn, vm, subgrid_size=1, trans_pairs=pairs, stif_den=sd, n_threads=3)
    np.testing.assert_array_equal(t3, t1)
    assert np.all(t1[:4, 4:] > 0)
    np.testing.assert_array_equal(M3.ray_len, M1.ray_len)
    for i in range(4):
        for j in range(4, n):
            for a, b in zip(M3.ray_path(i, j), M1.ray_path(i, j)):
                np.testing.assert_array_equal(a, b)


@pytest.mark.gpu
def test_sharded_contexts_bit_identical_c4(A, monkeypatch):
    """The same on BASELINE C4 (4096^2 weld-like, sources at z = 0): six of the 128 bench sources
    through update() on one context and through update_parallel() dealt over two contexts
    (ALIFMM_DEVICE_MAP=0,0 — the 2-GPU deal on one device) give bit-identical fields, although the
    two runs use different band-member counts per source (6 sources on one context vs 3 per
    context)."""
    veln, velpn, vm, sd = W.weldlike_model()
    dnx = W.weldlike_dnx()
    sx, sz = W.c4_sources(128)
    sel = [0, 1, 40, 64, 100, 127]
    sx, sz = sx[sel], sz[sel]
    M1 = A.ALI_FMM(veln, velpn, vm, sx, sz, stif_den=sd, dnx=dnx)
    F1 = M1.update(veln, velpn, vm, stif_den=sd, subgrid_size=1)
    monkeypatch.setenv("ALIFMM_DEVICE_MAP", "0,0")
    M2 = A.ALI_FMM(veln, velpn, vm, sx, sz, stif_den=sd, dnx=dnx)
    assert M2._devices(8) == [0, 1]
    F2 = M2.update_parallel(veln, velpn, vm, stif_den=sd, subgrid_size=1, n_threads=2)
    assert F1.shape == (6, 4096, 4096)
    np.testing.assert_array_equal(F2, F1)
    assert np.isfinite(F1).all()


def test_far_band_vs_band_model(ctx, envelope):
    """The far band (default: band width 1.4 x cdelta = 0.7 beyond Tmin = 768 dnx / vmax, ramped in
    up to 1536; subgrid 1), moved in to r_far = 256 so that it engages on a 401^2 anisotropic grain
    model whose front runs ~540 nodes from a corner source: the field equals the CPU band model's
    (oracle/band_model.c with the same schedule) to <= 1e-9 — the device applies the schedule the
    model states —, differs from the one-width band (the far band did engage), and stays within the
    small-grid bar vs the heap oracle (6e-3 / 2e-4)."""
    import _alifmm

    n, dnx = 401, 1e-3
    veln = W.voronoi_small(n, seed=5)
    velpn = np.zeros((n, n), dtype=np.int64)
    vm = np.ones((n, n))
    sd = W.stif_field(n, n)
    vt = W.default_table()
    sx, sz = 20, 20
    c1 = _alifmm.Context(0)
    c2 = _alifmm.Context(0)
    try:
        c1.set_model(veln, velpn, vm, sd, vt, vt, dnx)
        assert c1.get_option("cdelta") == 0.5 and c1.get_option("mat_jump") < 0.3  # grains: the default band
        assert c1.get_option("cdelta_far") == 0.7 and c1.get_option("r_far") == 768
        c1.set_option("r_far", 256)
        c1.travel([dnx * sx], [dnx * sz], copy_out=False)
        T = c1.get_field(0, 1)
        B, _ = O.band_travel(dnx * sx, dnx * sz, veln, velpn, vm, sd, vt, vt, c1.get_option("vmax"),
                             cdelta=c1.get_option("cdelta"), exact_init=True, r0=c1.get_option("r0"),
                             exact_r=c1.get_option("exact_r"), dnx=dnx, cdelta_far=0.7, r_far=256.0)
        dm = float(np.max(np.abs(T - B) / np.maximum(B, 1e-300)))
        envelope["far_band_vs_band_model_401"] = dm
        assert dm <= 1e-9, dm
        c2.set_option("cdelta_far", 0.0)
        c2.set_model(veln, velpn, vm, sd, vt, vt, dnx)
        c2.travel([dnx * sx], [dnx * sz], copy_out=False)
        assert not np.array_equal(c2.get_field(0, 1), T)
    finally:
        c1.close()
        c2.close()
    R = O.travel(dnx * sx, dnx * sz, veln, velpn, vm, sd, vt, vt, dnx=dnx)
    _check_field(envelope, "far_band_401", T, R, (sx, sz), tol=(6e-3, 2e-4))


@pytest.mark.parametrize("n", [61, 81])
def test_many_materials_paths(ctx, envelope, n):
    """Models past the kernels' LDS material tables: per-cell random orientations give n^2 distinct
    materials — 3 721 (> 256: the band kernel reads the model arrays, the ray tracer the per-cell
    ids and records from HBM) and 6 561 (> 4 096: no material ids at all).
      * field vs the CPU band model (oracle/band_model.c: the same band-synchronous reformulation,
        same band width, near-source schedule and exact prefix): the device arithmetic, <= 1e-9;
      * field vs the heap oracle within SURVEY's bar (1e-2 max, 1e-3 mean): the material changes at
        almost every cell pair (mat_jump ~1), so the library narrows the band to 0.2 by itself
        (context.h band_cdelta; at the default 0.5 this model measured 1.16e-2 / 1.2e-4);
      * a ray through the GPU field vs the oracle's on the same field: <= 1e-12."""
    rng = np.random.default_rng(n)
    dnx = 1e-3
    veln = rng.uniform(0.0, 180.0, (n, n))
    velpn = np.zeros((n, n), dtype=np.int64)
    vm = 1.0 + 0.2 * rng.random((n, n))
    sd = W.stif_field(n, n)
    vt = W.default_table()
    sx, sz = 17, 23
    ctx.set_model(veln, velpn, vm, sd, vt, vt, dnx)
    assert ctx.get_option("mat_jump") > 0.95
    assert ctx.get_option("cdelta") == 0.2 and abs(ctx.get_option("cdelta_far") - 0.28) < 1e-15
    ctx.travel([dnx * sx], [dnx * sz], copy_out=False)
    T = ctx.get_field(0, 1)
    B, _ = O.band_travel(dnx * sx, dnx * sz, veln, velpn, vm, sd, vt, vt, ctx.get_option("vmax"),
                         cdelta=ctx.get_option("cdelta"), exact_init=True, r0=ctx.get_option("r0"),
                         exact_r=ctx.get_option("exact_r"), dnx=dnx, cdelta_far=ctx.get_option("cdelta_far"),
                         r_far=ctx.get_option("r_far"))
    dm = float(np.max(np.abs(T - B) / np.maximum(B, 1e-300)))
    envelope["many_materials_vs_band_model_%d" % n] = dm
    assert dm <= 1e-9, (n, dm)
    R = O.travel(dnx * sx, dnx * sz, veln, velpn, vm, sd, vt, vt, dnx=dnx)
    _check_field(envelope, "many_materials_%d" % n, T, R, (sx, sz), tol=(1e-2, 1e-3))
    t, lens, flags, rays = ctx.find_rays([0], [[n - 5, n - 3]], [[sx, sz]])
    ox, oy, ot = O.find_ray(dnx, vt, [n - 5, n - 3], [sx, sz], T, veln, velpn, vm, sd, 1)
    envelope["many_materials_ray_%d" % n] = float(abs(t[0] - ot) / ot)
    assert int(lens[0]) == len(ox) and abs(t[0] - ot) <= EXACT * ot, (n, t[0], ot, int(lens[0]), len(ox))


def test_explicit_cdelta_far_band(envelope):
    """A caller's band width carries the far band with it: cdelta 0.3 alone gives a far
    band 1.4 x 0.3; an explicit cdelta_far narrower than the band width in force is raised to it;
    cdelta_far 0 turns it off.  The 401^2 grain field at cdelta 0.3 (far band engaged from r_far
    256) equals the CPU band model's with the same widths (<= 1e-9) and stays within the small-grid
    bar."""
    import _alifmm

    n, dnx = 401, 1e-3
    veln = W.voronoi_small(n, seed=5)
    velpn = np.zeros((n, n), dtype=np.int64)
    vm = np.ones((n, n))
    sd = W.stif_field(n, n)
    vt = W.default_table()
    sx, sz = 20, 20
    c = _alifmm.Context(0)
    try:
        c.set_option("cdelta", 0.3)
        c.set_option("r_far", 256)
        c.set_model(veln, velpn, vm, sd, vt, vt, dnx)
        cf = c.get_option("cdelta_far")
        assert c.get_option("cdelta") == 0.3 and abs(cf - 0.42) < 1e-15
        c.travel([dnx * sx], [dnx * sz], copy_out=False)
        T = c.get_field(0, 1)
        B, _ = O.band_travel(dnx * sx, dnx * sz, veln, velpn, vm, sd, vt, vt, c.get_option("vmax"),
                             cdelta=0.3, exact_init=True, r0=c.get_option("r0"), exact_r=c.get_option("exact_r"),
                             dnx=dnx, cdelta_far=cf, r_far=256.0)
        dm = float(np.max(np.abs(T - B) / np.maximum(B, 1e-300)))
        envelope["explicit_cdelta03_vs_band_model_401"] = dm
        assert dm <= 1e-9, dm
        R = O.travel(dnx * sx, dnx * sz, veln, velpn, vm, sd, vt, vt, dnx=dnx)
        _check_field(envelope, "explicit_cdelta03_401", T, R, (sx, sz), tol=(6e-3, 2e-4))
        c.set_option("cdelta_far", 0.25)
        assert c.get_option("cdelta_far") == 0.3  # never narrower than the band in force
        c.set_option("cdelta_far", 0.0)
        assert c.get_option("cdelta_far") == 0.0
    finally:
        c.close()


def test_rays_material_runs(ctx, envelope):
    """The ray kernel's material runs (rays.hip tbp_wave) on a model with many material changes per
    segment: per-cell orientations drawn from 100 values and a table / Christoffel mix (200
    materials: the LDS path with byte ids), so candidate segments cross up to five or more
    materials (runs past kRuns take the one-lane loop).  Rays through the GPU field: a request big
    enough for 9-lane groups (7 rays per wavefront) equals a small one (16-lane groups) bit for bit,
    and sampled rays equal the oracle's on the same field (<= 1e-12; bit-exact in practice)."""
    n = 61
    rng = np.random.default_rng(11)
    dnx = 1e-3
    veln = rng.integers(0, 100, (n, n)).astype(np.float64) * 1.7
    velpn = (rng.random((n, n)) < 0.3).astype(np.int64)  # 30 % table materials, the rest Christoffel
    vm = np.where(velpn == 1, 5790.0, 1.0)
    sd = W.stif_field(n, n)
    vt = W.default_table()
    sx, sz = 30, 2
    ctx.set_model(veln, velpn, vm, sd, vt, vt, dnx)
    assert 100 < ctx.get_option("nmat") <= 256
    ctx.travel([dnx * sx], [dnx * sz], copy_out=False)
    T = ctx.get_field(0, 1)
    srcs = np.array([[x, n - 1 - (x % 7)] for x in range(3, n - 3, 4)], dtype=np.float64)
    m = len(srcs)
    rec = np.tile([[sx, sz]], (m, 1)).astype(np.float64)
    t1, l1, f1, _ = ctx.find_rays(np.zeros(m, dtype=np.int32), srcs, rec, with_points=False)
    assert ctx.get_option("ray_lanes") == 16
    # 9-lane groups from the request that fills the device: n_cu x 4 SIMDs x waves per SIMD x 7 rays
    big = int(ctx.get_option("n_cu")) * 4 * int(ctx.get_option("ray_waves_per_simd")) * 7 + 5
    reps = -(-big // m)
    tb, lb, fb, _ = ctx.find_rays(np.zeros(m * reps, dtype=np.int32), np.tile(srcs, (reps, 1)),
                                  np.tile(rec, (reps, 1)), with_points=False)
    assert ctx.get_option("ray_lanes") == 9
    assert np.array_equal(tb.reshape(reps, m), np.tile(t1, (reps, 1)))
    assert np.array_equal(lb.reshape(reps, m), np.tile(l1, (reps, 1)))
    worst = 0.0
    for k in range(0, m, 3):
        ox, oy, ot = O.find_ray(dnx, vt, list(srcs[k]), [sx, sz], T, veln, velpn, vm, sd, 1)
        worst = max(worst, float(abs(t1[k] - ot) / ot))
        assert int(l1[k]) == len(ox) and abs(t1[k] - ot) <= EXACT * ot, (k, t1[k], ot, int(l1[k]), len(ox))
    envelope["ray_material_runs"] = worst


def test_empty_and_degenerate_requests(A, ctx, envelope):
    """Edge cases of the drop-in surface: no selected sources, no ray pairs, a 1-column grid, a
    source outside the grid (reference: IndexError-like failure -> the C-ABI's argument error)."""
    import _alifmm

    n = 41
    veln = np.zeros((n, n))
    velpn = np.ones((n, n), dtype=np.int64)
    vm = np.full((n, n), 5790.0)
    sx, sz = 1e-3 * np.array([5.0, 20.0, 35.0]), 1e-3 * np.array([0.0, 20.0, 40.0])
    M = A.ALI_FMM(veln, velpn, vm, sx, sz, dnx=1e-3)
    F = M.update(veln, velpn, vm, sources=np.zeros(3))
    assert F.shape == (3, n, n) and not F.any()
    t = M.find_all_TTF_rays(veln, velpn, vm, subgrid_size=1, trans_pairs=np.zeros((3, 3)))
    assert t.shape == (3, 3) and not t.any() and not M.ray_len.any()
    assert M.ray_path(0, 1) == (None, None)
    # empty batch through the C-ABI
    vt = W.default_table()
    ctx.set_model(veln, velpn, vm, None, vt, vt, 1e-3)
    assert ctx.travel(np.zeros(0), np.zeros(0), copy_out=True).shape[0] == 0
    # two-column grid (ragged extreme), source in the top corner: against the oracle
    v2, p2, m2 = np.zeros((n, 2)), np.ones((n, 2), dtype=np.int64), np.full((n, 2), 5790.0)
    T = A.travel(0.0, 0.0, None, None, 0, np.zeros((n, 2)), v2, p2, m2, None, vt, vt, 0, 0, 1e-3, 1e-3, 2, n)
    R = O.travel(0.0, 0.0, v2, p2, m2, None, vt, vt, dnx=1e-3)
    _check_field(envelope, "two_column", T, R, (0, 0), tol=(SMALL_MAX, SMALL_MEAN))
    # a source outside the grid is an argument error, not a fault
    with pytest.raises(_alifmm.AlifmmError):
        ctx.travel(np.array([1.0]), np.array([0.0]))
    # maximum sizes: a field side of 32 768 nodes (subgrid 1, or a subgrid that refines past it)
    # is refused up front (the kernels' packed 15-bit cell keys), not computed wrongly
    tall = 32768
    ctx.set_model(np.zeros((tall, 2)), np.ones((tall, 2), dtype=np.int64), np.full((tall, 2), 5790.0), None, vt, vt,
                  1e-3)
    with pytest.raises(_alifmm.AlifmmError, match="32768"):
        ctx.travel(np.array([0.0]), np.array([0.0]))
    ctx.set_model(np.zeros((3642, 2)), np.ones((3642, 2), dtype=np.int64), np.full((3642, 2), 5790.0), None, vt, vt,
                  1e-3)
    with pytest.raises(_alifmm.AlifmmError, match="32768"):
        ctx.travel(np.array([0.0]), np.array([0.0]), subgrid=9)  # 9 * 3641 + 1 = 32 770 fine rows
