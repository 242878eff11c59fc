"""GPU parity: the MI355X path (libalifmm.so through the drop-in module) against the oracle and the
reference's own golden vectors.  Run on the GPU box: pytest -m gpu.

Tolerances (justified by SURVEY.md §7 hard part 2 and Appendix C):
  * local operators, time_between_points, rays on a given field: bit-exact except where ocml's
    f64 atan/tan/sin/cos differ from glibc by an ulp -> rel <= 1e-12 per value, >= 99 % exact;
  * travel-time fields (band-synchronous reformulation of the heap FMM), cells > 5 nodes from
    the source: rel L-inf <= 1e-2, rel mean <= 1e-3;
  * ray travel times end-to-end (GPU fields + GPU rays): rel <= 5e-3.
"""
import numpy as np
import pytest

import oracle as O
import workloads as W

pytestmark = pytest.mark.gpu

FIELD_MAX, FIELD_MEAN, RAY_END2END = 1e-2, 1e-3, 5e-3


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
    return r.max(), r.mean()


def test_library_is_the_hip_build():
    import _alifmm

    assert _alifmm.device_count() >= 1
    assert b"gfx950" in _alifmm.lib().alifmm_version()


def test_local_ops_vs_reference_vectors(golden, ctx):
    g = golden("local_ops")
    n = len(g["u_out"])
    a = g["u_args"]
    out = ctx.local_ops(0, g["u_ttn"], g["u_nsts"].astype(np.int32), a[:, 0], a[:, 1], a[:, 2], a[:, 2], a[:, 3],
                        a[:, 4], g["u_mat"][:, 0], g["u_mat"][:, 1].astype(np.int64), g["u_mat"][:, 2], g["u_stif"],
                        g["tab_p"])
    ref = g["u_out"]
    exact = np.sum(out == ref)
    rel = np.abs(out - ref) / np.maximum(np.abs(ref), 1e-300)
    assert exact >= 0.99 * n and rel.max() <= 1e-12, (exact, n, rel.max())
    f = g["f_args"]
    m = len(g["f_out"])
    outf = ctx.local_ops(1, g["f_ttn"], g["f_nsts"].astype(np.int32), f[:, 0], f[:, 1], f[:, 2], f[:, 2],
                         np.full(m, 7), np.full(m, 7), g["f_mat"][:, 0], g["f_mat"][:, 1].astype(np.int64),
                         g["f_mat"][:, 2], g["f_stif"], g["tab_g"])
    reff = g["f_out"]
    exact = np.sum(outf == reff)
    rel = np.abs(outf - reff) / np.maximum(np.abs(reff), 1e-300)
    assert exact >= 0.99 * m and rel.max() <= 1e-12, (exact, m, rel.max())


def test_time_between_points_vs_reference_vectors(golden, ctx):
    rows = golden("tbp_weld")["rows"]
    veln, velpn, vm, sd = W.weld_model()
    vt = W.default_table()
    ctx.set_model(veln, velpn, vm, sd, vt, vt, 2e-4)
    for sg in (1, 3, 9):
        r = rows[rows[:, 4] == sg]
        out = ctx.time_between_points(r[:, 0], r[:, 1], r[:, 2], r[:, 3], sg)
        rel = np.abs(out - r[:, 5]) / np.maximum(r[:, 5], 1e-300)
        # every piece of the DDA evaluates atan/tan/cos (ocml vs glibc ulps): most values bit-exact
        assert np.mean(out == r[:, 5]) >= 0.9 and rel.max() <= 1e-12, (sg, np.mean(out == r[:, 5]), rel.max())


def test_fmm_small_fields(golden, A):
    g = golden("fmm_small")
    worst = []
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
        mx, mean = _field_err(T, ref, src, excl=5 * int(sg))
        worst.append((k, mx, mean))
    bad = [w for w in worst if w[1] > FIELD_MAX or w[2] > FIELD_MEAN]
    assert not bad, bad


def test_c1_fields_and_analytic(golden, A):
    g = golden("c1_fields")
    veln, velpn, vm, _ = W.c1_model()
    M = A.ALI_FMM(veln, velpn, vm, 1e-3 * g["src"][:, 0].astype(float), 1e-3 * g["src"][:, 1].astype(float))
    T = M.update(veln, velpn, vm)
    zz, xx = np.mgrid[0:201, 0:201]
    for k, (x, z) in enumerate(g["src"]):
        mx, mean = _field_err(T[k], g["out"][k], (x, z))
        assert mx <= FIELD_MAX and mean <= FIELD_MEAN, (k, mx, mean)
        r = np.hypot(zz - z, xx - x)
        m = r > 20
        rel = np.abs(T[k][m] - 1e-3 * r[m] / 5790.0) / (1e-3 * r[m] / 5790.0)
        assert rel.max() < 2.0e-2 and rel.mean() < 9e-3


def test_weld_sg1_field_and_rays(golden, A, ctx):
    g = golden("weld_sg1")
    veln, velpn, vm, sd = W.weld_model()
    vt = W.default_table()
    scx, scz = W.weld_transducers()
    T = A.travel(scx[46], scz[46], None, None, 0, np.zeros(veln.shape), veln, velpn, vm, sd, vt, vt, 0, 0, 2e-4, 2e-4,
                 500, 424)
    mx, mean = _field_err(T, g["field"], (250, 423))
    assert mx <= FIELD_MAX and mean <= FIELD_MEAN, (mx, mean)
    # ray tracer in isolation: the reference's own field in, the reference's rays out
    isx, isz = np.round(scx / 2e-4), np.round(scz / 2e-4)
    for i in (0, 15, 30):
        rx, ry, t = A.find_ray(2e-4, vt, [isx[i], isz[i]], [isx[46], isz[46]], g["field"], veln, velpn, vm, sd, 1)
        ref_t = float(g["time_%d" % i])
        assert abs(t - ref_t) / ref_t <= 1e-12, (i, t, ref_t)
        assert len(rx) == len(g["ray_x_%d" % i])
        assert np.max(np.abs(rx - g["ray_x_%d" % i])) <= 1e-9 and np.max(np.abs(ry - g["ray_y_%d" % i])) <= 1e-9


def test_weld_sg9_field_and_rays(golden, A):
    """travel_finer_grid, subgrid 9 (the reference's weld example): 3808 x 4492 fine field, then
    rays 0/15/30 -> 46 on the GPU field vs the reference's rays on its own field."""
    g = golden("weld_sg9")
    veln, velpn, vm, sd = W.weld_model()
    vt = W.default_table()
    scx, scz = W.weld_transducers()
    T = A.travel_finer_grid(scx[46], scz[46], veln, velpn, vm, sd, 9, vt, vt, 0, 0, 2e-4, 2e-4)
    assert T.shape == tuple(g["fine_shape"])
    dec = T[::9, ::9]
    mx, mean = _field_err(dec, g["field_dec"], (250, 423))
    assert mx <= FIELD_MAX and mean <= FIELD_MEAN, (mx, mean)
    for line, ref in ((T[T.shape[0] // 2], g["row_mid"]), (T[:, T.shape[1] // 2], g["col_mid"])):
        r = np.abs(line - ref) / np.maximum(ref, 1e-300)
        assert r.max() <= FIELD_MAX, r.max()
    isx, isz = np.round(scx / 2e-4), np.round(scz / 2e-4)
    for i in (0, 15, 30):
        rx, ry, t = A.find_ray(2e-4, vt, [9 * isx[i], 9 * isz[i]], [9 * isx[46], 9 * isz[46]], T, veln, velpn, vm,
                               sd, 9)
        ref_t = float(g["time_%d" % i])
        assert abs(t - ref_t) / ref_t <= RAY_END2END, (i, t, ref_t)


def test_notebook_kats_end_to_end(golden, A):
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
    assert abs(t[0, 1] - 5.08845096e-05) / 5.08845096e-05 <= RAY_END2END
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
        assert abs(t[i, j] - tp) / tp <= RAY_END2END
    sd = W.stif_field(201, 201)
    veln3 = 20 * np.ones((201, 201))
    velpn3 = 0 * np.ones((201, 201), dtype=int)
    M2 = A.ALI_FMM(veln3, velpn3, vm1, dnx * np.array([1, 199, 100]), dnx * np.array([100, 140, 1]), stif_den=sd,
                   dnx=1e-3)
    t = M2.find_all_TTF_rays(veln3, velpn3, vm1, stif_den=sd)
    for (i, j), tp in {(0, 1): 3.56081540e-05, (0, 2): 2.53646805e-05, (1, 2): 2.76255662e-05}.items():
        assert abs(t[i, j] - tp) / tp <= RAY_END2END


def test_c3_2048_field(golden, ctx):
    """BASELINE C3: 2048^2 Voronoi grains, stiffness everywhere, source (1024, 682), vs the reference
    field (every 8th node + the source row)."""
    g = golden("c3_2048")
    vt = W.default_table()
    ctx.set_model(*W.c3_model(), vt, vt, 1e-3)
    x, z = W.c3_source()
    T = ctx.travel([x], [z])[0]
    mx, mean = _field_err(T[::8, ::8], g["field_dec8"], (1024 / 8, 682 / 8), excl=1)
    assert mx <= FIELD_MAX and mean <= FIELD_MEAN, (mx, mean)
    r = np.abs(T[682] - g["row_src"]) / np.maximum(g["row_src"], 1e-300)
    r[1019:1030] = 0  # within 5 nodes of the source
    assert r.max() <= FIELD_MAX, r.max()


def test_c4_4096_fields_rays_and_batch_consistency(golden, ctx):
    """BASELINE C4/C5 grid (4096^2 weld-like): a top-surface source field and a bottom receiver
    field vs the reference (every 8th node), the 5 reference rays through the REFERENCE's receiver
    field (ray kernel in isolation, bit-level), and per-source fields that do not depend on the
    batch they were computed in (a 4-source batch vs single-source calls: bit-identical)."""
    g = golden("c4_weldlike")
    vt = W.default_table()
    dnx = W.weldlike_dnx()
    veln, velpn, vm, sd = W.weldlike_model()
    ctx.set_model(veln, velpn, vm, sd, vt, vt, dnx)
    sx, sz = W.c4_sources(128)
    k = int(g["src_index"])
    T = ctx.travel([sx[k]], [sz[k]])[0]
    mx, mean = _field_err(T[::8, ::8], g["field_dec8"], ((16 + 32 * k) / 8, 0), excl=1)
    assert mx <= FIELD_MAX and mean <= FIELD_MEAN, (mx, mean)
    TR = ctx.travel([dnx * 2056], [dnx * 4095])[0]
    mx, mean = _field_err(TR[::8, ::8], g["rec_field_dec8"], (2056 / 8, 4095 / 8), excl=1)
    assert mx <= FIELD_MAX and mean <= FIELD_MEAN, (mx, mean)
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
        ref_t = float(g["time_%d" % x])
        assert abs(t[i] - ref_t) / ref_t <= RAY_END2END, (x, t[i], ref_t)
        rx = g["ray_x_%d" % x]
        assert abs(len(rays[i][0]) - len(rx)) <= 0.02 * len(rx), (x, len(rays[i][0]), len(rx))


def test_weld_example_end_to_end(golden, A):
    """Weld_rays.py (the reference's example) through the unchanged ALI_FMM surface, minus plots:
    31 bottom receiver fields at subgrid 9 + 961 top->bottom rays (find_all_TTF_rays_parallel),
    the trimmed ray arrays the script saves, and rays 0/15/30 -> 46 vs the reference's times."""
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
        ref = float(g["time_%d" % i])
        assert abs(t[i, 46] - ref) / ref <= RAY_END2END, (i, t[i, 46], ref)
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


def test_pair_kernel_identical_to_single_workgroup(ctx):
    """Two workgroups per source (fmm_band_pair.hip) vs one (fmm_band.hip): bit-identical fields,
    subgrid 1 on the C4 grid (sources across stripe boundaries and the grid corner) and subgrid 3
    on the weld model."""
    vt = W.default_table()
    dnx = W.weldlike_dnx()
    ctx.set_model(*W.weldlike_model(), vt, vt, dnx)
    xs = dnx * np.array([0.0, 63.0, 64.0, 2047.0, 4095.0, 1000.0])
    zs = dnx * np.array([0.0, 0.0, 100.0, 4095.0, 4095.0, 2000.0])
    ctx.set_option("pair", 1)
    A = ctx.travel(xs, zs)
    assert ctx.get_option("last_pair") == 1.0
    ctx.set_option("pair", 0)
    Bf = ctx.travel(xs, zs)
    assert ctx.get_option("last_pair") == 0.0
    ctx.set_option("pair", 1)
    assert np.array_equal(A, Bf), [float(np.max(np.abs(A[i] - Bf[i]))) for i in range(len(xs))]
    del A, Bf
    veln, velpn, vm, sd = W.weld_model()
    ctx.set_model(veln, velpn, vm, sd, vt, vt, 2e-4)
    scx, scz = W.weld_transducers()
    A = ctx.travel(scx[[0, 46]], scz[[0, 46]], subgrid=3)
    ctx.set_option("pair", 0)
    Bf = ctx.travel(scx[[0, 46]], scz[[0, 46]], subgrid=3)
    ctx.set_option("pair", 1)
    assert np.array_equal(A, Bf)


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


def test_empty_and_degenerate_requests(A, ctx):
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
    mx, mean = _field_err(T, R, (0, 0))
    assert mx <= FIELD_MAX and mean <= FIELD_MEAN, (mx, mean)
    # a source outside the grid is an argument error, not a fault
    with pytest.raises(_alifmm.AlifmmError):
        ctx.travel(np.array([1.0]), np.array([0.0]))
