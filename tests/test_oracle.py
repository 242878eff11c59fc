"""Pin the CPU oracle (oracle/alifmm_oracle.c) against vectors produced by the reference itself
(tests/golden/*.npz from oracle/gen_golden.py: numba 0.54, padded stage-1 semantics) and against the
published notebook outputs.  Bit-exact unless stated."""
import numpy as np
import pytest

import oracle as O
import workloads as W


def test_local_update_bitexact(golden):
    g = golden("local_ops")
    n = g["u_ttn"].shape[1]
    bad = 0
    for k in range(len(g["u_out"])):
        veln, velpn, vm = g["u_mat"][k]
        iz, ix, dnx, nnz_arg, nnx_arg = g["u_args"][k]
        sd = np.empty((n, n, 5), dtype=np.int64); sd[:, :] = g["u_stif"][k]
        v = O.update(np.full((n, n), veln), np.full((n, n), int(velpn)), np.full((n, n), vm), g["u_nsts"][k],
                     g["u_ttn"][k], int(iz), int(ix), dnx, int(nnz_arg), int(nnx_arg), g["tab_p"], sd)
        bad += v != g["u_out"][k]
    assert bad == 0


def test_local_fouds18_bitexact(golden):
    g = golden("local_ops")
    n = g["f_ttn"].shape[1]
    bad = 0
    for k in range(len(g["f_out"])):
        veln, velpn, vm = g["f_mat"][k]
        iz, ix, dnx = g["f_args"][k]
        sd = np.empty((n, n, 5), dtype=np.int64); sd[:, :] = g["f_stif"][k]
        v = O.fouds18_A(int(iz), int(ix), g["f_nsts"][k], g["f_ttn"][k], dnx, dnx, n, n, np.full((n, n), veln),
                        np.full((n, n), int(velpn)), np.full((n, n), vm), g["tab_g"], sd)
        bad += v != g["f_out"][k]
    assert bad == 0


def test_group_vel_bitexact(golden):
    g = golden("group_vel")
    a = np.array([O.group_vel(x, 249000, 133000, 205000, 125000, 7850, 1.0) for x in g["angles"]])
    b = np.array([O.group_vel(x, 203600, 129800, 203600, 133500, 7874, 1.3) for x in g["angles"]])
    assert np.array_equal(a, g["set1"]) and np.array_equal(b, g["iron_scaled"])


def test_time_between_points_bitexact(golden):
    rows = golden("tbp_weld")["rows"]
    veln, velpn, vm, sd = W.weld_model()
    vt = W.default_table()
    got = np.array([O.time_between_points(r[0], r[1], r[2], r[3], 2e-4, int(r[4]), vt, veln, velpn, vm, sd)
                    for r in rows])
    assert np.array_equal(got, rows[:, 5])


def test_fmm_small_bitexact(golden):
    g = golden("fmm_small")
    for k in range(int(g["ncases"])):
        p = "c%d_" % k
        dnx, x, z, sg = g[p + "meta"]
        stif = g[p + "stif"] if (p + "stif") in g else None
        args = (dnx * x, dnx * z, g[p + "veln"], g[p + "velpn"], g[p + "vel_map"], stif)
        if int(sg) == 1:
            T = O.travel(*args, g[p + "av"], g[p + "ph"], dnx=dnx)
        else:
            T = O.travel_finer_grid(*args, int(sg), g[p + "av"], g[p + "ph"], dnx=dnx)
        assert np.array_equal(T, g[p + "out"]), "case %d (src %s, sg %d)" % (k, (x, z), sg)


def test_c1_fields_bitexact_and_analytic(golden):
    g = golden("c1_fields")
    veln, velpn, vm, _ = W.c1_model()
    vt = W.default_table()
    zz, xx = np.mgrid[0:201, 0:201]
    for k, (x, z) in enumerate(g["src"]):
        T = O.travel(1e-3 * x, 1e-3 * z, veln, velpn, vm, None, vt, vt)
        assert np.array_equal(T, g["out"][k])
        r = np.hypot(zz - z, xx - x)
        m = r > 20
        rel = np.abs(T[m] - 1e-3 * r[m] / 5790.0) / (1e-3 * r[m] / 5790.0)
        # the reference's own discretisation error on C1: max 1.9e-2, mean <= 8.5e-3
        assert rel.max() < 2.0e-2 and rel.mean() < 9e-3


def test_weld_sg1_field_and_rays(golden):
    g = golden("weld_sg1")
    veln, velpn, vm, sd = W.weld_model()
    vt = W.default_table()
    scx, scz = W.weld_transducers()
    T = O.travel(scx[46], scz[46], veln, velpn, vm, sd, vt, vt, dnx=2e-4)
    assert np.array_equal(T, g["field"])
    isx, isz = np.round(scx / 2e-4), np.round(scz / 2e-4)
    for i in (0, 15, 30):
        rx, ry, t = O.find_ray(2e-4, vt, [isx[i], isz[i]], [isx[46], isz[46]], g["field"], veln, velpn, vm, sd, 1)
        assert np.array_equal(rx, g["ray_x_%d" % i]) and np.array_equal(ry, g["ray_y_%d" % i])
        assert t == float(g["time_%d" % i])


def test_weld_sg9_field_and_rays(golden):
    g = golden("weld_sg9")
    veln, velpn, vm, sd = W.weld_model()
    vt = W.default_table()
    scx, scz = W.weld_transducers()
    T = O.travel_finer_grid(scx[46], scz[46], veln, velpn, vm, sd, 9, vt, vt, dnx=2e-4)
    assert T.shape == tuple(g["fine_shape"])
    assert np.array_equal(T[::9, ::9], g["field_dec"])
    assert np.array_equal(T[T.shape[0] // 2], g["row_mid"]) and np.array_equal(T[:, T.shape[1] // 2], g["col_mid"])
    isx, isz = np.round(scx / 2e-4), np.round(scz / 2e-4)
    for i in (0, 15, 30):
        rx, ry, t = O.find_ray(2e-4, vt, [9 * isx[i], 9 * isz[i]], [9 * isx[46], 9 * isz[46]], T, veln, velpn, vm,
                               sd, 9)
        assert np.array_equal(rx, g["ray_x_%d" % i]) and np.array_equal(ry, g["ray_y_%d" % i])
        assert t == float(g["time_%d" % i])


def test_c3_2048_bitexact(golden):
    g = golden("c3_2048")
    veln, velpn, vm, sd = W.c3_model()
    x, z = W.c3_source()
    T = O.travel(x, z, veln, velpn, vm, sd, W.default_table(), W.default_table())
    assert np.array_equal(T[::8, ::8], g["field_dec8"]) and np.array_equal(T[682], g["row_src"])


def test_c4_weldlike_fields_and_rays(golden):
    g = golden("c4_weldlike")
    veln, velpn, vm, sd = W.weldlike_model()
    vt = W.default_table()
    dnx = W.weldlike_dnx()
    scx, scz = W.c4_sources(128)
    k = int(g["src_index"])
    T = O.travel(scx[k], scz[k], veln, velpn, vm, sd, vt, vt, dnx=dnx)
    assert np.array_equal(T[::8, ::8], g["field_dec8"]) and np.array_equal(T[0], g["row_top"])
    TR = O.travel(dnx * 2056, dnx * 4095, veln, velpn, vm, sd, vt, vt, dnx=dnx)
    assert np.array_equal(TR[::8, ::8], g["rec_field_dec8"])
    # the full-resolution windows around the source and the receiver (the GPU exact-prefix pin)
    w = golden("c4_window")
    for name, F in (("src", T), ("rec", TR)):
        z0, z1, x0, x1 = (int(v) for v in w[name + "_box"])
        assert np.array_equal(F[z0:z1, x0:x1], w[name + "_win"]), name
    for x in (8, 1032, 2056, 3080, 4088):
        rx, ry, t = O.find_ray(dnx, vt, [x, 0.0], [2056.0, 4095.0], TR, veln, velpn, vm, sd, 1)
        assert np.array_equal(rx, g["ray_x_%d" % x]) and np.array_equal(ry, g["ray_y_%d" % x])
        assert t == float(g["time_%d" % x])
    # the corridor fixture of the GPU ray pin (test_gpu_c5.py): the reference's own field values,
    # and the rays traced on the corridor alone are the reference's
    gc = golden("c4_ray_corridor")
    idx = gc["corridor_idx"]
    assert np.array_equal(TR.reshape(-1)[idx], gc["corridor_val"])
    TC = np.full(TR.size, np.nan)
    TC[idx] = gc["corridor_val"]
    TC = TC.reshape(TR.shape)
    for x in (8, 4088):
        rx, ry, t = O.find_ray(dnx, vt, [x, 0.0], [2056.0, 4095.0], TC, veln, velpn, vm, sd, 1)
        assert np.array_equal(rx, gc["ray_x_%d" % x]) and np.array_equal(ry, gc["ray_y_%d" % x])
        assert t == float(gc["time_%d" % x])


def _kat_rays(veln, velpn, vm, sd, vt, ph, scx, scz, pairs, sg, dnx=1e-3):
    isx, isz = np.round(scx / dnx), np.round(scz / dnx)
    out = {}
    for j in sorted(set(j for _, j in pairs)):
        T = O.travel_finer_grid(scx[j], scz[j], veln, velpn, vm, sd, sg, vt, ph, dnx=dnx)
        for (i, jj) in pairs:
            if jj == j:
                out[(i, j)] = O.find_ray(dnx, vt, [sg * isx[i], sg * isz[i]], [sg * isx[j], sg * isz[j]], T, veln,
                                         velpn, vm, sd, sg)
    return out


def test_notebook_kats(golden):
    """K1-K3: the notebook's published travel times (Ray tracing example.ipynb :305, :553-554, :733-734)."""
    g = golden("kat_notebook")
    dnx = 1e-3
    vt = W.default_table()
    # K1
    vm = np.zeros((201, 201)); vm[:, :] = 3000 + 21 * np.arange(201)[None, :]
    r = _kat_rays(np.zeros((201, 201)), np.ones((201, 201), dtype=np.int64), vm, np.zeros((201, 201, 5), np.int64),
                  vt, vt, dnx * np.array([1, 199]), dnx * np.array([30, 180]), [(0, 1)], 9)
    rx, ry, t = r[(0, 1)]
    assert t == g["k1_times"][0, 1]
    assert np.array_equal(rx / 9, g["k1_ray_x"]) and np.array_equal(ry / 9, g["k1_ray_y"])
    assert abs(t - 5.08845096e-05) / 5.08845096e-05 < 1e-8
    # K2 (first constant set; SURVEY B-D12)
    r = _kat_rays(np.zeros((201, 201)), np.ones((201, 201), dtype=np.int64), np.ones((201, 201)),
                  np.zeros((201, 201, 5), np.int64), g["k2_group"], g["k2_phase"], dnx * np.array([1, 199]),
                  dnx * np.array([100, 140]), [(0, 1), (1, 0)], 9)
    for (i, j) in [(0, 1), (1, 0)]:
        assert r[(i, j)][2] == g["k2_times"][i, j]
        assert np.array_equal(r[(i, j)][0] / 9, g["k2_ray_x_%d%d" % (i, j)])
    assert abs(r[(1, 0)][2] - 3.54107926e-05) / 3.54107926e-05 < 1e-8
    assert abs(r[(0, 1)][2] - 3.54124066e-05) / 3.54124066e-05 < 1e-4
    # K3
    sd = W.stif_field(201, 201)
    r = _kat_rays(20 * np.ones((201, 201)), np.zeros((201, 201), dtype=np.int64), np.ones((201, 201)), sd, vt, vt,
                  dnx * np.array([1, 199, 100]), dnx * np.array([100, 140, 1]), [(0, 1), (0, 2), (1, 2)], 9)
    pub = {(0, 1): 3.56081540e-05, (0, 2): 2.53646805e-05, (1, 2): 2.76255662e-05}
    for ij, tp in pub.items():
        assert r[ij][2] == g["k3_times"][ij]
        assert abs(r[ij][2] - tp) / tp < 5e-7
