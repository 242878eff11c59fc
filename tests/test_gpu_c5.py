"""BASELINE C5 on one MI355X, and the F7 rays pinned on the reference's own 4096^2 receiver field.

* C5 (full-matrix capture, two-array variant — the pair pattern of Weld_rays.py:52-55): 256 top
  transducers (z = 0) and 256 bottom ones (z = 4095), x = 8 + 16 k, on the 4096^2 weld-like grid;
  trans_pairs[i, 256 + j] = 1 -> 256 receiver fields + 65 536 rays, through the drop-in
  ALI_FMM.find_all_TTF_rays_parallel (reference :4550-4685) with compact ray storage.
* The reference's find_ray (:3104-3465) on its own C4 receiver field, kept in a corridor around
  each reference ray (tests/golden/c4_ray_corridor.npz, oracle/gen_golden.py gen_c4_corridor: the
  reference itself returns identical rays on the corridor field), traced by the GPU kernel.
"""
import json
import os
import time

import numpy as np
import pytest

import workloads as W

pytestmark = pytest.mark.gpu

RAY_C4 = 2.5e-3  # end-to-end ray time through the GPU receiver field (test_gpu_parity.RAY_C4)
EXACT = 1e-12
F7_X = (8, 1032, 2056, 3080, 4088)  # sources at z = 0, receiver (2056, 4095)


def _envelope_file():
    d = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
    os.makedirs(d, exist_ok=True)
    return os.path.join(d, "c5_capture.json")


def test_c4_rays_on_reference_field_corridor(golden, envelope):
    """find_ray_kernel on the reference's receiver field (corridor around each reference ray, NaN
    elsewhere): times <= 1e-12 relative and points <= 1e-9 fine nodes of the reference's, the same
    point count (reference find_ray :3104-3465, ray_time :2992-3022)."""
    import _alifmm

    g = golden("c4_ray_corridor")
    vt = W.default_table()
    dnx = W.weldlike_dnx()
    ctx = _alifmm.Context(0)
    try:
        ctx.set_model(*W.weldlike_model(), vt, vt, dnx)
        nz, nx = (int(v) for v in g["shape"])
        TC = np.full(nz * nx, np.nan)
        TC[g["corridor_idx"]] = g["corridor_val"]
        ctx.put_field(0, 1, TC.reshape(nz, nx))
        rec = [float(v) for v in g["receiver"]]
        t, lens, flags, rays = ctx.find_rays([0] * len(F7_X), [[x, 0.0] for x in F7_X], [rec] * len(F7_X))
        worst_t, worst_p = 0.0, 0.0
        for i, x in enumerate(F7_X):
            rx, ry, tr = g["ray_x_%d" % x], g["ray_y_%d" % x], float(g["time_%d" % x])
            assert len(rays[i][0]) == len(rx), (x, len(rays[i][0]), len(rx))
            worst_t = max(worst_t, abs(t[i] - tr) / tr)
            worst_p = max(worst_p, float(np.max(np.abs(rays[i][0] - rx))), float(np.max(np.abs(rays[i][1] - ry))))
        envelope["ray_c4_reference_corridor"] = {"time_rel_max": worst_t, "point_abs_max": worst_p,
                                                 "points": [int(v) for v in lens]}
        assert worst_t <= EXACT and worst_p <= 1e-9, (worst_t, worst_p)
    finally:
        ctx.close()


def test_c5_full_matrix_capture(golden, envelope):
    """C5 through the drop-in: 256 receiver fields + 65 536 rays on one GPU.  The F7 rays among them
    match the reference's C4 ray times (end to end through the GPU receiver field); every time is
    finite and positive; the compact store is consistent with ray_len; sampled pairs are
    bit-identical to single-pair calls (update_i + find_ray through the module functions)."""
    import Anis_TTF_rays as A

    g = golden("c4_weldlike")
    vt = W.default_table()
    dnx = W.weldlike_dnx()
    veln, velpn, vm, sd = W.weldlike_model()
    scx, scz, tp = W.c5_transducers()
    ns = len(scx) // 2
    M = A.ALI_FMM(veln, velpn, vm, scx, scz, stif_den=sd, dnx=dnx)
    t0 = time.perf_counter()
    times = M.find_all_TTF_rays_parallel(veln, velpn, vm, subgrid_size=1, trans_pairs=tp, stif_den=sd, n_threads=2)
    wall = time.perf_counter() - t0
    fields_ms = M._ctx(0).last_timing()[2]
    rays = times[:ns, ns:]
    assert np.all(np.isfinite(rays)) and np.all(rays > 0)
    assert np.count_nonzero(times) == ns * ns
    # compact storage: exactly the requested pairs, lengths summing to the stored points
    st = M.rays
    assert isinstance(M.ray_paths_x, A.PackedRayPaths)
    lens = st.ray_len
    assert np.all(lens[:ns, ns:] >= 2) and np.count_nonzero(lens) == ns * ns
    assert int(lens.sum()) == len(st.points)
    assert np.array_equal(M.ray_len, lens)
    # F7: receiver (2056, 4095) = bottom element 128; sources x = 8 + 16 i at z = 0
    j = ns + (2056 - 8) // 16
    errs = {}
    for x in F7_X:
        i = (x - 8) // 16
        ref = float(g["time_%d" % x])
        errs[x] = abs(times[i, j] - ref) / ref
        rx = g["ray_x_%d" % x]
        assert abs(int(lens[i, j]) - len(rx)) <= 0.02 * len(rx), (x, int(lens[i, j]), len(rx))
    # sampled pairs == single-pair calls (receiver field via update_i, ray via the module function)
    same = 0
    for jj, iis in ((j, (0, 77, 255)), (ns, (0, 128)), (2 * ns - 1, (3, 255))):
        T = M.update_i(jj, veln, velpn, vm, sd, subgrid_size=1)
        for ii in iis:
            x, z, t = A.find_ray(dnx, vt, [M.isx[ii], M.isz[ii]], [M.isx[jj], M.isz[jj]], T, veln, velpn, vm, sd, 1)
            px, pz = M.ray_path(ii, jj)
            assert t == times[ii, jj] and np.array_equal(x, px) and np.array_equal(z, pz), (ii, jj)
            same += 1
    rec = {"variant": "two-array: 256 top (z=0) x 256 bottom (z=4095) transducers, x = 8 + 16 k, "
                      "trans_pairs[i, 256 + j] = 1 (Weld_rays.py:52-55 pattern)",
           "receiver_fields": ns, "rays": int(ns * ns), "wall_s": wall, "fields_ms": fields_ms,
           "rays_and_host_s": wall - fields_ms / 1e3, "points": int(len(st.points)),
           # kernel / host split of the call (ALI_FMM.last_timing): fields, then per GPU the ray and
           # packing kernels (HIP events), the find_rays call, the points' copy-out and the host store
           "split": M.last_timing,
           "f7_time_rel_err": {str(k): float(v) for k, v in errs.items()}, "sampled_pairs_bit_identical": same}
    envelope["c5_capture"] = rec
    with open(_envelope_file(), "w") as f:
        json.dump(rec, f, indent=1)
    assert max(errs.values()) <= RAY_C4, errs
    for d in list(M._ctxs):
        M._ctxs[d].release_fields()
