"""GPU tests of the host paths around the kernels: the resident-model key (in-place edits reach the
GPU), the single-copy result return of update()/update_parallel(), and the RCCL gather of resident
fields through the library's C-ABI (alifmm_comm_* / alifmm_gather_fields; one rank on the one-GPU
box — the 8-GPU gather is the driver's)."""
import numpy as np
import pytest

import workloads as W

pytestmark = pytest.mark.gpu


def _small(n=81):
    veln = W.voronoi_small(n, seed=7)
    velpn = np.zeros((n, n), dtype=np.int64)
    vm = np.ones((n, n))
    sd = W.stif_field(n, n)
    return veln, velpn, vm, sd


def test_inplace_model_edit_reaches_the_gpu():
    """Reference: fields are recomputed from the arrays passed on every call (:1463).  An in-place
    edit of one interior cell (no sampling can miss it) changes the next field, equal to a fresh
    object's field on the edited model; the module-level travel() sees it too."""
    import Anis_TTF_rays as A

    n, dnx = 81, 1e-3
    veln, velpn, vm, sd = _small(n)
    scx, scz = dnx * np.array([20.0, 60.0]), dnx * np.array([0.0, 80.0])
    M = A.ALI_FMM(veln, velpn, vm, scx, scz, stif_den=sd, dnx=dnx)
    F0 = M.update(veln, velpn, vm, sd)
    veln[40:44, 37:41] += 35.0  # interior cells, in place
    F1 = M.update(veln, velpn, vm, sd)
    assert not np.array_equal(F0, F1)
    F2 = A.ALI_FMM(veln.copy(), velpn, vm, scx, scz, stif_den=sd, dnx=dnx).update(veln.copy(), velpn, vm, sd)
    assert np.array_equal(F1, F2)
    t = A.travel(scx[0], scz[0], None, None, 0, np.zeros((n, n)), veln, velpn, vm, sd, W.default_table(),
                 W.default_table(), 0, 0, dnx, dnx, n, n)
    sd[41, 39, 3] += 20000  # stiffness of one interior cell, in place
    t2 = A.travel(scx[0], scz[0], None, None, 0, np.zeros((n, n)), veln, velpn, vm, sd, W.default_table(),
                  W.default_table(), 0, 0, dnx, dnx, n, n)
    assert np.array_equal(t, F1[0]) and not np.array_equal(t, t2)


def test_update_single_copy_and_rccl_return(monkeypatch):
    """update() writes each field once, straight into the caller's stack (rows of unselected
    sources stay 0 as in the reference :3904-3936); update_parallel() with result_return = "rccl"
    (resident fields gathered to GPU 0 through alifmm_gather_fields, then copied out) returns the
    same bits."""
    import Anis_TTF_rays as A

    n, dnx = 81, 1e-3
    veln, velpn, vm, sd = _small(n)
    scx = dnx * np.array([5.0, 20.0, 40.0, 60.0, 75.0])
    scz = dnx * np.array([0.0, 80.0, 40.0, 0.0, 80.0])
    M = A.ALI_FMM(veln, velpn, vm, scx, scz, stif_den=sd, dnx=dnx)
    sel = np.array([1, 0, 1, 1, 0])
    F = M.update(veln, velpn, vm, sd, sources=sel)
    assert F.shape == (5, n, n) and not F[1].any() and not F[4].any()
    for i in (0, 2, 3):
        assert np.array_equal(F[i], M.update_i(i, veln, velpn, vm, sd))
    monkeypatch.setattr(A, "result_return", "rccl")
    P = M.update_parallel(veln, velpn, vm, sd, sources=sel, n_threads=2)
    assert np.array_equal(P, F)


def test_rccl_gather_one_rank_paths():
    """alifmm_gather_fields on a one-rank communicator: in place (destination = own slots) and into
    other slots (device-to-device), then the bad cases are refused with an error, not a crash."""
    import _alifmm

    n, dnx = 61, 1e-3
    veln, velpn, vm, sd = _small(n)
    vt = W.default_table()
    ctx = _alifmm.Context(0)
    comm = None
    try:
        ctx.set_model(veln, velpn, vm, sd, vt, vt, dnx)
        xs = dnx * np.array([3.0, 30.0, 55.0])
        ctx.travel(xs, np.zeros(3), copy_out=False)
        ref = ctx.copy_fields(0, 3, 1)[0]
        comm = _alifmm.Comm.all([ctx])
        ms = comm.gather(0, 1, [0], [3], dst_slot=0)  # in place
        assert ms >= 0 and np.array_equal(ctx.copy_fields(0, 3, 1)[0], ref)
        comm.gather(0, 1, [0], [3], dst_slot=3)  # into slots 3..5
        assert np.array_equal(ctx.copy_fields(3, 3, 1)[0], ref)
        with pytest.raises(_alifmm.AlifmmError):
            comm.gather(0, 1, [0], [3], dst_slot=1)  # overlaps the root's own fields
        with pytest.raises(_alifmm.AlifmmError):
            comm.gather(0, 1, [0], [9], dst_slot=0)  # slots 3.. hold fields, 6..8 do not exist
        # the root's copy into caller-chosen rows (the drop-in's _gather_into layout)
        dest = np.zeros((4, n, n))
        ctx.copy_fields_into(3, dest, [3, 0, 1], 1)
        assert np.array_equal(dest[3], ref[0]) and np.array_equal(dest[0], ref[1]) and np.array_equal(dest[1], ref[2])
        assert not dest[2].any()
        # registered-destination copy (dst_kind 3) == staging ring copy
        reg = np.empty((3, n, n))
        ctx.copy_fields_into(0, reg, [0, 1, 2], 1, dst_kind=3)
        assert np.array_equal(reg, ref)
    finally:
        if comm is not None:
            comm.close()
        ctx.close()


def test_option_environment_hook(monkeypatch):
    """ALIFMM_OPT_<NAME>=value sets the option on every new context (README "Options"); an unknown
    name or a non-numeric value is reported with a warning and ignored, never fatal."""
    import _alifmm

    monkeypatch.setenv("ALIFMM_OPT_R0", "30")
    monkeypatch.setenv("ALIFMM_OPT_NO_SUCH_OPTION", "1")
    monkeypatch.setenv("ALIFMM_OPT_CDELTA", "not-a-number")
    with pytest.warns(UserWarning):
        c = _alifmm.Context(0)
    try:
        assert c.get_option("r0") == 30.0
        assert c.get_option("cdelta") == 0.5  # the bad value left the default
    finally:
        c.close()
