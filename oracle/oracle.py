"""ctypes front-end of the CPU oracle (oracle/alifmm_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the parity checker.  The product (ali-fmm-and-ray-tracing_amd/) never
imports it.  Every function mirrors the reference function of the same name in
/root/reference/Anis_TTF_rays.py (cited per function) with the reference's argument meaning.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# ALIFMM_ORACLE_LIB: another build of the same restatement (lib/liboracle_cr.so, the CR-trig one)
_LIB_PATH = os.environ.get("ALIFMM_ORACLE_LIB") or os.path.join(_HERE, "lib", "liboracle.so")
_lib = None

_d = ctypes.c_double
_i = ctypes.c_int
_l = ctypes.c_long
_p = ctypes.c_void_p


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.oref_travel.restype = _i
        L.oref_travel.argtypes = [_d, _d, _i, _i, _p, _p, _p, _p, _p, _p, _i, _d, _d, _d, _d, _p]
        L.oref_travel_finer_grid.restype = _i
        L.oref_travel_finer_grid.argtypes = [_d, _d, _i, _i, _p, _p, _p, _p, _i, _p, _p, _i, _d, _d, _d, _d, _p]
        L.oref_travel_batch.restype = _i
        L.oref_travel_batch.argtypes = [_i, _p, _p, _i, _i, _p, _p, _p, _p, _i, _p, _p, _i, _d, _d, _d, _d, _p, _i]
        L.oref_time_between_points.restype = _d
        L.oref_time_between_points.argtypes = [_d, _d, _d, _d, _d, _i, _p, _i, _i, _i, _p, _p, _p, _p]
        L.oref_find_ray.restype = _l
        L.oref_find_ray.argtypes = [_d, _p, _i, _d, _d, _d, _d, _p, _i, _i, _i, _i, _p, _p, _p, _p, _i, _p, _p, _l,
                                    _p, _p]
        L.oref_update.restype = _d
        L.oref_update.argtypes = [_i, _i, _p, _p, _i, _i, _d, _i, _i, _p, _p, _p, _p, _p, _i]
        L.oref_fouds18.restype = _d
        L.oref_fouds18.argtypes = [_i, _i, _p, _p, _i, _i, _d, _d, _p, _p, _p, _p, _p, _i]
        L.oref_group_vel.restype = _d
        L.oref_group_vel.argtypes = [_d, _l, _l, _l, _l, _l, _d]
        _lib = L
    return _lib


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def _i64(a):
    return np.ascontiguousarray(a, dtype=np.int64)


def _ptr(a):
    return None if a is None else a.ctypes.data


class _Model:
    """Model arrays converted once to the dtypes the oracle reads (int64 velpn / stiffness)."""

    def __init__(self, veln, velpn, vel_map, stif_den, avlist2, phase_vel):
        self.veln = _f64(veln)
        self.velpn = _i64(velpn)
        self.vel_map = _f64(vel_map)
        self.stif = None if stif_den is None else _i64(stif_den)
        self.av = _f64(avlist2)
        self.ph = _f64(phase_vel if phase_vel is not None else avlist2)
        assert self.av.shape == self.ph.shape and self.av.shape[0] == 361
        self.nnz, self.nnx = self.veln.shape
        self.ncol = self.av.shape[1]


def travel(scx, scz, veln, velpn, vel_map, stif_den, avlist2, phase_vel, gox=0.0, goz=0.0, dnx=1e-3, dnz=None):
    """travel() Anis_TTF_rays.py:1463-2117 (fresh zero ttn; padded stage-1 semantics)."""
    m = _Model(veln, velpn, vel_map, stif_den, avlist2, phase_vel)
    dnz = dnx if dnz is None else dnz
    out = np.zeros((m.nnz, m.nnx))
    rc = lib().oref_travel(scx, scz, m.nnz, m.nnx, _ptr(m.veln), _ptr(m.velpn), _ptr(m.vel_map), _ptr(m.stif),
                           _ptr(m.av), _ptr(m.ph), m.ncol, gox, goz, dnx, dnz, _ptr(out))
    if rc:
        raise RuntimeError("oracle travel failed rc=%d" % rc)
    return out


def travel_finer_grid(scx, scz, veln, velpn, vel_map, stif_den, subgrid_size, avlist2, phase_vel, gox=0.0, goz=0.0,
                      dnx=1e-3, dnz=None):
    """travel_finer_grid() Anis_TTF_rays.py:2120-2832 (returns ttn / subgrid_size)."""
    m = _Model(veln, velpn, vel_map, stif_den, avlist2, phase_vel)
    dnz = dnx if dnz is None else dnz
    sg = int(subgrid_size)
    out = np.zeros((sg * (m.nnz - 1) + 1, sg * (m.nnx - 1) + 1))
    rc = lib().oref_travel_finer_grid(scx, scz, m.nnz, m.nnx, _ptr(m.veln), _ptr(m.velpn), _ptr(m.vel_map),
                                      _ptr(m.stif), sg, _ptr(m.av), _ptr(m.ph), m.ncol, gox, goz, dnx, dnz,
                                      _ptr(out))
    if rc:
        raise RuntimeError("oracle travel_finer_grid failed rc=%d" % rc)
    return out


def travel_batch(scx, scz, veln, velpn, vel_map, stif_den, avlist2, phase_vel, subgrid_size=1, gox=0.0, goz=0.0,
                 dnx=1e-3, dnz=None, n_threads=1):
    """Many independent sources, one per pthread (the reference's update_parallel :3938, minus its race)."""
    m = _Model(veln, velpn, vel_map, stif_den, avlist2, phase_vel)
    dnz = dnx if dnz is None else dnz
    scx = _f64(scx)
    scz = _f64(scz)
    sg = int(subgrid_size)
    fz, fx = (m.nnz, m.nnx) if sg <= 1 else (sg * (m.nnz - 1) + 1, sg * (m.nnx - 1) + 1)
    out = np.zeros((len(scx), fz, fx))
    rc = lib().oref_travel_batch(len(scx), _ptr(scx), _ptr(scz), m.nnz, m.nnx, _ptr(m.veln), _ptr(m.velpn),
                                 _ptr(m.vel_map), _ptr(m.stif), sg, _ptr(m.av), _ptr(m.ph), m.ncol, gox, goz, dnx,
                                 dnz, _ptr(out), int(n_threads))
    if rc:
        raise RuntimeError("oracle travel_batch failed rc=%d" % rc)
    return out


def time_between_points(x1, x2, y1, y2, dnx, subgrid_size, velocity_dat, veln, velpn, vel_map, stif_den):
    """time_between_points() Anis_TTF_rays.py:2835-2989."""
    m = _Model(veln, velpn, vel_map, stif_den, velocity_dat, velocity_dat)
    return lib().oref_time_between_points(float(x1), float(x2), float(y1), float(y2), dnx, int(subgrid_size),
                                          _ptr(m.av), m.ncol, m.nnz, m.nnx, _ptr(m.veln), _ptr(m.velpn),
                                          _ptr(m.vel_map), _ptr(m.stif))


def find_ray(dnx, velocity_dat, source, receiver, rec_TTF, veln, velpn, vel_map, stif_den, subgrid_size):
    """find_ray() Anis_TTF_rays.py:3104-3465 -> (ray_x, ray_y, trav_time) on the fine grid."""
    m = _Model(veln, velpn, vel_map, stif_den, velocity_dat, velocity_dat)
    ttf = _f64(rec_TTF)
    cap = 5 * (m.nnz + m.nnx)
    rx = np.zeros(cap)
    ry = np.zeros(cap)
    t = ctypes.c_double(0.0)
    early = ctypes.c_int(0)
    n = lib().oref_find_ray(dnx, _ptr(m.av), m.ncol, float(source[0]), float(source[1]), float(receiver[0]),
                            float(receiver[1]), _ptr(ttf), ttf.shape[0], ttf.shape[1], m.nnz, m.nnx, _ptr(m.veln),
                            _ptr(m.velpn), _ptr(m.vel_map), _ptr(m.stif), int(subgrid_size), _ptr(rx), _ptr(ry), cap,
                            ctypes.byref(t), ctypes.byref(early))
    if n < 0:
        raise RuntimeError("oracle find_ray failed rc=%d" % n)
    return rx[:n].copy(), ry[:n].copy(), t.value


def update(veln, velpn, vel_map, nsts, ttn, iz, ix, dnx, nnz, nnx, phase_vel, stif_den):
    """update() Anis_TTF_rays.py:904-1410 on caller arrays (nnz/nnx are the reference arguments)."""
    ttn = _f64(ttn)
    nsts = np.ascontiguousarray(nsts, dtype=np.int32)
    m = _Model(veln, velpn, vel_map, stif_den, phase_vel, phase_vel)
    return lib().oref_update(ttn.shape[0], ttn.shape[1], _ptr(ttn), _ptr(nsts), int(iz), int(ix), dnx, int(nnz),
                             int(nnx), _ptr(m.veln), _ptr(m.velpn), _ptr(m.vel_map), _ptr(m.stif), _ptr(m.ph), m.ncol)


def fouds18_A(iz, ix, nsts, ttn, dnx, dnz, nnx, nnz, veln, velpn, vel_map, avlist2, stif_den):
    """fouds18_A() Anis_TTF_rays.py:240-901 on caller arrays."""
    ttn = _f64(ttn)
    nsts = np.ascontiguousarray(nsts, dtype=np.int32)
    assert ttn.shape == (nnz, nnx)
    m = _Model(veln, velpn, vel_map, stif_den, avlist2, avlist2)
    return lib().oref_fouds18(int(nnz), int(nnx), _ptr(ttn), _ptr(nsts), int(iz), int(ix), dnx, dnz, _ptr(m.veln),
                              _ptr(m.velpn), _ptr(m.vel_map), _ptr(m.stif), _ptr(m.av), m.ncol)


def group_vel(angle, c_22, c_23, c_33, c_44, sigma, vel_scale=1):
    """group_vel() Anis_TTF_rays.py:3521-3558."""
    return lib().oref_group_vel(float(angle), int(c_22), int(c_23), int(c_33), int(c_44), int(sigma),
                                float(vel_scale))


def band_travel(scx, scz, veln, velpn, vel_map, stif_den, avlist2, phase_vel, vmax, cdelta=0.25, exact_init=False,
                sweeps=1, r0=0.0, exact_r=0.0, gox=0.0, goz=0.0, dnx=1e-3, dnz=None, cdelta_far=0.0, r_far=0.0):
    """CPU model of the MI355X band-synchronous formulation (oracle/band_model.c). Returns (T, steps[4]).
    cdelta_far / r_far: the device's optional wider band far from the source (0: off)."""
    m = _Model(veln, velpn, vel_map, stif_den, avlist2, phase_vel)
    dnz = dnx if dnz is None else dnz
    out = np.zeros((m.nnz, m.nnx))
    steps = np.zeros(4, dtype=np.int64)
    L = lib()
    L.oband_set_far.argtypes = [_d, _d]
    L.oband_set_far(float(cdelta_far), float(r_far))
    L.oband_travel.restype = _i
    L.oband_travel.argtypes = [_d, _d, _i, _i, _p, _p, _p, _p, _p, _p, _i, _d, _d, _d, _d, _d, _d, _i, _i, _d, _d, _p, _p]
    rc = L.oband_travel(scx, scz, m.nnz, m.nnx, _ptr(m.veln), _ptr(m.velpn), _ptr(m.vel_map), _ptr(m.stif),
                        _ptr(m.av), _ptr(m.ph), m.ncol, gox, goz, dnx, dnz, cdelta, vmax, int(exact_init),
                        int(sweeps), float(r0), float(exact_r), _ptr(out), _ptr(steps))
    if rc:
        raise RuntimeError("band model failed rc=%d" % rc)
    return out, steps
