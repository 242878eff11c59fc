"""
Anisotropic travel-time fields and ray tracing — MI355X drop-in for the reference module
``Anis_TTF_rays`` (WiPi-UoS/ALI-FMM-and-ray-tracing, Anis_TTF_rays.py).

Same names, positional signatures, argument meaning, return values and error behaviour as the
reference, so ``Weld_rays.py`` and the tutorial notebook run unchanged.  The hot path runs on the
GPU through the C-ABI of ``lib/libalifmm.so`` (include/alifmm.h):

  travel / travel_finer_grid        -> alifmm_travel      (exact-heap source init in LDS +
                                                           band-synchronous FMM, csrc/fmm_*.hip)
  find_ray / ray_time               -> alifmm_find_rays   (one wavefront per ray, csrc/rays.hip)
  time_between_points               -> alifmm_time_between_points
  update / fouds18_A                -> alifmm_local_ops   (the reference's local operators)

Host-side utilities that are not on the hot path (velocity-table generation, material tables,
grid refinement helpers, plotting) are plain Python/numpy with the reference's semantics.
There is no CPU fallback: without the library or a GPU every GPU entry point raises.
Parity contract (what matches the reference bit-for-bit and what within a stated tolerance):
DESIGN.md §4.
"""
import math
import os
import sys
import threading

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import _alifmm  # noqa: E402
import sharding  # noqa: E402
from raystore import PackedRayPaths, RayStore  # noqa: E402

# Parameter used to enable/disable progress bars (reference :22-24; kept for API compatibility)
tqdm_disable = False

_EARLY_MSG = "Travel time to receiver increasing: Finishing ray early"

# Largest dense ray array (bytes, per coordinate) that find_all_TTF_rays* still materialises like
# the reference (:4286-4289); above it ray_paths_x / ray_paths_y are PackedRayPaths views of the
# compact RayStore (ALI_FMM.rays), e.g. for the 4096² full-matrix capture (86 GB per dense array).
ray_dense_limit_bytes = 4 << 30

# How update_parallel() returns the fields of several GPUs: "d2h" — every GPU copies its own fields
# into the caller's stack at once (one host thread per GPU; host bandwidth adds up over the PCIe
# links); "rccl" — the fields are first gathered onto GPU 0 over xGMI (alifmm_gather_fields, the
# counterpart of the reference's queue2 result return :3610, :3659), then copied out from there.
result_return = "d2h"


# ------------------------------------------------------------------------------------------------
def _device_map():
    """HIP devices the *_parallel methods spread sources over: all visible GPUs, or the list in
    ALIFMM_DEVICE_MAP (e.g. "0,0,0": three independent contexts, streams and field sets on GPU 0 —
    the multi-GPU sharding path exercised on a one-GPU box)."""
    m = os.environ.get("ALIFMM_DEVICE_MAP")
    if m:
        return [int(d) for d in m.split(",") if d.strip() != ""]
    return list(range(_alifmm.device_count()))


# ------------------------------------------------------------------------------------------------
# model hashing (re-upload only when the arrays change)
def _digest(*arrays):
    import xxhash

    h = xxhash.xxh3_64()
    for a in arrays:
        if a is None:
            h.update(b"None")
            continue
        a = np.ascontiguousarray(a)
        h.update(str((a.dtype.str, a.shape)).encode())
        h.update(memoryview(a).cast("B"))
    return h.hexdigest()


def _prep_model(veln, velpn, vel_map, stif_den, group_tab, phase_tab):
    veln = np.ascontiguousarray(veln, dtype=np.float64)
    velpn = np.ascontiguousarray(velpn).astype(np.int64, copy=False)
    vel_map = np.ones(veln.shape) if vel_map is None else np.ascontiguousarray(vel_map, dtype=np.float64)
    stif = None if stif_den is None else np.ascontiguousarray(stif_den).astype(np.int64, copy=False)
    gt = np.ascontiguousarray(group_tab, dtype=np.float64)
    pt = gt if phase_tab is None else np.ascontiguousarray(phase_tab, dtype=np.float64)
    return veln, velpn, vel_map, stif, gt, pt


# The resident model is keyed on a digest of the FULL content of every model argument, computed on
# every call (the reference recomputes from its arguments on every call, :1463): an in-place edit
# of any cell, or new data at a recycled address, always reaches the GPU.  xxh3 runs at ~8 GB/s
# here, ~0.15 s for the C4 model (4096^2, stiffness 0.67 GB); the class methods hash once per call
# for all their GPUs.  trust_model_identity = True opts into an identity cache (object, buffer,
# shape, strides) that skips the hash when the same arrays come back — only valid for callers that
# never edit a model array in place.
trust_model_identity = False
_identity_cache = {}


def _identity(a):
    if a is None:
        return None
    if not isinstance(a, np.ndarray):
        return ("obj", _digest(np.asarray(a)))
    return (id(a), a.__array_interface__["data"][0], a.shape, a.dtype.str, a.strides)


def _model_digest(arrays):
    if not trust_model_identity:
        return _digest(*_prep_model(*arrays))
    ident = tuple(_identity(a) for a in arrays)
    d = _identity_cache.get(ident)
    if d is None:
        d = _digest(*_prep_model(*arrays))
        if len(_identity_cache) >= 8:
            _identity_cache.pop(next(iter(_identity_cache)))
        _identity_cache[ident] = d
    return d


def _model_key(veln, velpn, vel_map, stif_den, group_tab, phase_tab, dnx, dnz, gox=0.0, goz=0.0):
    return (_model_digest((veln, velpn, vel_map, stif_den, group_tab, phase_tab)), float(dnx), float(dnz),
            float(gox), float(goz))


def _load_model(ctx, veln, velpn, vel_map, stif_den, group_tab, phase_tab, dnx, dnz, gox=0.0, goz=0.0, key=None):
    args = (veln, velpn, vel_map, stif_den, group_tab, phase_tab)
    if key is None:
        key = _model_key(*args, dnx, dnz, gox, goz)
    if ctx.model_key != key:
        veln, velpn, vel_map, stif, gt, pt = _prep_model(*args)
        ctx.set_model(veln, velpn, vel_map, stif, gt, pt, dnx, dnz, gox, goz, key=key)
    return np.shape(veln)


_module_ctx = None
_module_lock = threading.Lock()


def _mctx():
    global _module_ctx
    with _module_lock:
        if _module_ctx is None:
            _module_ctx = _alifmm.Context(0)
        return _module_ctx


# ------------------------------------------------------------------------------------------------
# Host utilities (reference :26-91, :3521-3558, :3737-3787)
def finer_grid_n(veln, scale, dtype=np.int32):
    """Nearest-neighbour refinement by odd `scale` (reference :26-56); default dtype int32 truncates."""
    veln = np.asarray(veln)
    side = (scale - 1) // 2
    nz, nx = scale * (veln.shape[0] - 1) + 1, scale * (veln.shape[1] - 1) + 1
    iz = (np.arange(nz) + side) // scale
    ix = (np.arange(nx) + side) // scale
    return veln[iz][:, ix].astype(dtype)


def finer_grid_n_2(data, scale):
    """Refinement of the (nnz, nnx, 5) stiffness/density array (reference :59-91); None -> None."""
    if data is None:
        return None
    data = np.asarray(data)
    side = (scale - 1) // 2
    nz, nx = scale * (data.shape[0] - 1) + 1, scale * (data.shape[1] - 1) + 1
    iz = (np.arange(nz) + side) // scale
    ix = (np.arange(nx) + side) // scale
    return data[iz][:, ix].astype(np.int64)


# ------------------------------------------------------------------------------------------------
# Christoffel velocities of a 2D orthotropic medium (host side).  The reference spells the same
# closed forms out four times: the module function group_vel (:3521-3558, compiled by numba) and
# the class's table generators generate_group_vel / generate_phase_vel (:4112-4206, plain
# Python).  Here one off-axis formula per velocity serves both; every value keeps the reference's
# operation order, so the tables and group_vel are bit-identical to the reference's
# (tests/test_host.py pins both against reference-generated vectors).  The one difference
# between the two callers is how sin/cos of the same argument are evaluated: numba fuses the
# pair into one libm sincos() call (which can differ from separate sin()/cos() by an ulp), plain
# Python calls them separately.
def _libm_sincos(x):
    """sin(x), cos(x) through libm's sincos() (what numba emits for a sin/cos pair)."""
    import ctypes
    import ctypes.util

    global _libm
    if _libm is None:
        _libm = ctypes.CDLL(ctypes.util.find_library("m"))
        _libm.sincos.argtypes = [ctypes.c_double, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
        _libm.sincos.restype = None
    s, c = ctypes.c_double(), ctypes.c_double()
    _libm.sincos(x, ctypes.byref(s), ctypes.byref(c))
    return s.value, c.value


_libm = None


def _math_sincos(x):
    return math.sin(x), math.cos(x)


def _group_off_axis(theta, c22, c23, c33, c44, rho, scale, sincos):
    """Group velocity at group angle theta [deg] away from the symmetry axes: the phase angle
    solves the Christoffel quadratic (root on the group angle's side of 90 deg), then
    v = scale * sqrt(lambda / rho) / cos(theta - phase)."""
    t = math.tan(math.radians(theta))
    a_ = c22 + c33 - 2 * c44
    b_ = (c23 + c44) * (t - 1 / t)
    c_ = c22 - c33
    root = math.sqrt(b_ ** 2 + a_ ** 2 - c_ ** 2)
    phase = math.atan(((-b_ - root) if theta < 90 else (-b_ + root)) / (c_ - a_)) % math.pi
    s2, c2 = sincos(2 * phase)
    lam = 0.5 * (c2 * (c22 - c44) + s2 * (c23 + c44) * t + c22 + c44)
    return scale * math.sqrt(lam / rho) / math.cos(math.radians(theta) - phase)


def _phase_off_axis(theta, c22, c23, c33, c44, rho):
    """Phase velocity at phase angle theta [deg]: the larger Christoffel eigenvalue over rho."""
    ca, sa = math.cos(math.radians(theta)), math.sin(math.radians(theta))
    a_ = ca ** 2 * c22 + sa ** 2 * c44
    b_ = ca * sa * (c23 + c44)
    c_ = ca ** 2 * c44 + sa ** 2 * c33
    return math.sqrt((a_ + c_ + math.sqrt((a_ - c_) ** 2 + 4 * b_ ** 2)) / (2 * rho))


def _velocity_table(off_axis, c22, c33, rho):
    """361-row table over 0..360 deg in 1-deg steps: on the axes sqrt(c22 / rho) (0 deg) or
    sqrt(c33 / rho) (90 deg), off-axis `off_axis(angle)`; the curve repeats every 180 deg."""
    half = [math.sqrt((c33 if a == 90 else c22) / rho) if a % 90 == 0 else off_axis(a) for a in range(180)]
    return np.array(half + half + half[:1])


def group_vel(angle, c_22, c_23, c_33, c_44, sigma, vel_scale=1):
    """Closed-form 2D orthotropic Christoffel group velocity (reference :3521-3558): within
    0.01 deg of an axis the on-axis value (c_33 near 90 deg, else c_22), else the off-axis form."""
    a90 = angle % 90
    if a90 < 0.01 or a90 > 90 - 0.01:
        return 1000 * vel_scale * math.sqrt((c_33 if abs((angle % 180) - 90) < 1 else c_22) / sigma)
    return _group_off_axis(angle, c_22, c_23, c_33, c_44, sigma, 1000 * vel_scale, _libm_sincos)


def min_max_vel(veln, velpn, vel_map, stif_den, group_vel_table):
    """Model velocity range sanity check (reference :3737-3787; note it branches on velpn[0, 0])."""
    velpn = np.asarray(velpn)
    vel_map = np.asarray(vel_map, dtype=np.float64)
    tab = np.asarray(group_vel_table, dtype=np.float64)
    gmin = tab.min(axis=0)
    gmax = tab.max(axis=0)
    if velpn[0, 0] == 0:
        sd = np.asarray(stif_den)
        s0 = sd[0, 0]
        mn = mx = group_vel(0, int(s0[0]), int(s0[1]), int(s0[2]), int(s0[3]), int(s0[4]), vel_map[0, 0])
        rows = np.concatenate([sd.reshape(-1, 5).astype(np.float64), vel_map.reshape(-1, 1)], axis=1)
        uniq = np.unique(rows, axis=0)
        for r in uniq:
            c = [int(v) for v in r[:5]]
            for a in (0, 45, 90, 135):
                v = group_vel(a, c[0], c[1], c[2], c[3], c[4], r[5])
                mn, mx = min(mn, v), max(mx, v)
        return mn, mx
    mn = mx = vel_map[0, 0] * tab[0, velpn[0, 0]]
    mn = min(mn, float(np.min(vel_map * gmin[velpn])))
    mx = max(mx, float(np.max(vel_map * gmax[velpn])))
    return mn, mx


# ------------------------------------------------------------------------------------------------
# Hot-path module functions (GPU)
def travel(scx, scz, nsts, btg, ntr, ttn, veln, velpn, vel_map, stif_den, avlist2, phase_vel, gox, goz, dnx, dnz,
           nnx, nnz):
    """Travel-time field of one source, subgrid 1 (reference :1463-2117).

    Like the reference, writes the field into `ttn` and returns it; nsts/btg/ntr are ignored
    (the GPU keeps its own node status and work lists)."""
    ctx = _mctx()
    _load_model(ctx, veln, velpn, vel_map, stif_den, avlist2, phase_vel, dnx, dnz, gox, goz)
    T = ctx.travel([scx], [scz], subgrid=1, first_slot=0)[0]
    ttn[...] = T
    return ttn


def travel_finer_grid(scx, scz, veln0, velpn0, vel_map0, stif_den0, subgrid_size, avlist2, phase_vel, gox, goz, dnx,
                      dnz):
    """Travel-time field on the subgrid_size-refined grid, divided by subgrid_size (reference :2120-2832)."""
    ctx = _mctx()
    _load_model(ctx, veln0, velpn0, vel_map0, stif_den0, avlist2, phase_vel, dnx, dnz, gox, goz)
    return ctx.travel([scx], [scz], subgrid=int(subgrid_size), first_slot=0)[0]


def find_ray(dnx, velocity_dat, source, receiver, rec_TTF, veln, velpn, vel_map, stif_den, subgrid_size):
    """Ray back-trace through the receiver's field (reference :3104-3465) -> (ray_x, ray_y, time)."""
    ctx = _mctx()
    _load_model(ctx, veln, velpn, vel_map, stif_den, velocity_dat, velocity_dat, dnx, dnx)
    sg = int(subgrid_size)
    ctx.put_field(0, sg, rec_TTF)
    times, lens, flags, rays = ctx.find_rays([0], [source[0], source[1]], [receiver[0], receiver[1]])
    if flags[0] & 1:
        print(_EARLY_MSG)
    return rays[0][0], rays[0][1], float(times[0])


def time_between_points(x1, x2, y1, y2, dnx, subgrid_size, velocity_dat, veln, velpn, vel_map, stif_den):
    """Straight-segment travel time over coarse cells (reference :2835-2989)."""
    ctx = _mctx()
    _load_model(ctx, veln, velpn, vel_map, stif_den, velocity_dat, velocity_dat, dnx, dnx)
    return float(ctx.time_between_points([x1], [x2], [y1], [y2], int(subgrid_size))[0])


def ray_time(ray_x, ray_y, dnx, subgrid_size, velocity_dat, veln, velpn, vel_map, stif_den):
    """Travel time along a ray: segment times summed in order (reference :2992-3022)."""
    ray_x = np.asarray(ray_x, dtype=np.float64)
    ray_y = np.asarray(ray_y, dtype=np.float64)
    if len(ray_x) < 2:
        return 0.0
    ctx = _mctx()
    _load_model(ctx, veln, velpn, vel_map, stif_den, velocity_dat, velocity_dat, dnx, dnx)
    seg = ctx.time_between_points(ray_x[:-1], ray_x[1:], ray_y[:-1], ray_y[1:], int(subgrid_size))
    t = 0.0
    for s in seg:
        t += float(s)
    return t


def _fine_shape(veln, subgrid_size):
    sg = int(subgrid_size)
    return (sg * (np.shape(veln)[0] - 1) + 1, sg * (np.shape(veln)[1] - 1) + 1)


def _cell(a, iz, ix):
    return np.asarray(a)[iz, ix]


def update(veln, velpn, vel_map, nsts, ttn, iz, ix, dnx, nnz, nnx, phase_vel, stif_den):
    """ALI local wavefront update of cell (iz, ix) (reference :904-1410); -1.0 if no stencil."""
    ttn = np.asarray(ttn, dtype=np.float64)
    st = None if stif_den is None else np.asarray(stif_den)[iz, ix][None, :]
    out = _mctx().local_ops(0, ttn[None], np.asarray(nsts)[None], [iz], [ix], [dnx], [dnx], [nnz], [nnx],
                            [_cell(veln, iz, ix)], [_cell(velpn, iz, ix)], [_cell(vel_map, iz, ix)], st, phase_vel)
    return float(out[0])


def fouds18_A(iz, ix, nsts, ttn, dnx, dnz, nnx, nnz, veln, velpn, vel_map, avlist2, stif_den):
    """Multi-stencil quadratic fallback of cell (iz, ix) with group velocity (reference :240-901)."""
    ttn = np.asarray(ttn, dtype=np.float64)
    st = None if stif_den is None else np.asarray(stif_den)[iz, ix][None, :]
    out = _mctx().local_ops(1, ttn[None], np.asarray(nsts)[None], [iz], [ix], [dnx], [dnz], [nnz], [nnx],
                            [_cell(veln, iz, ix)], [_cell(velpn, iz, ix)], [_cell(vel_map, iz, ix)], st, avlist2)
    return float(out[0])


# ------------------------------------------------------------------------------------------------
class ALI_FMM:
    """
    Class for calculating travel time fields and performing ray tracing through the travel time fields
    (reference :3789-4705).  GPU work goes to one context per MI355X (device 0 unless n_threads > 1
    spreads the sources of the *_parallel methods over the visible GPUs).
    """

    _STIF_TYPE_MSG = ("Stifness tensors and density array must have the type np.int64. 32bit integers will not "
                      "work correctly.")
    _STIF_UNIT_MSG = ("Warning: Stifness tensors must be in MPa, due to 64 bit integer limitations when solving the "
                      "christoffel equation")
    _VELPN_MSG = "velpn must be a numpy array of integers"

    def __init__(self, veln, velpn, vel_map, scx, scz, group_vel=None, phase_vel=None, stif_den=None, dnx=1e-3):
        # validation order and messages as the reference's (:3818-3838): stiffness first, then velpn
        self._check_stiffness(stif_den)
        if group_vel is None:  # isotropic unit curves; vel_map scales them per cell
            self.velocity_dat, self.phase_vel = self._unit_tables()
        else:
            self.velocity_dat, self.phase_vel = group_vel, phase_vel
        self._check_material_index(velpn)
        self.stif_den, self.veln, self.velpn, self.vel_map = stif_den, veln, velpn, vel_map
        self.dnx = self.dnz = dnx
        self.nnz, self.nnx = veln.shape[0], veln.shape[1]
        self.ttn = np.zeros(veln.shape)
        self.scx, self.scz = scx, scz
        self.gox = self.goz = 0
        # transducer nodes: Python round() (half-even) of the grid coordinate, kept as floats
        self.isx = np.array([float(round((x - self.gox) / self.dnx)) for x in scx])
        self.isz = np.array([float(round((z - self.goz) / self.dnz)) for z in scz])
        self.nsrc = len(scx)
        self.ntr = 0
        # the reference's CPU heap buffers (nsts, btg) have no counterpart: the GPU keeps its own
        self.maxbt = round(0.5 * self.nnx * self.nnz)
        self.nsts = self.btg = None
        self.ray_paths_x = self.ray_paths_y = self.ray_len = None
        self.rays = None  # RayStore of the last find_all_TTF_rays* call (compact layout)
        self.last_timing = None  # time split of the last find_all_TTF_rays* call
        self._ctxs = {}
        self._comms = {}  # device tuple -> _alifmm.Comm (result_return = "rccl")

    @classmethod
    def _check_stiffness(cls, stif_den):
        if stif_den is None:
            return
        first = stif_den[0, 0, 0]
        if type(first) != np.int64:
            raise TypeError(cls._STIF_TYPE_MSG)
        if first > 1e9:
            print(cls._STIF_UNIT_MSG)

    @classmethod
    def _check_material_index(cls, velpn):
        try:
            integral = np.issubdtype(velpn[0, 0], np.integer)
        except Exception:
            integral = False
        if not integral:
            raise TypeError(cls._VELPN_MSG)

    @staticmethod
    def _unit_tables():
        t = np.ones((361, 2))
        t[:, 0] = np.arange(0, 361)
        return t, t.copy()

    # ---- GPU plumbing ----
    def _ctx(self, device=0):
        """Context of logical GPU `device` (an index into _device_map())."""
        c = self._ctxs.get(device)
        if c is None:
            c = _alifmm.Context(_device_map()[device])
            self._ctxs[device] = c
        return c

    def _devices(self, n_threads):
        n = max(1, min(int(n_threads), len(_device_map())))
        return list(range(n))

    def _fields(self, veln, velpn, vel_map, stif_den, subgrid_size, idx, devices, copy_out=True, dest=None):
        """Fields of the sources `idx`, block-distributed over `devices` (one host thread per GPU).

        copy_out: each GPU's fields come back to the host; with `dest` (an (nsrc, fz, fx) float64
        C-contiguous array) straight into dest[i] (one copy, no intermediate stack), else as
        per-source arrays.  copy_out=False leaves them resident (results carry (device, slot))."""
        idx = list(idx)
        parts = sharding.deal(idx, len(devices))
        results = {}
        errors = []
        # The model digest runs in its own thread beside the GPU work (the library calls release the
        # GIL).  A GPU that holds a resident model computes on it speculatively; if the digest then
        # differs, the new model is uploaded and the fields are computed again (never returned from
        # the old model).  A GPU without a model uploads it while the digest runs.
        mtab = (veln, velpn, vel_map, stif_den, self.velocity_dat, self.phase_vel)
        box = {}

        def digest():
            try:
                box["key"] = _model_key(*mtab, self.dnx, self.dnz, self.gox, self.goz)
            except Exception as e:  # surfaced by key()
                box["err"] = e

        hasher = threading.Thread(target=digest)
        hasher.start()

        def key():
            hasher.join()
            if "err" in box:
                raise box["err"]
            return box["key"]

        def work(dev, ids):
            try:
                ctx = self._ctx(dev)
                speculative = ctx.model_key is not None and bool(ids) and ctx.shape == tuple(np.shape(veln))
                if not speculative:
                    if ctx.model_key is None:
                        ctx.set_model(*_prep_model(*mtab), self.dnx, self.dnz, self.gox, self.goz)
                        ctx._model_key = key()
                    else:
                        _load_model(ctx, *mtab, self.dnx, self.dnz, self.gox, self.goz, key=key())
                if not ids:
                    return
                x = np.array([float(self.scx[i]) for i in ids])
                z = np.array([float(self.scz[i]) for i in ids])
                into = copy_out and dest is not None  # straight into the caller's rows, streamed

                def run():
                    if into:
                        ctx.travel_into(x, z, dest, ids, subgrid=int(subgrid_size), first_slot=0)
                    else:
                        ctx.travel(x, z, subgrid=int(subgrid_size), first_slot=0, copy_out=False)

                run()
                if speculative and ctx.model_key != key():  # computed on a stale model: redo
                    _load_model(ctx, *mtab, self.dnx, self.dnz, self.gox, self.goz, key=key())
                    run()
                out = None
                if copy_out and not into:
                    out = ctx.copy_fields(0, len(ids), int(subgrid_size))[0]
                    # the device slots stay allocated for the next call (a hipMalloc / hipFree of
                    # every 134 MB field per call cost more than the copy's overlap gains); they are
                    # reused in place, reallocated only for a larger grid, freed with the context
                for k, i in enumerate(ids):
                    results[i] = (dev, k, None if out is None else out[k])
            except Exception as e:  # surfaced below
                errors.append(e)

        if len(devices) == 1:
            work(devices[0], parts[0])
        else:
            th = [threading.Thread(target=work, args=(d, p)) for d, p in zip(devices, parts)]
            for t in th:
                t.start()
            for t in th:
                t.join()
        hasher.join()
        if errors:
            raise errors[0]
        return results

    # ---- reference API ----
    def update(self, veln, velpn, vel_map=None, stif_den=None, subgrid_size=1, sources=None):
        """Travel-time fields for all (or the selected) sources (reference :3870-3936)."""
        if type(stif_den) == type(None):
            self.stif_den = np.zeros((veln.shape[0], veln.shape[1], 5))
        else:
            self.stif_den = stif_den
        self.veln = veln
        self.velpn = velpn
        self.vel_map = np.ones(veln.shape) if type(vel_map) == type(None) else vel_map
        if type(sources) == type(None):
            sources = np.ones(len(self.scx))
        idx = [i for i in range(self.nsrc) if sources[i] == 1]
        # the caller's stack is the copy's destination (one copy per field, no intermediate stack)
        travel_time_field = np.zeros((self.nsrc,) + _fine_shape(veln, subgrid_size))
        self._fields(veln, velpn, self.vel_map, stif_den, subgrid_size, idx, [0], dest=travel_time_field)
        return travel_time_field

    def update_parallel(self, veln, velpn, vel_map=None, stif_den=None, subgrid_size=1, sources=None, n_threads=2,
                        low_mem=False):
        """As update(), spread over min(n_threads, #GPUs) GPUs (reference :3938-4051).

        low_mem=True saves each field to temp_TTF_<i>.npy in the working directory and returns None."""
        if type(stif_den) == type(None):
            self.stif_den = np.zeros((veln.shape[0], veln.shape[1], 5))
        else:
            self.stif_den = stif_den
        self.veln = veln
        self.velpn = velpn
        self.vel_map = np.ones(veln.shape) if type(vel_map) == type(None) else vel_map
        if type(sources) == type(None):
            sources = np.ones(len(self.scx), dtype=int)
        idx = [i for i in range(self.nsrc) if sources[i] == 1]
        devices = self._devices(n_threads)
        if low_mem:  # one field at a time from its GPU to its file: host memory stays at one field
            res = self._fields(veln, velpn, self.vel_map, stif_den, subgrid_size, idx, devices, copy_out=False)
            try:
                for i, (dev, slot, _) in sorted(res.items()):
                    np.save("temp_TTF_" + str(i) + ".npy", self._ctx(dev).get_field(slot, int(subgrid_size)))
            finally:
                for d in devices:
                    self._ctx(d).release_fields()
            return None
        travel_time_field = np.zeros((self.nsrc,) + _fine_shape(veln, subgrid_size))
        if result_return == "rccl":
            self._fields(veln, velpn, self.vel_map, stif_den, subgrid_size, idx, devices, copy_out=False)
            self._gather_into(devices, sharding.deal(idx, len(devices)), int(subgrid_size), travel_time_field)
        else:
            self._fields(veln, velpn, self.vel_map, stif_den, subgrid_size, idx, devices, dest=travel_time_field)
        return travel_time_field

    def _gather_into(self, devices, parts, sg, dest):
        """RCCL gather of the resident fields of every device onto devices[0] (one communicator per
        device set, kept), then one copy from there into dest rows parts[r][k]."""
        key = tuple(devices)
        comm = self._comms.get(key)
        if comm is None:
            comm = _alifmm.Comm.all([self._ctx(d) for d in devices])
            self._comms[key] = comm
        counts = [len(p) for p in parts]
        off = _alifmm.gather_layout(counts)
        try:
            comm.gather(0, sg, [0] * len(devices), counts, dst_slot=0)
            root = self._ctx(devices[0])
            for r, p in enumerate(parts):
                if p:
                    root.copy_fields_into(int(off[r]), dest, p, sg)
        finally:
            for d in devices:
                self._ctx(d).release_fields()

    def update_i(self, source_i, veln, velpn, vel_map, stif_den=None, subgrid_size=1):
        """Travel-time field of one source (reference :4053-4088)."""
        if type(vel_map) == type(None):
            vel_map = np.ones(veln.shape)
        if type(stif_den) == type(None):
            stif_den = np.zeros((veln.shape[0], veln.shape[1], 5))
        res = self._fields(veln, velpn, vel_map, stif_den, subgrid_size, [source_i], [0])
        return res[source_i][2]

    def plot_phase(self, material_index=1):
        import matplotlib.pyplot as plt

        plt.polar(math.pi / 180 * self.velocity_dat[:, 0], self.phase_vel[:, material_index])
        plt.show()

    def plot_group(self, material_index=1):
        import matplotlib.pyplot as plt

        plt.polar(math.pi / 180 * self.velocity_dat[:, 0], self.velocity_dat[:, material_index])
        plt.show()

    @staticmethod
    def _plot_table(values, title):
        import matplotlib.pyplot as plt

        plt.polar(math.pi / 180 * np.arange(0, 361), values)
        plt.title(title)
        plt.show()

    def generate_group_vel(self, c_22, c_23, c_33, c_44, density, plot=True):
        """Group velocity table over 0..360 deg (reference :4112-4160)."""
        table = _velocity_table(lambda a: _group_off_axis(a, c_22, c_23, c_33, c_44, density, 1, _math_sincos),
                                c_22, c_33, density)
        if plot == True:  # noqa: E712
            self._plot_table(table, "Group Velocity")
        return table

    def generate_phase_vel(self, c_22, c_23, c_33, c_44, density, plot=True):
        """Phase velocity table over 0..360 deg (reference :4162-4206)."""
        table = _velocity_table(lambda a: _phase_off_axis(a, c_22, c_23, c_33, c_44, density), c_22, c_33, density)
        if plot == True:  # noqa: E712
            self._plot_table(table, "Phase Velocity")
        return table

    def add_materials(self, materials, keep_materials=False):
        """Table materials from stiffness/density rows [c22, c23, c33, c44, density] (reference
        :4208-4256): appended after the current columns (keep_materials=True) or replacing them
        (column 0 = angle).  The reference's column counts are kept as they are: 2D input adds
        materials.shape[1] columns when appending, and without keep_materials it sizes the tables
        and iterates by materials.shape[1] (SURVEY B-D10)."""
        single = materials.ndim == 1
        if keep_materials == True:  # noqa: E712
            width = self.velocity_dat.shape[1]
            extra = 1 if single else materials.shape[1]
            group = np.zeros((361, width + extra))
            phase = np.zeros((361, (self.phase_vel.shape[1] if single else width) + extra))
            group[:, 0:width] = self.velocity_dat
            phase[:, 0:width] = self.phase_vel
            first, count = width, 1 if single else materials.shape[0]
        else:
            width = 2 if single else materials.shape[1] + 1
            group, phase = np.zeros((361, width)), np.zeros((361, width))
            group[:, 0] = phase[:, 0] = np.arange(0, 361)
            first, count = 1, 1 if single else materials.shape[1]
        for k in range(count):
            m = materials if single else materials[k]
            group[:, first + k] = self.generate_group_vel(m[0], m[1], m[2], m[3], m[4], False)
            phase[:, first + k] = self.generate_phase_vel(m[0], m[1], m[2], m[3], m[4], False)
        if keep_materials == True:  # noqa: E712
            if single:
                print("material id of new material is " + str(first))
            else:
                print("material id's of new materials are " + str(first) + " - " + str(first + count - 1))
        self.velocity_dat = group
        self.phase_vel = phase

    def _rays(self, veln, velpn, vel_map, stif_den, subgrid_size, trans_pairs, save_rays, n_devices, include_self):
        n_trans = len(self.isx)
        max_pts = 5 * (veln.shape[0] + veln.shape[1])
        store = RayStore(n_trans, max_pts) if save_rays else None
        if type(trans_pairs) == type(None):
            trans_pairs = np.zeros((n_trans, n_trans))
            for i in range(n_trans):
                for j in range(n_trans):
                    if i < j:
                        trans_pairs[i, j] = 1
        trans_pairs = np.asarray(trans_pairs)
        rec = [j for j in range(n_trans) if np.sum(trans_pairs[:, j]) > 0]
        sg = int(subgrid_size)
        new_trans_x = sg * self.isx
        new_trans_y = sg * self.isz
        times = np.zeros((n_trans, n_trans))
        devices = self._devices(n_devices)
        # receivers block-distributed over GPUs; each ray is traced on the GPU holding its receiver field
        import time

        t0 = time.perf_counter()
        res = self._fields(veln, velpn, vel_map, stif_den, sg, rec, devices, copy_out=False)
        t_fields = time.perf_counter() - t0
        errors = []
        # where the call's time goes, per GPU (last_timing): receiver fields, the find_rays call (ray
        # and packing kernels, points left on the GPU) and its copy-out (take_rays), the host store
        per_dev = {}

        def trace(dev):
            try:
                ii, jj, slots = [], [], []
                for j, (d, slot, _) in sorted(res.items()):
                    if d != dev:
                        continue
                    sel = np.nonzero(trans_pairs[:, j] == 1)[0]
                    if not include_self:
                        sel = sel[sel != j]
                    ii.append(sel)
                    jj.append(np.full(len(sel), j))
                    slots.append(np.full(len(sel), slot))
                if not ii:
                    return
                ii, jj, slots = np.concatenate(ii), np.concatenate(jj), np.concatenate(slots)
                if len(ii) == 0:
                    return
                ctx = self._ctx(dev)
                src = np.stack([new_trans_x[ii], new_trans_y[ii]], axis=1)
                dst = np.stack([new_trans_x[jj], new_trans_y[jj]], axis=1)
                ta = time.perf_counter()
                t, lens, flags, pts = ctx.find_rays(slots, src, dst, with_points=save_rays, packed=True)
                tb = time.perf_counter()
                for _ in range(int(np.count_nonzero(flags & 1))):
                    print(_EARLY_MSG)
                times[ii, jj] = t
                if save_rays:
                    store.add(ii, jj, lens, pts if sg == 1 else pts / sg)  # (x / 1 == x: no pass over the points)
                per_dev[dev] = {"rays": int(len(ii)), "points": int(np.sum(lens, dtype=np.int64)),
                                "rays_s": tb - ta, "store_s": time.perf_counter() - tb,
                                **{k: ctx.get_option(k) for k in ("ray_kernel_ms", "ray_pack_ms", "find_rays_ms",
                                                                  "take_rays_ms")}}
            except Exception as e:
                errors.append(e)

        if len(devices) == 1:
            trace(devices[0])
        else:
            th = [threading.Thread(target=trace, args=(d,)) for d in devices]
            for t_ in th:
                t_.start()
            for t_ in th:
                t_.join()
        for d in devices:
            self._ctx(d).release_fields()
        if errors:
            raise errors[0]
        self.last_timing = {"fields_s": t_fields, "rays_total_s": time.perf_counter() - t0 - t_fields,
                            "per_gpu": per_dev}
        if save_rays:
            self.rays = store
            self.ray_len = store.ray_len
            if n_trans * n_trans * max_pts * 8 <= ray_dense_limit_bytes:
                self.ray_paths_x = store.dense(0)
                self.ray_paths_y = store.dense(1)
            else:
                self.ray_paths_x = PackedRayPaths(store, 0)
                self.ray_paths_y = PackedRayPaths(store, 1)
        return times

    def find_all_TTF_rays(self, veln, velpn, vel_map=None, subgrid_size=9, trans_pairs=None, stif_den=None,
                          save_rays=True):
        """Receiver fields + rays for all transducer pairs (reference :4258-4364); returns times (n, n)."""
        if type(vel_map) == type(None):
            vel_map = np.ones(veln.shape)
        if type(stif_den) == type(None):
            stif_den = np.zeros((veln.shape[0], veln.shape[1], 5), dtype=np.int64)
        return self._rays(veln, velpn, vel_map, stif_den, subgrid_size, trans_pairs, save_rays, 1, False)

    def find_all_TTF_rays_parallel(self, veln, velpn, vel_map=None, subgrid_size=9, trans_pairs=None, stif_den=None,
                                   n_threads=2, save_rays=True):
        """As find_all_TTF_rays over min(n_threads, #GPUs) GPUs (reference :4550-4685).

        Like the reference: ValueError for n_threads == 1, and pairs (j, j) are traced when
        trans_pairs[j, j] == 1.  Subgrid-1 fields use travel() semantics (SURVEY B-D4)."""
        if n_threads == 1:
            raise ValueError("n_threads should not equal one. Use find_all_TTF_rays for single process.")
        if type(vel_map) == type(None):
            vel_map = np.ones(veln.shape)
        if type(stif_den) == type(None):
            stif_den = np.zeros((veln.shape[0], veln.shape[1], 5), dtype=np.int64)
        return self._rays(veln, velpn, vel_map, stif_den, subgrid_size, trans_pairs, save_rays, n_threads, True)

    def ray_path(self, i, j):
        """Ray (i, j) from the last find_all_TTF_rays* call (reference :4687-4705)."""
        if self.ray_len[i, j] == 0:
            print("Ray path has not been calculated")
            return None, None
        if self.rays is not None:
            x, z = self.rays.path(i, j)
            return x.copy(), z.copy()
        ray_len = self.ray_len[i, j]
        return self.ray_paths_x[i, j, 0:ray_len], self.ray_paths_y[i, j, 0:ray_len]

    def save_ray_store(self, path):
        """Write the last call's rays in the compact layout (raystore.RayStore.save: ray_len,
        ray_off, points, max_pts in one .npz, np.load-able without pickles)."""
        if self.rays is None:
            raise ValueError("no rays: call find_all_TTF_rays* with save_rays=True first")
        self.rays.save(path)
