"""ctypes binding of libalifmm.so (include/alifmm.h) — the MI355X hot path.

The library is built in-tree (csrc/Makefile -> lib/libalifmm.so).  There is no CPU fallback:
if the library or a GPU is missing, every entry point raises AlifmmError.
"""
import atexit
import ctypes
import os
import threading
import weakref

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ALIFMM_LIB") or os.path.join(HERE, "lib", "libalifmm.so")  # override: experiments

_d, _i, _l, _p = ctypes.c_double, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p
_lib = None
_lib_closed = False
_lock = threading.Lock()
_live = weakref.WeakSet()  # open Contexts (shutdown() destroys them)


class AlifmmError(RuntimeError):
    pass


class RayCapacityError(AlifmmError, IndexError):
    """A ray reached the reference's point capacity 5 (nnz + nnx): the reference writes past its
    ray arrays there and raises IndexError (Anis_TTF_rays.py:4287, :3440-3442)."""


# ray flags (kernels.h RayParams::flags)
RAY_EARLY_EXIT, RAY_CAPACITY, RAY_BAD_PLANE = 1, 2, 4


def check_ray_flags(flags):
    """Raise for rays the kernel stopped short of the receiver (capacity, empty search plane);
    bit 0 (the reference's "Travel time to receiver increasing" early exit) is normal output."""
    flags = np.asarray(flags)
    bad = np.nonzero(flags & RAY_CAPACITY)[0]
    if len(bad):
        raise RayCapacityError("ray %d reached the point capacity 5 (nnz + nnx)" % int(bad[0]))
    bad = np.nonzero(flags & RAY_BAD_PLANE)[0]
    if len(bad):
        raise AlifmmError("ray %d: empty plane-search candidate set" % int(bad[0]))


def _load():
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if _lib_closed:
            raise AlifmmError("libalifmm.so was unloaded by shutdown() (interpreter exit)")
        if not os.path.exists(LIB_PATH):
            raise AlifmmError("libalifmm.so not built (%s); run `make -C %s/csrc` or __graft_entry__.build()"
                              % (LIB_PATH, HERE))
        L = ctypes.CDLL(LIB_PATH)
        sig = {
            "alifmm_version": (ctypes.c_char_p, []),
            "alifmm_device_count": (_i, [_p]),
            "alifmm_ctx_create": (_i, [_i, _p]),
            "alifmm_ctx_destroy": (_i, [_p]),
            "alifmm_last_error": (ctypes.c_char_p, [_p]),
            "alifmm_set_model": (_i, [_p, _i, _i, _p, _p, _p, _p, _p, _p, _i, _d, _d, _d, _d]),
            "alifmm_set_option": (_i, [_p, ctypes.c_char_p, _d]),
            "alifmm_get_option": (_i, [_p, ctypes.c_char_p, _p]),
            "alifmm_field_shape": (_i, [_p, _i, _p, _p]),
            "alifmm_travel": (_i, [_p, _i, _i, _p, _p, _i, _p]),
            "alifmm_travel_into": (_i, [_p, _i, _i, _p, _p, _i, _p]),
            "alifmm_get_field": (_i, [_p, _i, _p]),
            "alifmm_release_fields": (_i, [_p]),
            "alifmm_copy_fields": (_i, [_p, _i, _i, _p, _i, _p]),
            "alifmm_find_rays": (_i, [_p, _i, _p, _p, _p, _p, _p, _p, _p, _l]),
            "alifmm_take_rays": (_i, [_p, _p, _l, _p]),
            "alifmm_source_stats": (_i, [_p, _i, _p, _p]),
            "alifmm_last_timing": (_i, [_p, _p, _p, _p]),
            "alifmm_band_profile": (_i, [_p, _i, _p]),
            "alifmm_band_span": (_i, [_p, _i, _p]),
            "alifmm_init_profile": (_i, [_p, _i, _p]),
            "alifmm_put_field": (_i, [_p, _i, _i, _p]),
            "alifmm_time_between_points": (_i, [_p, _i, _p, _p, _p, _p, _i, _p]),
            "alifmm_local_ops": (_i, [_p, _i, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i,
                                      _p]),
            "alifmm_fouds18_band": (_i, [_p, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i, _p]),
            "alifmm_comm_unique_id": (_i, [_p]),
            "alifmm_comm_init_rank": (_i, [_p, _i, _i, _p, _p]),
            "alifmm_comm_init_all": (_i, [_p, _i, _p]),
            "alifmm_comm_destroy": (_i, [_p]),
            "alifmm_comm_last_error": (ctypes.c_char_p, [_p]),
            "alifmm_gather_fields": (_i, [_p, _i, _i, _p, _p, _i, _p]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
        return L


def lib():
    return _load()


def _profiler_attached():
    """True under rocprofv3 (its tool library is configured through ROCPROF* / ROCP_* variables)."""
    return any(k.startswith(("ROCPROF", "ROCP_")) for k in os.environ)


def shutdown():
    """Destroy every open context and communicator at interpreter exit (atexit), while the HIP
    runtime is intact: their streams, events, pinned buffers and device memory are released in
    order instead of by the runtime's own static teardown.

    The library stays mapped (its path shows in the process maps to the end, as any loaded
    extension's), except under a profiler: rocprofv3 registers its finalisation after the
    library's HIP module destructor (__hip_module_dtor, registered with __cxa_atexit when the
    library is loaded), so that destructor would run from exit() after the tool has torn down;
    there the library is unloaded here, which runs the destructor now."""
    global _lib, _lib_closed
    live = list(_live)
    for c in [c for c in live if isinstance(c, Comm)] + [c for c in live if not isinstance(c, Comm)]:
        try:
            c.close()
        except Exception:
            pass
    _default.clear()
    if not _profiler_attached():
        return
    with _lock:
        L, _lib, _lib_closed = _lib, None, True
    if L is not None:
        import _ctypes

        _ctypes.dlclose(L._handle)


atexit.register(shutdown)


def device_count():
    n = ctypes.c_int(0)
    lib().alifmm_device_count(ctypes.byref(n))
    return n.value


def _c64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def _ci64(a):
    return np.ascontiguousarray(a, dtype=np.int64)


def _ci32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


KEEP_RAYS = -1  # ALIFMM_KEEP_RAYS (include/alifmm.h)


def _ptr(a):
    return None if a is None else a.ctypes.data


class Context:
    """One GPU (HIP device index).  Holds the resident model and travel-time fields."""

    def __init__(self, device=0, cdelta=None, r0=None, batch=None):
        L = lib()
        h = ctypes.c_void_p()
        rc = L.alifmm_ctx_create(int(device), ctypes.byref(h))
        if rc != 0 or not h.value:
            raise AlifmmError("alifmm_ctx_create(device=%d) failed (rc=%d): no usable MI355X/HIP device"
                              % (device, rc))
        self._h = h
        self.device = device
        _live.add(self)
        self._model_key = None
        self.shape = None
        for k, v in (("cdelta", cdelta), ("r0", r0), ("batch", batch)):
            if v is not None:
                self.set_option(k, v)
        # experiments (tools/*.sh): ALIFMM_OPT_<NAME>=value sets alifmm_set_option(name, value) on
        # every context (README "Options"); a bad name or value is reported and ignored, never fatal
        for k, v in os.environ.items():
            if k.startswith("ALIFMM_OPT_"):
                try:
                    self.set_option(k[len("ALIFMM_OPT_"):].lower(), float(v))
                except (ValueError, AlifmmError) as e:
                    import warnings

                    warnings.warn("ignoring %s=%r: %s" % (k, v, e))

    def _chk(self, rc, what):
        if rc != 0:
            msg = lib().alifmm_last_error(self._h)
            raise AlifmmError("%s failed (rc=%d): %s" % (what, rc, msg.decode() if msg else ""))

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value and _lib is not None:
            _lib.alifmm_ctx_destroy(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def model_key(self):
        """Key of the resident model (set_model(key=...)), None when unknown."""
        return self._model_key

    def set_option(self, name, value):
        self._chk(lib().alifmm_set_option(self._h, name.encode(), float(value)), "set_option(%s)" % name)

    def get_option(self, name):
        v = ctypes.c_double(0)
        self._chk(lib().alifmm_get_option(self._h, name.encode(), ctypes.byref(v)), "get_option(%s)" % name)
        return v.value

    def set_model(self, veln, velpn, vel_map, stif_den, group_tab, phase_tab, dnx, dnz=None, gox=0.0, goz=0.0,
                  key=None):
        """Upload the model unless `key` equals the key of the resident model."""
        if key is not None and key == self._model_key:
            return
        veln = _c64(veln)
        nnz, nnx = veln.shape
        velpn = _ci64(velpn)
        vel_map = _c64(vel_map)
        stif = None if stif_den is None else _ci64(stif_den)
        gt = _c64(group_tab)
        pt = _c64(phase_tab if phase_tab is not None else group_tab)
        if velpn.shape != veln.shape or vel_map.shape != veln.shape:
            raise ValueError("veln, velpn and vel_map must have the same shape")
        if stif is not None and stif.shape != (nnz, nnx, 5):
            raise ValueError("stif_den must have shape (nnz, nnx, 5)")
        if gt.ndim != 2 or gt.shape[0] != 361 or pt.shape != gt.shape:
            raise ValueError("velocity tables must have shape (361, ncol)")
        dnz = dnx if dnz is None else dnz
        # forget the resident key first: if the upload fails, the next call must upload again
        self._model_key = None
        self._chk(lib().alifmm_set_model(self._h, nnz, nnx, _ptr(veln), _ptr(velpn), _ptr(vel_map), _ptr(stif),
                                         _ptr(gt), _ptr(pt), gt.shape[1], float(dnx), float(dnz), float(gox),
                                         float(goz)), "set_model")
        self._model_key = key
        self.shape = (nnz, nnx)

    def field_shape(self, subgrid):
        a, b = ctypes.c_int(0), ctypes.c_int(0)
        self._chk(lib().alifmm_field_shape(self._h, int(subgrid), ctypes.byref(a), ctypes.byref(b)), "field_shape")
        return a.value, b.value

    def travel(self, scx, scz, subgrid=1, first_slot=0, copy_out=True):
        """Travel-time fields for sources (scx, scz) [m]; resident in slots first_slot.. ."""
        scx = _c64(np.atleast_1d(scx))
        scz = _c64(np.atleast_1d(scz))
        fz, fx = self.field_shape(subgrid)
        out = np.empty((len(scx), fz, fx)) if copy_out else None
        self._chk(lib().alifmm_travel(self._h, int(subgrid), len(scx), _ptr(scx), _ptr(scz), int(first_slot),
                                      _ptr(out)), "travel")
        return out

    def travel_into(self, scx, scz, dest, rows, subgrid=1, first_slot=0):
        """travel() with field i written to dest[rows[i]] of a caller-visible C-contiguous float64
        (n, fnz, fnx) stack (alifmm_travel_into: at subgrid 1 the fields stream out of the band
        kernel tile by tile while it runs).  The fields also stay resident in slots first_slot.. ."""
        scx = _c64(np.atleast_1d(scx))
        scz = _c64(np.atleast_1d(scz))
        if not (isinstance(dest, np.ndarray) and dest.dtype == np.float64 and dest.flags.c_contiguous
                and dest.ndim == 3):
            raise ValueError("dest must be a C-contiguous float64 (n, fnz, fnx) array")
        if dest.shape[1:] != self.field_shape(subgrid):
            raise ValueError("dest fields %s, travel fields %s" % (dest.shape[1:], self.field_shape(subgrid)))
        rows = [int(r) for r in rows]
        if len(rows) != len(scx):
            raise ValueError("one dest row per source")
        if rows and (min(rows) < 0 or max(rows) >= dest.shape[0]):
            raise IndexError("travel_into: row outside dest")
        base, step = dest.ctypes.data, dest[0].nbytes if dest.shape[0] else 0
        ptrs = (ctypes.c_void_p * max(1, len(rows)))(*[base + r * step for r in rows])
        self._chk(lib().alifmm_travel_into(self._h, int(subgrid), len(scx), _ptr(scx), _ptr(scz), int(first_slot),
                                           ptrs), "travel_into")

    def get_field(self, slot, subgrid):
        fz, fx = self.field_shape(subgrid)
        out = np.empty((fz, fx))
        self._chk(lib().alifmm_get_field(self._h, int(slot), _ptr(out)), "get_field")
        return out

    def put_field(self, slot, subgrid, data):
        data = _c64(data)
        if data.shape != self.field_shape(subgrid):
            raise ValueError("field shape %s does not match subgrid %d" % (data.shape, subgrid))
        self._chk(lib().alifmm_put_field(self._h, int(slot), int(subgrid), _ptr(data)), "put_field")

    def copy_fields(self, first_slot, n, subgrid, out=None, dst_kind=0):
        """Resident fields of slots first_slot .. first_slot+n-1 as one (n, fnz, fnx) host array
        (alifmm_copy_fields: pageable destinations go through the pinned staging ring).
        Returns (array, GB/s)."""
        fz, fx = self.field_shape(subgrid)
        if out is None:
            out = np.empty((n, fz, fx))
        g = ctypes.c_double(0)
        self._chk(lib().alifmm_copy_fields(self._h, int(first_slot), int(n), _ptr(out), int(dst_kind), ctypes.byref(g)),
                  "copy_fields")
        return out, g.value

    def copy_fields_into(self, first_slot, dest, rows, subgrid, dst_kind=0):
        """Resident slots first_slot, first_slot+1, ... straight into dest[rows[0]], dest[rows[1]], ...
        of a caller-visible C-contiguous float64 (n, fnz, fnx) stack: one copy per field, no
        intermediate array (runs of consecutive rows go in one alifmm_copy_fields call).
        dst_kind 0: through the pinned staging ring; 3: DMA straight into dest (registered for the
        copy).  Returns the bytes copied."""
        if not (isinstance(dest, np.ndarray) and dest.dtype == np.float64 and dest.flags.c_contiguous
                and dest.ndim == 3):
            raise ValueError("dest must be a C-contiguous float64 (n, fnz, fnx) array")
        if dest.shape[1:] != self.field_shape(subgrid):
            raise ValueError("dest fields %s, resident fields %s" % (dest.shape[1:], self.field_shape(subgrid)))
        rows = [int(r) for r in rows]
        if rows and (min(rows) < 0 or max(rows) >= dest.shape[0]):
            raise IndexError("copy_fields_into: row outside dest")
        g = ctypes.c_double(0)
        k = 0
        while k < len(rows):
            e = k + 1
            while e < len(rows) and rows[e] == rows[e - 1] + 1:
                e += 1
            self._chk(lib().alifmm_copy_fields(self._h, int(first_slot + k), e - k, dest[rows[k]].ctypes.data,
                                               int(dst_kind), ctypes.byref(g)), "copy_fields")
            k = e
        return len(rows) * dest[0].nbytes

    def copy_fields_to_device(self, first_slot, n, dev_ptr):
        """Copy resident fields into device memory of this GPU at dev_ptr (e.g. a torch tensor's
        data_ptr(), for an RCCL gather).  Returns GB/s."""
        g = ctypes.c_double(0)
        self._chk(lib().alifmm_copy_fields(self._h, int(first_slot), int(n), ctypes.c_void_p(int(dev_ptr)), 2,
                                           ctypes.byref(g)), "copy_fields")
        return g.value

    def release_fields(self):
        self._chk(lib().alifmm_release_fields(self._h), "release_fields")

    def find_rays(self, slots, src_xy, rec_xy, with_points=True, packed=False, check=True):
        """Rays through resident receiver fields.

        Returns (times, lens, flags, rays): rays is a list of (x, z) arrays per ray, or with
        packed=True one (sum(lens), 2) array of all points in ray order (ray k starts at row
        sum(lens[:k])) — no per-ray copies, and the host buffer is sized exactly (the points wait
        in the context between alifmm_find_rays and alifmm_take_rays).  check: raise
        (check_ray_flags) for a ray cut short at the point capacity or on an empty search plane."""
        slots = _ci32(slots)
        n = len(slots)
        src_xy = _c64(src_xy).reshape(n, 2)
        rec_xy = _c64(rec_xy).reshape(n, 2)
        times = np.zeros(n)
        lens = np.zeros(n, dtype=np.int32)
        flags = np.zeros(n, dtype=np.int32)
        keep = with_points and n > 0
        self._chk(lib().alifmm_find_rays(self._h, n, _ptr(slots), _ptr(src_xy), _ptr(rec_xy), _ptr(times),
                                         _ptr(lens), _ptr(flags), None, KEEP_RAYS if keep else 0), "find_rays")
        if check:
            check_ray_flags(flags)
        if not with_points:
            return times, lens, flags, None
        npts = int(lens.sum(dtype=np.int64))
        pts = np.empty((npts, 2))
        if keep:
            got = ctypes.c_int64(0)
            self._chk(lib().alifmm_take_rays(self._h, _ptr(pts), npts, ctypes.byref(got)), "take_rays")
            if got.value != npts:
                raise AlifmmError("take_rays: %d points kept, %d expected" % (got.value, npts))
        if packed:
            return times, lens, flags, pts
        rays = []
        off = 0
        for k in range(n):
            p = pts[off:off + lens[k]]
            rays.append((p[:, 0].copy(), p[:, 1].copy()))
            off += lens[k]
        return times, lens, flags, rays

    def source_stats(self, slot):
        steps = np.zeros(4, dtype=np.int64)
        sw = ctypes.c_int64(0)
        self._chk(lib().alifmm_source_stats(self._h, int(slot), _ptr(steps), ctypes.byref(sw)), "source_stats")
        return steps, sw.value

    def band_profile(self, slot):
        out = np.zeros(14, dtype=np.int64)
        self._chk(lib().alifmm_band_profile(self._h, int(slot), _ptr(out)), "band_profile")
        return out

    def band_span(self, slot):
        """(start, end) wall clock [100 MHz ticks] of the band kernel's member 0 for a slot's source."""
        out = np.zeros(2, dtype=np.int64)
        self._chk(lib().alifmm_band_span(self._h, int(slot), _ptr(out)), "band_span")
        return int(out[0]), int(out[1])

    def init_profile(self, i):
        """Source-init profile of source i of the last chunk: ticks (100 MHz) of stage 1/2/3 and the
        exact prefix, their pops, relax-role busy ticks, relaxations | fallbacks << 32
        (alifmm_init_profile)."""
        out = np.zeros(16, dtype=np.int64)
        self._chk(lib().alifmm_init_profile(self._h, int(i), _ptr(out)), "init_profile")
        return out

    def last_timing(self):
        a, b, c = ctypes.c_double(0), ctypes.c_double(0), ctypes.c_double(0)
        self._chk(lib().alifmm_last_timing(self._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)),
                  "last_timing")
        return a.value, b.value, c.value

    def time_between_points(self, x1, x2, y1, y2, subgrid):
        x1, x2, y1, y2 = (_c64(np.atleast_1d(v)) for v in (x1, x2, y1, y2))
        out = np.empty(len(x1))
        self._chk(lib().alifmm_time_between_points(self._h, len(x1), _ptr(x1), _ptr(x2), _ptr(y1), _ptr(y2),
                                                   int(subgrid), _ptr(out)), "time_between_points")
        return out

    def local_ops(self, op, ttn, nsts, iz, ix, dnx, dnz, nnz_arg, nnx_arg, cveln, cvelpn, cvm, cstif, tab):
        """Batched update() (op 0) / fouds18_A() (op 1) on (n, pz, px) patches."""
        ttn = _c64(ttn)
        n, pz, px = ttn.shape
        nsts = _ci32(nsts)
        out = np.empty(n)
        tab = _c64(tab)
        cst = None if cstif is None else _ci64(cstif).reshape(n, 5)
        args = [_ci32(iz), _ci32(ix), _c64(dnx), _c64(dnz), _ci32(nnz_arg), _ci32(nnx_arg), _c64(cveln),
                _ci64(cvelpn), _c64(cvm)]
        self._chk(lib().alifmm_local_ops(self._h, int(op), n, pz, px, _ptr(ttn), _ptr(nsts), *[_ptr(a) for a in args],
                                         _ptr(cst), _ptr(tab), tab.shape[1], _ptr(out)), "local_ops")
        return out

    def fouds18_band(self, ttn, nsts, iz, ix, dnx, dnz, nnz_arg, nnx_arg, mz, mx, quant=0):
        """fouds18_A() as the band kernel evaluates it: material of resident-model cell (mz, mx)
        through the per-material record and precomputed slownesses (alifmm_fouds18_band)."""
        ttn = _c64(ttn)
        n, pz, px = ttn.shape
        out = np.empty(n)
        nsts = _ci32(nsts)
        args = [_ci32(iz), _ci32(ix), _c64(dnx), _c64(dnz), _ci32(nnz_arg), _ci32(nnx_arg), _ci32(mz), _ci32(mx)]
        self._chk(lib().alifmm_fouds18_band(self._h, n, pz, px, _ptr(ttn), _ptr(nsts), *[_ptr(a) for a in args],
                                            int(quant), _ptr(out)), "fouds18_band")
        return out


class Comm:
    """RCCL communicator over contexts on distinct GPUs (include/alifmm.h alifmm_comm_*): gathers
    resident fields onto one GPU over xGMI.  Comm.all(ctxs): one process driving every context;
    Comm.rank(ctx, nranks, rank, uid): one process per GPU, uid = Comm.unique_id() made by one rank
    and shared by the caller (e.g. torch.distributed.broadcast_object_list)."""

    def __init__(self, handle, ctxs):
        self._h = handle
        self.ctxs = list(ctxs)
        _live.add(self)

    @staticmethod
    def unique_id():
        buf = ctypes.create_string_buffer(128)
        if lib().alifmm_comm_unique_id(buf) != 0:
            raise AlifmmError("alifmm_comm_unique_id failed (RCCL unavailable)")
        return buf.raw

    @classmethod
    def all(cls, ctxs):
        arr = (ctypes.c_void_p * len(ctxs))(*[c._h.value for c in ctxs])
        h = ctypes.c_void_p()
        ctxs[0]._chk(lib().alifmm_comm_init_all(arr, len(ctxs), ctypes.byref(h)), "comm_init_all")
        return cls(h, ctxs)

    @classmethod
    def rank(cls, ctx, nranks, rank, uid):
        if len(uid) != 128:
            raise ValueError("RCCL unique id must be 128 bytes")
        h = ctypes.c_void_p()
        ctx._chk(lib().alifmm_comm_init_rank(ctx._h, int(nranks), int(rank), ctypes.create_string_buffer(uid, 128),
                                             ctypes.byref(h)), "comm_init_rank")
        return cls(h, [ctx])

    def gather(self, root, subgrid, first_slot, count, dst_slot=0):
        """Rank r's slots first_slot[r] .. +count[r]-1 -> the root's slots dst_slot + sum(count[:r]) + i.
        Every rank passes the same lists.  Returns the wall time [ms]."""
        fs = np.ascontiguousarray(first_slot, dtype=np.int32)
        cn = np.ascontiguousarray(count, dtype=np.int32)
        ms = ctypes.c_double(0)
        rc = lib().alifmm_gather_fields(self._h, int(root), int(subgrid), _ptr(fs), _ptr(cn), int(dst_slot),
                                        ctypes.byref(ms))
        if rc != 0:
            msg = lib().alifmm_comm_last_error(self._h)
            raise AlifmmError("gather_fields failed (rc=%d): %s" % (rc, msg.decode() if msg else ""))
        return ms.value

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value and _lib is not None:
            _lib.alifmm_comm_destroy(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def gather_layout(counts):
    """Root slot offset of every rank's first field in alifmm_gather_fields (rank order)."""
    return np.concatenate(([0], np.cumsum(np.asarray(counts, dtype=np.int64))))[:-1]


_default = {}


def default_context(device=0):
    """Process-wide context per device (created on first use)."""
    with _lock:
        ctx = _default.get(device)
    if ctx is None:
        ctx = Context(device)
        with _lock:
            _default[device] = ctx
    return ctx
