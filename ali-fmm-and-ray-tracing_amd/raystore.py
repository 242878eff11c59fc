"""Compact ray storage for full-matrix captures.

The reference keeps every ray of ``find_all_TTF_rays*`` in two dense float64 arrays of shape
(n_trans, n_trans, 5 * (nnz + nnx)) (``ALI_FMM.find_all_TTF_rays`` Anis_TTF_rays.py:4286-4289,
read back by ``ray_path`` :4687-4705 and by ``Weld_rays.py:64-72``).  For the 4096² full-matrix
capture (BASELINE C5: 512 transducers) each of those arrays would be 86 GB, while the rays
themselves hold ≈5 % of it.  ``RayStore`` keeps the rays ragged — one (P, 2) float64 point array
in trace order plus per-pair lengths and offsets — and ``PackedRayPaths`` presents one coordinate
of it with the dense array's read interface (shape, slicing, ``np.asarray``), so callers written
for the dense layout (``ray_paths_x[:, :, 0:max_len]``) keep working; only the pieces they index
are materialised.
"""
import threading

import numpy as np


class RayStore:
    """Rays of one find_all_TTF_rays* call.

    ray_len[i, j]  number of points of ray (i, j) (0: not traced) — the reference's ``ray_len``
    ray_off[i, j]  first row of ray (i, j) in ``points``
    points         (P, 2) float64, columns (x, z) on the model grid (already divided by subgrid)
    max_pts        the reference's per-ray capacity 5 * (nnz + nnx) (the dense arrays' last axis)
    """

    def __init__(self, n_trans, max_pts):
        self.n = int(n_trans)
        self.max_pts = int(max_pts)
        self.ray_len = np.zeros((self.n, self.n), dtype=int)
        self.ray_off = np.zeros((self.n, self.n), dtype=np.int64)
        self._chunks = []
        self._npts = 0
        self._points = None
        self._lock = threading.Lock()

    def add(self, ii, jj, lens, pts):
        """Append rays (ii[k], jj[k]) whose points are consecutive in pts (lens[k] rows each)."""
        ii = np.asarray(ii, dtype=np.int64)
        jj = np.asarray(jj, dtype=np.int64)
        lens = np.asarray(lens, dtype=np.int64)
        pts = np.ascontiguousarray(pts, dtype=np.float64).reshape(-1, 2)
        if int(lens.sum()) != len(pts):
            raise ValueError("RayStore.add: %d points for lengths summing to %d" % (len(pts), int(lens.sum())))
        starts = np.concatenate(([0], np.cumsum(lens)[:-1])) if len(lens) else lens
        with self._lock:
            self.ray_len[ii, jj] = lens
            self.ray_off[ii, jj] = self._npts + starts
            self._chunks.append(pts)
            self._npts += len(pts)
            self._points = None

    @property
    def points(self):
        with self._lock:
            if self._points is None:
                self._points = np.concatenate(self._chunks) if self._chunks else np.zeros((0, 2))
                self._chunks = [self._points]
            return self._points

    def path(self, i, j):
        """(x, z) of ray (i, j) as views into the store (empty arrays if it was not traced)."""
        n, o = int(self.ray_len[i, j]), int(self.ray_off[i, j])
        p = self.points[o:o + n]
        return p[:, 0], p[:, 1]

    def gather(self, axis, I, J, kk):
        """Dense values of coordinate `axis` at broadcast pair indices (I, J) and point indices kk
        (0-d or 1-d); points past a ray's length are 0.0 as in the reference's dense arrays."""
        lens = self.ray_len[I, J]
        offs = self.ray_off[I, J]
        kk = np.asarray(kk)
        k = kk.reshape((1,) * np.ndim(lens) + (-1,))
        valid = k < lens[..., None]
        idx = np.where(valid, offs[..., None] + k, 0)
        pts = self.points
        vals = pts[idx, axis] if len(pts) else np.zeros(idx.shape)
        out = np.where(valid, vals, 0.0)
        return out[..., 0] if kk.ndim == 0 else out

    def dense(self, axis):
        """The reference's dense (n, n, max_pts) array of one coordinate (memory permitting)."""
        out = np.zeros((self.n, self.n, self.max_pts))
        pts = self.points
        for i, j in zip(*np.nonzero(self.ray_len)):
            n, o = self.ray_len[i, j], self.ray_off[i, j]
            out[i, j, :n] = pts[o:o + n, axis]
        return out

    def save(self, path):
        """Write the store as an .npz readable with np.load (no pickles)."""
        np.savez(path, ray_len=self.ray_len, ray_off=self.ray_off, points=self.points,
                 max_pts=np.int64(self.max_pts))

    @classmethod
    def load(cls, path):
        with np.load(path, allow_pickle=False) as z:
            s = cls(z["ray_len"].shape[0], int(z["max_pts"]))
            s.ray_len[...] = z["ray_len"]
            s.ray_off[...] = z["ray_off"]
            s._points = np.ascontiguousarray(z["points"])
            s._chunks = [s._points]
            s._npts = len(s._points)
        return s


class PackedRayPaths:
    """Read-only view of one coordinate (0: x, 1: z) of a RayStore with the interface of the
    reference's dense ray_paths_x / ray_paths_y arrays (shape (n, n, max_pts), zero padded)."""

    def __init__(self, store, axis):
        self.store = store
        self.axis = int(axis)

    @property
    def shape(self):
        return (self.store.n, self.store.n, self.store.max_pts)

    ndim = 3
    dtype = np.dtype(np.float64)

    def __len__(self):
        return self.store.n

    def __getitem__(self, key):
        if not isinstance(key, tuple):
            key = (key,)
        if any(k is Ellipsis for k in key):
            e = key.index(Ellipsis)
            key = key[:e] + (slice(None),) * (4 - len(key)) + key[e + 1:]
        if len(key) > 3:
            raise IndexError("too many indices for a 3-dimensional ray array")
        key = key + (slice(None),) * (3 - len(key))
        i, j, k = key
        ar = np.arange(self.store.n)
        I, J = ar[i], ar[j]
        kk = np.arange(self.store.max_pts)[k]
        if isinstance(i, slice) or isinstance(j, slice) or np.ndim(I) == 0 or np.ndim(J) == 0:
            # outer (basic-indexing) semantics; scalar axes are dropped afterwards
            Ia, Ja = np.ix_(np.atleast_1d(I), np.atleast_1d(J))
            out = self.store.gather(self.axis, Ia, Ja, kk)
            drop = tuple(a for a, v in ((0, I), (1, J)) if np.ndim(v) == 0)
            return out.reshape(tuple(s for d, s in enumerate(out.shape) if d not in drop)) if drop else out
        Ib, Jb = np.broadcast_arrays(I, J)  # two index arrays: numpy's broadcast semantics
        return self.store.gather(self.axis, Ib, Jb, kk)

    def __array__(self, dtype=None, copy=None):
        a = self.store.dense(self.axis)
        return a if dtype is None else a.astype(dtype)

    def __repr__(self):
        return "PackedRayPaths(axis=%d, shape=%s, points=%d)" % (self.axis, self.shape, len(self.store.points))
