"""Synthetic inputs for the BASELINE configurations.

Shared by tests/, oracle/gen_golden.py (runs under numpy 1.26) and bench.py (numpy 2.x):
only numpy features whose results are identical across those versions are used.
The weld arrays are the reference's own data files (weld_veln/velpn/vel_map.npy), stored
losslessly in tests/golden/weld_model.npz so that nothing reads /root/reference at run time.
"""
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")

# Stiffness row of the notebook (MPa, kg/m^3; Ray tracing example.ipynb cell 34).
STIF_ROW = np.array([249000, 133000, 205000, 125000, 7850], dtype=np.int64)


def default_table():
    """ALI_FMM default velocity table (Anis_TTF_rays.py:3826-3828): column 0 angle, column 1 ones."""
    t = np.ones((361, 2))
    t[:, 0] = np.arange(0, 361)
    return t


def stif_field(nnz, nnx, row=STIF_ROW):
    s = np.empty((nnz, nnx, 5), dtype=np.int64)
    s[:, :] = row
    return s


def c1_model(n=201):
    """C1: isotropic 5790 m/s, table path (velpn=1), dnx=1e-3."""
    veln = np.zeros((n, n))
    velpn = np.ones((n, n), dtype=np.int64)
    vel_map = 5790.0 * np.ones((n, n))
    return veln, velpn, vel_map, None


def weld_model():
    """C2: the reference's weld arrays (424x500) + synthesised per-cell stiffness (weld_stif_den.npy is absent)."""
    z = np.load(os.path.join(GOLDEN, "weld_model.npz"))
    veln = z["veln"].astype(np.float64)
    velpn = z["velpn"].astype(np.int64)
    vel_map = z["vel_map"].astype(np.float64)
    return veln, velpn, vel_map, stif_field(*veln.shape)


def weld_transducers(nnz=424, nnx=500, dnx=2e-4):
    """Weld_rays.py:15-35: 31 elements on top (z=0) and bottom (z=nnz-1), pitch 15 cells."""
    n_trans, gap = 31, 15
    center = nnx / 2
    start_x = center - gap * (n_trans - 1) / 2
    end_x = center + gap * (n_trans - 1) / 2
    sx = dnx * np.arange(start_x, end_x + gap / 2, gap)
    sy = dnx * np.array([0, nnz - 1])
    scx = np.concatenate([sx, sx])
    scz = np.concatenate([np.full(n_trans, sy[0]), np.full(n_trans, sy[1])])
    return scx, scz


def voronoi_orientations(n, nseeds, seed):
    """Voronoi grain orientations: nearest seed (squared Euclid, first minimum wins)."""
    rng = np.random.default_rng(seed)
    seeds = rng.uniform(0, n, (nseeds, 2))
    orient = rng.uniform(0, 180, nseeds)
    zz = np.arange(n, dtype=np.float64)
    out = np.empty((n, n))
    for r0 in range(0, n, 64):
        r1 = min(n, r0 + 64)
        dz = (zz[r0:r1, None, None] - seeds[None, None, :, 0]) ** 2
        dx = (zz[None, :, None] - seeds[None, None, :, 1]) ** 2
        lab = np.argmin(dz + dx, axis=2)
        out[r0:r1] = orient[lab]
    return out


def c3_model(n=2048):
    """C3: n x n Voronoi grains (n//16 seeds, rng 1234), stiffness everywhere, dnx=1e-3."""
    veln = voronoi_orientations(n, n // 16, 1234)
    velpn = np.zeros((n, n), dtype=np.int64)
    vel_map = np.ones((n, n))
    return veln, velpn, vel_map, stif_field(n, n)


def c3_source(n=2048, dnx=1e-3):
    return dnx * (n // 2), dnx * (n // 3)


def weldlike_model(n=4096):
    """C4/C5: weld arrays edge-padded to n/8 x n/8 then 8x nearest (np.repeat) -> n x n."""
    veln, velpn, vel_map, _ = weld_model()
    m = n // 8

    def up(a):
        p = np.pad(a, ((0, m - a.shape[0]), (0, m - a.shape[1])), mode="edge")
        return np.repeat(np.repeat(p, 8, axis=0), 8, axis=1)

    veln = up(veln)
    velpn = up(velpn).astype(np.int64)
    vel_map = up(vel_map)
    return veln, velpn, vel_map, stif_field(n, n)


def weldlike_dnx():
    return 2e-4 / 8


def c4_sources(nsrc=128, n=4096, dnx=None, offset=0):
    """C4: nsrc sources on the top surface z=0, x = 16 + 32k (k = offset .. offset+nsrc-1, wrapped)."""
    dnx = weldlike_dnx() if dnx is None else dnx
    k = (np.arange(nsrc) + offset) % (n // 32)
    scx = dnx * (16 + 32 * k).astype(np.float64)
    scz = np.zeros(nsrc)
    return scx, scz


def c5_transducers(n=4096, per_side=256, dnx=None):
    """C5 (two-array variant, the pattern of Weld_rays.py:52-55): per_side transducers on the top
    surface (z = 0) and per_side on the bottom (z = n-1), x = 8 + 16 k; every top element i sends to
    every bottom element j: trans_pairs[i, per_side + j] = 1 -> per_side receiver fields and
    per_side^2 rays.  Returns (scx, scz, trans_pairs) in metres."""
    dnx = weldlike_dnx() if dnx is None else dnx
    x = (8 + 16 * np.arange(per_side)).astype(np.float64)
    scx = dnx * np.concatenate([x, x])
    scz = dnx * np.concatenate([np.zeros(per_side), np.full(per_side, float(n - 1))])
    tp = np.zeros((2 * per_side, 2 * per_side))
    tp[:per_side, per_side:] = 1
    return scx, scz, tp


def voronoi_small(n, seed=99, nseeds=None):
    nseeds = max(4, n // 16) if nseeds is None else nseeds
    return voronoi_orientations(n, nseeds, seed)
