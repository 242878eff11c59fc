"""CPU sweep behind the automatic band width (api.cpp band_cdelta): the band formulation's field
error against the heap oracle as a function of the model's material-interface density and cdelta.
Runs the CPU band model (oracle/band_model.c, which the device matches to 1e-9) and the heap
oracle on small models: per-cell random orientations, random-orientation blocks of g x g cells,
and Voronoi grains.  Prints one JSON line per (model, cdelta).
python tools/cdelta_auto_sweep.py [n] [cdelta ...]"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle as O  # noqa: E402
import workloads as W  # noqa: E402


def vmax_of(velpn, vm, sd, vt):
    """api.cpp set_model's vmax: the fastest group velocity over the model."""
    ang = 0.05 * np.arange(3601)
    rows = {}
    v = 0.0
    for i in np.ndindex(velpn.shape):
        if velpn[i] != 0:
            v = max(v, vt[:181, velpn[i]].max() * vm[i])
        else:
            key = tuple(sd[i])
            if key not in rows:
                rows[key] = max(O.group_vel(a, *[float(k) for k in key]) for a in ang)
            v = max(v, rows[key] * vm[i])
    return v


def jump_density(veln, velpn, vm, sd):
    """Fraction of 4-neighbour pairs whose materials differ (api.cpp material_jump)."""
    key = np.stack([veln, vm, velpn.astype(np.float64)] + [sd[..., k].astype(np.float64) for k in range(5)], -1)
    dh = np.any(key[:, 1:] != key[:, :-1], -1)
    dv = np.any(key[1:, :] != key[:-1, :], -1)
    return float((dh.sum() + dv.sum()) / (dh.size + dv.size))


def models(n):
    rng = np.random.default_rng(n)
    out = {}
    for g in (1, 2, 3, 4, 6, 8, 16):
        nb = -(-n // g)
        o = rng.uniform(0.0, 180.0, (nb, nb))
        out["blocks%d" % g] = np.repeat(np.repeat(o, g, 0), g, 1)[:n, :n]
    for ng in (n // 2, n // 8, n // 32 + 1):
        seeds = rng.uniform(0, n, (ng, 2))
        ori = rng.uniform(0, 180, ng)
        zz, xx = np.mgrid[0:n, 0:n]
        d = (zz[..., None] - seeds[:, 1]) ** 2 + (xx[..., None] - seeds[:, 0]) ** 2
        out["voronoi%d" % ng] = ori[np.argmin(d, -1)]
    return out


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 61
    cds = [float(a) for a in sys.argv[2:]] or [0.5, 0.3, 0.2, 0.1]
    dnx = 1e-3
    vt = W.default_table()
    sd = W.stif_field(n, n)
    velpn = np.zeros((n, n), dtype=np.int64)
    rng = np.random.default_rng(7)
    items = [(k, v, np.ones((n, n))) for k, v in models(n).items()]
    for g in (1, 2, 4, 8):  # velocity contrast as well (vel_map 1 .. 1.2 per block)
        nb = -(-n // g)
        vmb = np.repeat(np.repeat(1.0 + 0.2 * rng.random((nb, nb)), g, 0), g, 1)[:n, :n]
        items.append(("blocks%d_vm" % g, models(n)["blocks%d" % g], vmb))
    only = os.environ.get("SWEEP_ONLY")
    for name, veln, vm in items:
        if only and only not in name:
            continue
        vmax = vmax_of(velpn, vm, sd, vt)
        jd = jump_density(veln, velpn, vm, sd)
        for sx, sz in ((n // 4, n // 3), (n // 2, 0)):
            R = O.travel(dnx * sx, dnx * sz, veln, velpn, vm, sd, vt, vt, dnx=dnx)
            zz, xx = np.mgrid[0:n, 0:n]
            far = np.hypot(zz - sz, xx - sx) > 5
            for cd in cds:
                B, st = O.band_travel(dnx * sx, dnx * sz, veln, velpn, vm, sd, vt, vt, vmax, cdelta=cd,
                                      exact_init=True, r0=40.0, exact_r=20.0, dnx=dnx,
                                      cdelta_far=1.2 * cd, r_far=256.0)
                rel = np.abs(B - R)[far] / R[far]
                print(json.dumps({"n": n, "model": name, "jump": round(jd, 4), "src": [sx, sz], "cdelta": cd,
                                  "rel_max": float(rel.max()), "rel_mean": float(rel.mean()),
                                  "steps": int(st[3])}), flush=True)


if __name__ == "__main__":
    main()
