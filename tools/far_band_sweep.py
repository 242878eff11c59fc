"""Parity cost of a wider band far from the source, on the CPU model of the band formulation
(oracle/band_model.c, bit-equal to the device kernel up to trig ulps) against the reference's own
fields (tests/golden: C3 2048^2 source, C4 4096^2 source 64 and receiver (2056, 4095)).

python tools/far_band_sweep.py [procs]  ->  one JSON line per (case, schedule): rel max / mean error
over the decimated golden nodes more than one decimated node from the source, and main-grid steps.
"""
import json
import math
import os
import sys
from multiprocessing import Pool

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import oracle as O  # noqa: E402
import workloads as W  # noqa: E402

SCHEDULES = [(0.0, 0.0), (0.75, 256.0), (1.0, 256.0), (0.75, 512.0), (1.0, 512.0), (1.5, 512.0), (1.0, 1024.0)]


def vmax_of(velpn, vm, sd, vt):
    """The host's band-width scale (api.cpp alifmm_set_model): fastest group speed in the model."""
    v = 0.0
    cols = vt[:181, 1:].max(axis=0)
    tab = velpn != 0
    if tab.any():
        v = max(v, float(np.max(cols[velpn[tab] - 1] * vm[tab])))
    if (~tab).any():
        rows = np.unique(np.concatenate([sd[~tab].reshape(-1, 5), vm[~tab].reshape(-1, 1)], axis=1), axis=0)
        for r in rows:
            g = max(O.group_vel(0.05 * k, *[int(c) for c in r[:5]], 1.0) for k in range(3601))
            v = max(v, g * r[5])
    return v


def case(name):
    vt = W.default_table()
    if name == "c3":
        veln, velpn, vm, sd = W.c3_model()
        x, z = W.c3_source()
        return veln, velpn, vm, sd, vt, 1e-3, x, z, "c3_2048", "field_dec8"
    veln, velpn, vm, sd = W.weldlike_model()
    dnx = W.weldlike_dnx()
    if name == "c4_src":
        sx, sz = W.c4_sources(128)
        return veln, velpn, vm, sd, vt, dnx, sx[64], sz[64], "c4_weldlike", "field_dec8"
    return veln, velpn, vm, sd, vt, dnx, dnx * 2056, dnx * 4095, "c4_weldlike", "rec_field_dec8"


def run(job):
    name, (cf, rf) = job
    veln, velpn, vm, sd, vt, dnx, x, z, gname, key = case(name)
    vmax = vmax_of(velpn, vm, sd, vt)
    T, steps = O.band_travel(x, z, veln, velpn, vm, sd, vt, vt, vmax, cdelta=0.5, exact_init=True, r0=40.0,
                             exact_r=20.0, dnx=dnx, cdelta_far=cf, r_far=rf)
    ref = np.load(os.path.join(REPO, "tests", "golden", gname + ".npz"))[key]
    D = T[::8, ::8]
    zz, xx = np.mgrid[0:D.shape[0], 0:D.shape[1]]
    m = np.hypot(zz - z / dnx / 8, xx - x / dnx / 8) > 1
    r = np.abs(D[m] - ref[m]) / ref[m]
    return {"case": name, "cdelta_far": cf, "r_far": rf, "rel_max": float(r.max()), "rel_mean": float(r.mean()),
            "steps_main": int(steps[3]), "vmax": vmax}


if __name__ == "__main__":
    procs = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    jobs = [(c, s) for c in ("c4_src", "c4_rec", "c3") for s in SCHEDULES]
    with Pool(procs) as p:
        for res in p.imap_unordered(run, jobs):
            print(json.dumps(res), flush=True)
