"""BASELINE C3 on one GPU: the 2048^2 Voronoi-grain anisotropic grid, one source (all CUs on one
source: K members), timed per kernel, with the band kernel's roofline at SURVEY §8(d)'s 18.1
algorithmic bytes per cell-sweep, and the field checked against the reference (tests/golden/c3_2048)
-> one JSON line.  python tools/c3_bench.py"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "ali-fmm-and-ray-tracing_amd"), os.path.join(REPO, "tests")]
import _alifmm  # noqa: E402
import workloads as W  # noqa: E402

ctx = _alifmm.Context(0)
vt = W.default_table()
ctx.set_model(*W.c3_model(), vt, vt, 1e-3)
x, z = W.c3_source()
ctx.travel([x], [z], copy_out=False)
best = None
for _ in range(3):
    ctx.travel([x], [z], copy_out=False)
    ti, tb, tt = ctx.last_timing()
    best = (ti, tb, tt) if best is None or tt < best[2] else best
st = ctx.source_stats(0)
T = ctx.get_field(0, 1)
g = np.load(os.path.join(REPO, "tests", "golden", "c3_2048.npz"))
R = g["field_dec8"]
D = T[::8, ::8]
zz, xx = np.mgrid[0:D.shape[0], 0:D.shape[1]]
m = np.hypot(zz - z / 1e-3 / 8, xx - x / 1e-3 / 8) > 1
rel = np.abs(D[m] - R[m]) / R[m]
sweeps = float(st[1]) if len(st) > 1 else None
out = {"config": "C3: 2048x2048 Voronoi grains, one source", "init_ms": round(best[0], 2), "band_ms": round(best[1], 2),
       "total_ms": round(best[2], 2), "members": int(ctx.get_option("last_k")), "steps": [int(v) for v in st[0]],
       "cell_sweeps": sweeps, "field_rel_max_dec8": float(rel.max()), "field_rel_mean_dec8": float(rel.mean())}
if sweeps:
    out["band_GBps_at_18.1B_per_sweep"] = round(18.1 * sweeps / (best[1] * 1e-3) / 1e9, 1)
print(json.dumps(out))
