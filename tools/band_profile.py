"""Per-phase profile of the band kernel on the C4 workload (run on the GPU box).

usage: python tools/band_profile.py [--n 4096] [--sources 128] [--cdelta X]
Prints, averaged over sources: ms per phase, steps, mean close/accepted/evaluated list sizes.
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ali-fmm-and-ray-tracing_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import _alifmm  # noqa: E402
import workloads as W  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=4096)
ap.add_argument("--sources", type=int, default=128)
ap.add_argument("--cdelta", type=float, default=None)
ap.add_argument("--opt", action="append", default=[], help="name=value library option")
a = ap.parse_args()

veln, velpn, vm, sd = W.weldlike_model(a.n)
dnx = W.weldlike_dnx() * 4096 / a.n
vt = W.default_table()
ctx = _alifmm.Context(0)
ctx.set_option("prof", 1)
if a.cdelta:
    ctx.set_option("cdelta", a.cdelta)
for o in a.opt:
    k, v = o.split("=")
    ctx.set_option(k, float(v))
ctx.set_model(veln, velpn, vm, sd, vt, vt, dnx)
scx, scz = W.c4_sources(a.sources, a.n, dnx)
ctx.travel(scx, scz, subgrid=1, copy_out=False)  # warm
ctx.travel(scx, scz, subgrid=1, copy_out=False)
ti, tb, tt = ctx.last_timing()
P = np.array([ctx.band_profile(i) for i in range(a.sources)], dtype=np.float64)
steps = np.array([ctx.source_stats(i)[0][3] for i in range(a.sources)], dtype=np.float64)
sweeps = np.array([ctx.source_stats(i)[1] for i in range(a.sources)], dtype=np.float64)
names = ["tmin", "accept", "claim", "evaluate", "fallback+wait", "commit"]
ms = P[:, :6].mean(0) / 1e5
out = {
    "init_ms": ti, "band_ms": tb, "total_ms": tt,
    "phase_ms_mean": dict(zip(names, ms.round(2).tolist())),
    "phase_sum_ms": float(ms.sum()),
    "steps_mean": float(steps.mean()),
    "us_per_step": float(ms.sum() * 1e3 / steps.mean()),
    "mean_close": float((P[:, 6] / steps).mean()),
    "mean_accepted": float((P[:, 7] / steps).mean()),
    "mean_evaluated": float((P[:, 8] / steps).mean()),
    "max_close": float(P[:, 9].max()),
    "sweeps_per_source": float(sweeps.mean()),
    "sub_ms_mean": dict(zip(["sub0", "sub1", "sub2", "sub3"],
                            (P[:, 10:14].mean(0) / 1e5).round(2).tolist())),
}
print(json.dumps(out, indent=1))
