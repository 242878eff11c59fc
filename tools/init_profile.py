"""Source-init profile (GPU box): per stage ms, pops, us per pop and relax-role share, on the C4
grid (128 sources) -> one JSON line."""
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
if len(sys.argv) > 1 and sys.argv[1] == "c3":  # BASELINE C3: one interior source on the grain model
    ctx.set_model(*W.c3_model(), vt, vt, 1e-3)
    cx, cz = W.c3_source()
    sx, sz = np.array([cx]), np.array([cz])
    ns = 1
else:
    ctx.set_model(*W.weldlike_model(), vt, vt, W.weldlike_dnx())
    sx, sz = W.c4_sources(128)
    ns = int(sys.argv[1]) if len(sys.argv) > 1 else 128
ctx.travel(sx[:ns], sz[:ns], copy_out=False)
ctx.travel(sx[:ns], sz[:ns], copy_out=False)
ti, tb, _ = ctx.last_timing()
P = np.array([ctx.init_profile(i) for i in range(ns)], dtype=np.float64)
m = P.mean(axis=0)
out = {"sources": ns, "init_ms": ti, "band_ms": tb}
for k, name in enumerate(("stage1", "stage2", "stage3", "prefix")):
    out[name] = {"ms": m[k] / 1e5, "pops": m[4 + k], "us_per_pop": m[k] / 100 / max(m[4 + k], 1),
                 "relax_share": m[8 + k] / max(m[k], 1),
                 "jobs": float(np.mean(P[:, 12 + k].astype(np.int64) & 0xffffff)),
                 "passes": float(np.mean((P[:, 12 + k].astype(np.int64) >> 24) & 0xfffff)),
                 "fouds18": float(np.mean(P[:, 12 + k].astype(np.int64) >> 44))}
out["sum_ms"] = float(m[:4].sum() / 1e5)
print(json.dumps(out))
