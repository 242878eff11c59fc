"""Ray kernel A/B (GPU box): NAME [receivers] -> rays/s of find_rays on C5-pattern rays (256 sources
per bottom receiver) at 4096^2, and a fingerprint of the times, lengths and points (bit-identity
across library variants; ALIFMM_LIB selects the library) -> one JSON line."""
import hashlib
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "ali-fmm-and-ray-tracing_amd"), os.path.join(REPO, "tests")]
import _alifmm  # noqa: E402
import workloads as W  # noqa: E402

name = sys.argv[1]
nrec = int(sys.argv[2]) if len(sys.argv) > 2 else 64
n = 4096
dnx = W.weldlike_dnx()
vt = W.default_table()
ctx = _alifmm.Context(0)
ctx.set_model(*W.weldlike_model(n), vt, vt, dnx)
rx = 8 + 16 * np.arange(256)[:: 256 // nrec][:nrec]
ctx.travel(dnx * rx.astype(float), np.full(len(rx), dnx * (n - 1)), first_slot=0, copy_out=False)
src = np.stack([8.0 + 16 * np.arange(256), np.zeros(256)], 1)
slots = np.repeat(np.arange(nrec), 256)
s_xy = np.tile(src, (nrec, 1))
r_xy = np.repeat(np.stack([rx.astype(float), np.full(nrec, n - 1.0)], 1), 256, axis=0)
ctx.find_rays(slots[:64], s_xy[:64], r_xy[:64], with_points=False)  # warm
best = None
for _ in range(2):
    t0 = time.perf_counter()
    times, lens, flags, _ = ctx.find_rays(slots, s_xy, r_xy, with_points=False)
    dt = time.perf_counter() - t0
    best = dt if best is None else min(best, dt)
_, _, _, pts = ctx.find_rays(slots[:512], s_xy[:512], r_xy[:512], with_points=True, packed=True)
h = hashlib.sha256(times.tobytes() + lens.tobytes() + pts.tobytes()).hexdigest()[:16]
print(json.dumps({"variant": name, "rays": len(slots), "s": round(best, 4), "rays_per_s": round(len(slots) / best),
                  "mean_points": float(lens.mean()), "fingerprint": h}), flush=True)
