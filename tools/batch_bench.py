"""Sources per band launch for large batches (GPU box): 256 C5 receivers (z = n-1) at 4096^2 with
the whole batch in one launch (K = 1) vs chunks of 128 (K = 2) and 64 (K = 4) -> one JSON line."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "ali-fmm-and-ray-tracing_amd"), os.path.join(REPO, "tests")]
import _alifmm  # noqa: E402
import workloads as W  # noqa: E402

ctx = _alifmm.Context(0)
vt = W.default_table()
ctx.set_model(*W.weldlike_model(), vt, vt, W.weldlike_dnx())
scx, scz, _ = W.c5_transducers()
rx, rz = scx[256:], scz[256:]
out = {}
for b in [int(a) for a in sys.argv[1:]] or [256, 128, 64]:
    ctx.set_option("batch", b)
    ctx.travel(rx, rz, copy_out=False)
    t0 = time.perf_counter()
    ctx.travel(rx, rz, copy_out=False)
    ti, tb, tt = ctx.last_timing()
    out[str(b)] = {"wall_ms": round(1e3 * (time.perf_counter() - t0), 1), "init_ms": round(ti, 1), "band_ms": round(tb, 1),
                   "total_ms": round(tt, 1), "k": int(ctx.get_option("last_k"))}
print(json.dumps(out), flush=True)
