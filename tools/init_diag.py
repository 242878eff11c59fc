"""Init-kernel activity breakdown (diagnostic build AF_INIT_DIAG=1, GPU box): mean shader-clock
cycles per pop of the heap role (wait for relaxations, downtree, add/upd, classify) and of the relax
role (wait for a pop, verification passes, evaluation passes), C4 grid -> one JSON line.
ALIFMM_LIB=variants/idiag/libalifmm.so python tools/init_diag.py [sources]"""
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
pops = float(m[4:8].sum())
names = ["heap_wait_relax", "heap_down", "heap_addupd", "heap_classify", "relax_wait_pop", "relax_entry",
         "relax_pass", "relax_recheck"]
out = {"sources": ns, "init_ms": ti, "pops": pops, "walk_us_per_pop": ti * 1e3 / pops,
       "cycles_per_pop": {n: round(m[8 + k] / pops, 1) for k, n in enumerate(names) if n != "-"}}
# diagnostic builds put counts in the stage-tick slots: re-checks, clean entries, re-checks on one lane
out["per_pop"] = {n: round(m[k] / pops, 3) for k, n in enumerate(("rechecks", "clean_entries", "serial_rechecks"))}
print(json.dumps(out))
