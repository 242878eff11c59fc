"""Band kernel: cooperative vs plain launch on C4 (16 sources): status, time and field fingerprint.
python tools/coop_check.py COOP NSRC"""
import hashlib
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ali-fmm-and-ray-tracing_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import _alifmm  # noqa: E402
import workloads as W  # noqa: E402

coop, ns = int(sys.argv[1]), int(sys.argv[2])
ctx = _alifmm.Context(0)
ctx.set_option("coop", coop)
vt = W.default_table()
ctx.set_model(*W.weldlike_model(), vt, vt, W.weldlike_dnx())
sx, sz = W.c4_sources(128)
out = {"coop": coop, "nsrc": ns}
try:
    ctx.travel(sx[:ns], sz[:ns], copy_out=False)
    out["band_ms"] = ctx.last_timing()[1]
    out["k"] = int(ctx.get_option("last_k"))
    out["steps0"] = int(ctx.source_stats(0)[0][3])
    out["fields"] = hashlib.sha256(ctx.get_field(0, 1).tobytes()).hexdigest()[:16]
except _alifmm.AlifmmError as e:
    out["error"] = str(e)
print(json.dumps(out), flush=True)
ctx.close()
