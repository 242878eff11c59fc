"""Time alifmm_set_model on the C4 model (4096^2 weld-like, stiffness field) — the one-time model
upload of a first call (host checks, distinct stiffness rows and material records, bricks, H2D)."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "ali-fmm-and-ray-tracing_amd"), os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402

import _alifmm  # noqa: E402
import workloads as W  # noqa: E402

t0 = time.perf_counter()
ctx = _alifmm.Context(0)
t_ctx = time.perf_counter() - t0
vt = W.default_table()
veln, velpn, vm, stif = W.weldlike_model(4096)
veln = np.ascontiguousarray(veln, dtype=np.float64)
velpn = np.ascontiguousarray(velpn, dtype=np.int64)
vm = np.ascontiguousarray(vm, dtype=np.float64)
stif = np.ascontiguousarray(stif, dtype=np.int64)
ts = []
for _ in range(3):
    t0 = time.perf_counter()
    ctx.set_model(veln, velpn, vm, stif, vt, vt, W.weldlike_dnx())
    ts.append(time.perf_counter() - t0)
print(json.dumps({"context_s": t_ctx, "set_model_s": ts, "cells": int(veln.size)}))
