"""Subgrid-9 weld fields (the reference example's default, travel_finer_grid) on one GPU: the 31
bottom receiver fields of Weld_rays.py in one alifmm_travel call, split into the source-init
kernel (fmm_exact_kernel: the x9 / x3 stage heaps and the exact fine-grid prefix) and the band
kernel (GPU box).

usage: python tools/weld_split.py [--dump fields.npz]   (decimated fields, for bit-identity checks)
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ali-fmm-and-ray-tracing_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import _alifmm  # noqa: E402
import workloads as W  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dump", default=None)
    a = ap.parse_args()
    veln, velpn, vm, sd = W.weld_model()
    vt = W.default_table()
    ctx = _alifmm.Context(0)
    ctx.set_model(veln, velpn, vm, sd, vt, vt, 2e-4)
    sx, sz = W.weld_transducers()
    rx, rz = sx[31:], sz[31:]
    ctx.travel(rx[:2], rz[:2], subgrid=9, copy_out=False)  # warm-up
    for _ in range(2):
        t0 = time.perf_counter()
        ctx.travel(rx, rz, subgrid=9, copy_out=False)
        t1 = time.perf_counter()
        init_ms, band_ms, total_ms = ctx.last_timing()
        bp = ctx.band_profile(0)
        print(json.dumps({"relaxations_src0": int(bp[10]), "evaluation_passes_src0": int(bp[11])}))
        print(json.dumps({"fields": len(rx), "subgrid": 9, "wall_s": t1 - t0, "init_ms": init_ms, "band_ms": band_ms,
                          "steps_src0": ctx.source_stats(0)[0].tolist()}))
    if a.dump:
        f = ctx.travel(rx, rz, subgrid=9, copy_out=True)
        np.savez(a.dump, **{"f%d" % i: f[i][::3, ::3] for i in range(len(rx))},
                 sums=np.array([[np.sum(x), np.sum(x * x)] for x in f]))
    ctx.close()


if __name__ == "__main__":
    main()
