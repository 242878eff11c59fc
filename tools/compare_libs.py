"""Bit-identity check of two builds of the library (GPU box): travel-time fields of the same
sources through ALIFMM_LIB=<lib> (set by the caller) are saved to an npz; `compare` checks two
such files for exact equality.

usage: ALIFMM_LIB=a.so python tools/compare_libs.py run out_a.npz
       ALIFMM_LIB=b.so python tools/compare_libs.py run out_b.npz
       python tools/compare_libs.py compare out_a.npz out_b.npz
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ali-fmm-and-ray-tracing_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))


def run(path):
    import _alifmm
    import workloads as W

    vt = W.default_table()
    ctx = _alifmm.Context(0)
    out = {}
    dnx = W.weldlike_dnx()
    ctx.set_model(*W.weldlike_model(), vt, vt, dnx)
    xs = dnx * np.array([0.0, 1.0, 63.0, 64.0, 2047.0, 4095.0, 1000.0, 16.0])
    zs = dnx * np.array([0.0, 0.0, 100.0, 4095.0, 4095.0, 2000.0, 1.0, 0.0])
    f = ctx.travel(xs, zs)
    for i in range(len(xs)):
        out["c4_%d" % i] = f[i][::4, ::4].copy()
        out["c4_sum_%d" % i] = np.array([np.sum(f[i]), np.sum(f[i] * f[i])])
    del f
    veln, velpn, vm, sd = W.weld_model()
    ctx.set_model(veln, velpn, vm, sd, vt, vt, 2e-4)
    scx, scz = W.weld_transducers()
    f = ctx.travel(scx[[0, 20, 46, 61]], scz[[0, 20, 46, 61]])
    for i in range(4):
        out["weld_%d" % i] = f[i]
    ctx.close()
    np.savez(path, **out)


def compare(a, b):
    A, B = np.load(a), np.load(b)
    bad = [k for k in A.files if not np.array_equal(A[k], B[k])]
    print("identical" if not bad else "DIFFER: %s" % bad)
    return 0 if not bad else 1


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2])
    else:
        sys.exit(compare(sys.argv[2], sys.argv[3]))
