"""Band width sweep (GPU box): field parity vs the reference goldens and band time per cdelta.

usage: python tools/cdelta_sweep.py 0.5 0.6 0.75 ...     (env EXACT_R: the exact-prefix radius option)
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ali-fmm-and-ray-tracing_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import _alifmm  # noqa: E402
import workloads as W  # noqa: E402

G = os.path.join(REPO, "tests", "golden")


def err(T, R, src, excl=5, step=1):
    zz, xx = np.mgrid[0:R.shape[0], 0:R.shape[1]]
    m = np.hypot(zz * step - src[1], xx * step - src[0]) > excl
    r = np.abs(T[m] - R[m]) / R[m]
    return float(r.max()), float(r.mean())


def main():
    cds = [float(a) for a in sys.argv[1:]] or [0.5]
    vt = W.default_table()
    c3 = W.c3_model()
    c4 = W.weldlike_model()
    weld = W.weld_model()
    g3 = np.load(os.path.join(G, "c3_2048.npz"))
    g4 = np.load(os.path.join(G, "c4_weldlike.npz"))
    gw = np.load(os.path.join(G, "weld_sg1.npz"))
    out = []
    for cd in cds:
        ctx = _alifmm.Context(0)
        ctx.set_option("cdelta", cd)
        if os.environ.get("EXACT_R"):
            ctx.set_option("exact_r", float(os.environ["EXACT_R"]))
        res = {"cdelta": cd}
        ctx.set_model(*c3, vt, vt, 1e-3)
        x, z = W.c3_source()
        T = ctx.travel([x], [z])[0]
        res["c3"] = err(T[::8, ::8], g3["field_dec8"], (1024, 682), step=8)
        ctx.set_model(*weld, vt, vt, 2e-4)
        scx, scz = W.weld_transducers()
        T = ctx.travel([scx[46]], [scz[46]])[0]
        res["weld_sg1"] = err(T, gw["field"], (250, 423))
        dnx = W.weldlike_dnx()
        ctx.set_model(*c4, vt, vt, dnx)
        sx, sz = W.c4_sources(128)
        k = int(g4["src_index"])
        T = ctx.travel([sx[k]], [sz[k]])[0]
        res["c4_src"] = err(T[::8, ::8], g4["field_dec8"], (16 + 32 * k, 0), step=8)
        TR = ctx.travel([dnx * 2056], [dnx * 4095])[0]
        res["c4_rec"] = err(TR[::8, ::8], g4["rec_field_dec8"], (2056, 4095), step=8)
        ctx.travel(sx, sz, copy_out=False)
        res["c4_128src_band_ms"] = ctx.last_timing()[1]
        res["steps_mean"] = float(np.mean([ctx.source_stats(i)[0][3] for i in range(128)]))
        ctx.close()
        print(json.dumps(res), flush=True)
        out.append(res)


if __name__ == "__main__":
    main()
