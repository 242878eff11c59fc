"""K-member band kernel (fmm_band_k.hip): bit-identity of K = 2..16 against K = 1, timing, phase profile.

python tools/kcheck.py [quick]   (GPU box)
"""
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


def run(ctx, xs, zs, sg=1, members=0):
    ctx.set_option("members", members)
    t = time.perf_counter()
    F = ctx.travel(xs, zs, subgrid=sg)
    dt = time.perf_counter() - t
    return F, dt, ctx.get_option("last_k"), ctx.last_timing()


def main():
    quick = len(sys.argv) > 1 and sys.argv[1] == "quick"
    out = {}
    ctx = _alifmm.Context(0)
    vt = W.default_table()
    dnx = W.weldlike_dnx()
    ctx.set_model(*W.weldlike_model(), vt, vt, dnx)
    xs = dnx * np.array([0.0, 63.0, 64.0, 2047.0, 4095.0, 1000.0])
    zs = dnx * np.array([0.0, 0.0, 100.0, 4095.0, 4095.0, 2000.0])
    ref, dt, _, tm = run(ctx, xs, zs, members=1)
    out["c4_ref_s"] = dt
    for K in ([2, 16] if quick else [2, 4, 8, 16]):
        F, dt, k, tm = run(ctx, xs, zs, members=K)
        same = [bool(np.array_equal(F[i], ref[i])) for i in range(len(xs))]
        diff = [float(np.nanmax(np.abs(F[i] - ref[i]))) for i in range(len(xs))]
        out["c4_K%d" % K] = {"k": k, "same": same, "maxdiff": diff, "s": dt, "band_ms": tm[1]}
        print(json.dumps({"c4_K%d" % K: out["c4_K%d" % K]}), flush=True)
    del ref
    # weld, subgrid 1 and 3 (mode 1)
    veln, velpn, vm, sd = W.weld_model()
    ctx.set_model(veln, velpn, vm, sd, vt, vt, 2e-4)
    scx, scz = W.weld_transducers()
    for sg in (1, 3):
        ref, _, _, _ = run(ctx, scx[[0, 46]], scz[[0, 46]], sg=sg, members=1)
        for K in (2, 8):
            F, dt, k, tm = run(ctx, scx[[0, 46]], scz[[0, 46]], sg=sg, members=K)
            same = [bool(np.array_equal(F[i], ref[i])) for i in range(2)]
            out["weld_sg%d_K%d" % (sg, K)] = {"k": k, "same": same, "s": dt}
            print(json.dumps({"weld_sg%d_K%d" % (sg, K): out["weld_sg%d_K%d" % (sg, K)]}), flush=True)
    # timing: C4 128 and 16 sources, K = 1 vs auto K
    ctx.set_model(*W.weldlike_model(), vt, vt, dnx)
    sx, sz = W.c4_sources(128)
    for ns in (128, 16):
        for kern in (1, 0):  # members: 1, auto
            ctx.set_option("members", kern)
            ctx.travel(sx[:ns], sz[:ns], copy_out=False)  # warm
            t = time.perf_counter()
            ctx.travel(sx[:ns], sz[:ns], copy_out=False)
            dt = time.perf_counter() - t
            ti, tb, tt = ctx.last_timing()
            r = {"members_opt": kern, "k": ctx.get_option("last_k"), "wall_s": dt, "init_ms": ti, "band_ms": tb,
                 "steps": int(ctx.source_stats(0)[0][3]), "sweeps": int(sum(ctx.source_stats(i)[1] for i in range(ns)))}
            out["c4_time_%d_k%d" % (ns, kern)] = r
            print(json.dumps({"c4_time_%d_members%d" % (ns, kern): r}), flush=True)
    # phase profile (in-kernel wall clock, 100 MHz ticks -> us per step) of the K kernel
    for ns in (128, 16):
        ctx.set_option("members", 0)
        ctx.set_option("prof", 1)
        ctx.travel(sx[:ns], sz[:ns], copy_out=False)
        ctx.set_option("prof", 0)
        p = ctx.band_profile(0)
        st = int(ctx.source_stats(0)[0][3])
        names = ["p1_x1", "accept_rim", "claim", "evaluate", "fallback", "commit"]
        r = {n: p[i] / 100.0 / st for i, n in enumerate(names)}
        r.update({"x1_wait": p[10] / 100.0 / st, "rim_read": p[11] / 100.0 / st, "dedupe": p[12] / 100.0 / st,
                  "claim_loads": p[13] / 100.0 / st, "close_mean": p[6] / st, "acc_mean": p[7] / st,
                  "eval_mean": p[8] / st, "steps": st, "k": ctx.get_option("last_k")})
        out["prof_%d" % ns] = r
        print(json.dumps({"prof_%d" % ns: r}), flush=True)
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    json.dump(out, open(os.path.join(REPO, "gpurun_out", "kcheck.json"), "w"), indent=1)
    ctx.close()


if __name__ == "__main__":
    main()
