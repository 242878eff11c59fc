"""Full-matrix-capture throughput (BASELINE config 5 / SURVEY C5) on one GPU (run on the GPU box).

C5: 4096^2 weld-like grid, 256 top transducers (z = 0, x = 8 + 16 k) firing into 256 bottom
receivers (z = 4095, same x): one travel-time field per receiver, then one ray per
(top source, bottom receiver) pair traced through the receiver's resident field
(`trans_pairs[i, 256 + j] = 1`, Weld_rays.py:52-55).  On 8 GPUs the receivers shard 32 per GPU
(sharding.deal) and every GPU traces its receivers' 256 x 32 rays; this tool runs the share of
`--receivers` receivers on one GPU and reports the time, so the 8-GPU FMC time is that share's
time.  Default: times only (`with_points=False`) through the C-ABI binding.  --dropin runs the same
share through the unchanged reference surface, `ALI_FMM.find_all_TTF_rays(..., save_rays=True)`
with its 512 transducers, so every ray's points are kept — in the compact RayStore, since the
reference's dense ray arrays would be 86 GB each at this size.

usage: python tools/fmc_bench.py [--receivers 32] [--sources 256] [--dropin]
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
    ap.add_argument("--receivers", type=int, default=32, help="receiver fields on this GPU (C5 on 8 GPUs: 32)")
    ap.add_argument("--sources", type=int, default=256)
    ap.add_argument("--dropin", action="store_true", help="through ALI_FMM.find_all_TTF_rays, points kept")
    ap.add_argument("--dump", default=None, help="save the ray times and lengths (npz) for bit-identity checks")
    a = ap.parse_args()
    if a.dropin:
        return dropin(a)
    n = 4096
    veln, velpn, vm, sd = W.weldlike_model(n)
    dnx = W.weldlike_dnx()
    vt = W.default_table()
    ctx = _alifmm.Context(0)
    ctx.set_model(veln, velpn, vm, sd, vt, vt, dnx)
    xs = 8 + 16 * np.arange(256)
    rx = xs[:: 256 // a.receivers][: a.receivers]
    src = np.stack([xs[: a.sources].astype(float), np.zeros(a.sources)], 1)
    # warm-up (code objects, the travel arena, and the ray point buffers at the timed call's size:
    # the context keeps them, as it does across the drop-in's calls)
    ctx.travel(dnx * rx[:2].astype(float), np.full(2, dnx * (n - 1)), first_slot=0, copy_out=False)
    nw = min(8192, a.sources * len(rx))
    ctx.find_rays([0] * nw, np.tile(src, (nw // len(src) + 1, 1))[:nw],
                  np.tile([float(rx[0]), float(n - 1)], (nw, 1)), with_points=False)
    t0 = time.perf_counter()
    ctx.travel(dnx * rx.astype(float), np.full(len(rx), dnx * (n - 1)), first_slot=0, copy_out=False)
    t1 = time.perf_counter()
    slots = np.repeat(np.arange(len(rx)), a.sources)
    s_xy = np.tile(src, (len(rx), 1))
    r_xy = np.repeat(np.stack([rx.astype(float), np.full(len(rx), float(n - 1))], 1), a.sources, axis=0)
    times, lens, flags, _ = ctx.find_rays(slots, s_xy, r_xy, with_points=False)
    t2 = time.perf_counter()
    ok = bool(np.all(np.isfinite(times)) and np.all(times > 0))
    if a.dump:
        np.savez(a.dump, times=times, lens=lens, flags=flags)
    print(json.dumps({
        "workload": "C5 share: %d bottom-receiver fields (4096^2, subgrid 1) + %d x %d rays on one GPU"
                    % (len(rx), a.sources, len(rx)),
        "fields_s": t1 - t0, "rays_s": t2 - t1, "total_s": t2 - t0,
        "fields_per_s": len(rx) / (t1 - t0), "rays_per_s": len(slots) / (t2 - t1),
        "rays": int(len(slots)), "mean_points": float(lens.mean()), "early_exit": int(np.sum(flags & 1)),
        "times_finite_positive": ok,
        "c5_on_8_gpus_s": (t2 - t0) if a.receivers == 32 and a.sources == 256 else None,
    }))
    ctx.close()


def dropin(a):
    import Anis_TTF_rays as A

    n = 4096
    veln, velpn, vm, sd = W.weldlike_model(n)
    dnx = W.weldlike_dnx()
    xs = 8 + 16 * np.arange(256)
    sx = dnx * np.concatenate([xs, xs]).astype(float)
    sz = dnx * np.concatenate([np.zeros(256), np.full(256, n - 1)])
    rx = np.arange(256)[:: 256 // a.receivers][: a.receivers]
    pairs = np.zeros((512, 512))
    pairs[np.ix_(np.arange(a.sources), 256 + rx)] = 1
    M = A.ALI_FMM(veln, velpn.astype(int), vm, sx, sz, stif_den=sd, dnx=dnx)
    warm = np.zeros((512, 512))
    warm[0:2, 256 + rx[0]] = 1
    M.find_all_TTF_rays(veln, velpn.astype(int), vm, subgrid_size=1, trans_pairs=warm, stif_den=sd)
    t0 = time.perf_counter()
    times = M.find_all_TTF_rays(veln, velpn.astype(int), vm, subgrid_size=1, trans_pairs=pairs, stif_den=sd)
    t1 = time.perf_counter()
    sel = times[np.ix_(np.arange(a.sources), 256 + rx)]
    lens = M.ray_len[np.ix_(np.arange(a.sources), 256 + rx)]
    x, z = M.ray_path(0, 256 + rx[0])
    print(json.dumps({
        "workload": "C5 share through ALI_FMM.find_all_TTF_rays (save_rays=True, compact RayStore): %d bottom-"
                    "receiver fields (4096^2, subgrid 1) + %d x %d rays with points" % (len(rx), a.sources, len(rx)),
        "total_s": t1 - t0, "rays": int(sel.size), "points": int(len(M.rays.points)),
        "ray_store_MB": M.rays.points.nbytes / 1e6, "dense_arrays_would_be_GB": 2 * 512 * 512 * 5 * 2 * n * 8 / 1e9,
        "ray_paths_type": type(M.ray_paths_x).__name__, "mean_points": float(lens.mean()),
        "times_finite_positive": bool(np.all(np.isfinite(sel)) and np.all(sel > 0)),
        "ray0_ends": [float(x[0]), float(z[0]), float(x[-1]), float(z[-1])],
    }))


if __name__ == "__main__":
    main()
