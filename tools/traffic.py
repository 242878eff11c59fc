"""Summarise a tools/profile.sh run: kernel-trace stats -> profiles/TAG_kernel_stats.csv, and the
per-launch HBM-side traffic of one kernel (argv[3], default the band kernel fmm_band_k_kernel) from
the FETCH_SIZE / WRITE_SIZE passes, with its SQ issue profile when that pass ran ->
profiles/TAG_traffic.json (bench.py reports it as roofline.traffic when the library and the bench
workload match).

Correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts 128-B requests at 64 B on gfx950,
so read bytes = 2 x FETCH_SIZE; WRITE_SIZE is taken as is.  Both derive from the L2's memory-side
requests, i.e. Infinity-Cache hits are included: the figure is L2-miss traffic, an upper bound on
HBM bytes.  FETCH_SIZE / WRITE_SIZE are in KB.
"""
import csv
import glob
import hashlib
import json
import os
import shutil
import sys

out, tag = sys.argv[1], sys.argv[2]
kernel = sys.argv[3] if len(sys.argv) > 3 else "fmm_band_k_kernel"
repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
stats = glob.glob(os.path.join(out, "stats", "*kernel_stats.csv"))
if stats:
    shutil.copy(stats[0], os.path.join(repo, "profiles", tag + "_kernel_stats.csv"))


def per_launch(d, counter):
    vals = {}
    for f in glob.glob(os.path.join(out, d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return sum(vals.values()) / len(vals) if vals else None


def n_launch(d):
    ids = set()
    for f in glob.glob(os.path.join(out, d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"]:
                ids.add(r["Dispatch_Id"])
    return len(ids)


fetch_kb = per_launch("pmc_fetch", "FETCH_SIZE")
# issue profile (optional SQ pass): VALU wave-instructions per launch and the memory-wait share
sq = {c: per_launch("pmc_sq", c) for c in ("SQ_INSTS_VALU", "SQ_WAIT_ANY", "SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_VALU")}
write_kb = per_launch("pmc_write", "WRITE_SIZE")
lib = os.path.join(repo, "ali-fmm-and-ray-tracing_amd", "lib", "libalifmm.so")
# the workload the passes profiled (the bench line each pass printed): bench.py applies the
# figure only to a run of the same configuration
bench_config = None
for f in ("pmc_fetch.log", "pmc_write.log", "pmc_sq.log"):
    try:
        line = [l for l in open(os.path.join(out, f)) if l.startswith('{"metric"')][-1]
        cfg = json.loads(line)["config"]
        cfg.pop("total_sources", None)  # per-GPU workload: the same launch at any world size
        cfg.setdefault("cdelta", None)  # bench lines before these keys ran the defaults
        if bench_config is not None and cfg != bench_config:
            sys.exit("the PMC passes profiled different workloads: %s vs %s" % (bench_config, cfg))
        bench_config = cfg
    except (OSError, IndexError):
        pass
res = {
    "kernel": kernel,
    "launches": {d: n for d, n in (("pmc_fetch", n_launch("pmc_fetch")), ("pmc_sq", n_launch("pmc_sq"))) if n},
    "fetch_size_kb_per_launch": fetch_kb,
    "write_size_kb_per_launch": write_kb,
    "traffic_bytes_per_launch": (2 * fetch_kb + write_kb) * 1024 if fetch_kb and write_kb else None,
    "correction": "read = 2 x FETCH_SIZE (gfx950 128-B requests tallied at 64 B), write = WRITE_SIZE; "
                  "L2 memory-side requests (Infinity-Cache hits included)",
    "libalifmm_sha256": hashlib.sha256(open(lib, "rb").read()).hexdigest(),
    "bench_config": bench_config,
    "valu_insts_per_launch": sq["SQ_INSTS_VALU"],
    "sq_wait_any_frac": (sq["SQ_WAIT_ANY"] / sq["SQ_WAVE_CYCLES"]) if sq["SQ_WAIT_ANY"] and sq["SQ_WAVE_CYCLES"] else None,
    "sq_active_valu_frac": (sq["SQ_ACTIVE_INST_VALU"] / sq["SQ_WAVE_CYCLES"]) if sq["SQ_ACTIVE_INST_VALU"] and sq["SQ_WAVE_CYCLES"] else None,
    "sq_per_launch": sq,
    # the workload keys bench.py matches before it reports the figure as roofline.traffic
    "sources_per_gpu": (bench_config or {}).get("sources_per_gpu"),
    "grid": (bench_config or {}).get("grid"),
}
json.dump(res, open(os.path.join(repo, "profiles", tag + "_traffic.json"), "w"), indent=1)
print(json.dumps(res))
