"""Diagnostic (ALIFMM_LIB = a -DAF_INIT_UPD_PROF build of fmm_init.hip): ticks of the relax role's
parallel pass and sequential walk per pop, one C4 source."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "ali-fmm-and-ray-tracing_amd"), os.path.join(REPO, "tests")]
import _alifmm  # noqa: E402
import workloads as W  # noqa: E402

ctx = _alifmm.Context(0)
vt = W.default_table()
ctx.set_model(*W.weldlike_model(), vt, vt, W.weldlike_dnx())
sx, sz = W.c4_sources(128)
ctx.travel(sx[:1], sz[:1], copy_out=False)
p = ctx.init_profile(0)
pops = sum(int(p[4 + k]) for k in range(4))
print("pops", pops, "jobs", int(p[10]), "parallel us/pop", p[8] / 100 / pops, "sequential us/pop", p[9] / 100 / pops,
      "total init ms", ctx.last_timing()[0])
