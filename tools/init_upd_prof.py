import os, sys, numpy as np
sys.path[:0]=['ali-fmm-and-ray-tracing_amd','tests']
import _alifmm, workloads as W
ctx=_alifmm.Context(0); vt=W.default_table(); ctx.set_model(*W.weldlike_model(), vt, vt, W.weldlike_dnx())
sx,sz=W.c4_sources(128)
ctx.travel(sx[:1], sz[:1], copy_out=False)
p=ctx.init_profile(0)
jobs=sum(int(p[12+k])&0xffffffff for k in range(4))
print('jobs(src0)',jobs,'acc ticks load/sel/fin (whole launch incl. src0 only? one source):', p[8:11], 'per job us:', [p[8+i]/100/jobs for i in range(3)])
