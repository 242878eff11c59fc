#!/bin/bash
# far-band candidates (parity sweep + shares) and the ray-tracer change A/B (C5 full + share)
set -o pipefail
mkdir -p gpurun_out/r5i
for cfg in "0.6 256" "0.6 512" "0.65 512"; do
  set -- $cfg
  ALIFMM_OPT_CDELTA_FAR=$1 ALIFMM_OPT_R_FAR=$2 timeout -k 10 300 python -u tools/cdelta_sweep.py 0.5 | sed "s/^{/{\"cdelta_far\": $1, \"r_far\": $2, /" >> gpurun_out/r5i/far_sweep.jsonl || exit 1
  ALIFMM_OPT_CDELTA_FAR=$1 ALIFMM_OPT_R_FAR=$2 timeout -k 10 300 python -u tools/kbench.py far$1_$2 128 32 16 >> gpurun_out/r5i/far_kbench.jsonl || exit 1
done
for v in rold rnew; do
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 300 python -u tools/fmc_bench.py --receivers 256 --dump gpurun_out/r5i/$v.npz > gpurun_out/r5i/$v.json 2>&1 || exit 1
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 300 python -u tools/fmc_bench.py --dump gpurun_out/r5i/${v}_share.npz > gpurun_out/r5i/${v}_share.json 2>&1 || exit 1
done
python -c "
import numpy as np
for s in ('', '_share'):
    a,b=np.load('gpurun_out/r5i/rold%s.npz'%s),np.load('gpurun_out/r5i/rnew%s.npz'%s)
    print(s or 'full', 'identical' if all(np.array_equal(a[k],b[k]) for k in a.files) else 'DIFFER')" > gpurun_out/r5i/ident.txt
bash tools/ab_run.sh "idef0 idef1" python -u tools/kbench.py x 128 16 > gpurun_out/r5i/init_defer.txt &&
bash tools/ab_run.sh "idef0 idef1" python -u tools/c3_bench.py >> gpurun_out/r5i/init_defer.txt
