# band kernel: claimed interior chunks evaluated during the claim phase (early) vs after it (pre)
mkdir -p gpurun_out/r3k2
timeout -k 10 200 python -u tools/kbench.py early 128 16 >> gpurun_out/r3k2/kbench.jsonl || exit 1
ALIFMM_LIB=$PWD/variants/pre/libalifmm.so timeout -k 10 200 python -u tools/kbench.py pre 128 16 >> gpurun_out/r3k2/kbench.jsonl || exit 1
timeout -k 10 200 python -u tools/kbench.py early2 128 16 >> gpurun_out/r3k2/kbench.jsonl || exit 1
python3 -c "
import json
for l in open('gpurun_out/r3k2/kbench.jsonl'):
    d=json.loads(l); print(d['variant'], d['128']['band_ms'], d['16']['band_ms'], d['128']['fields'], d['16']['fields'], {k: d['128']['us_per_step'][k] for k in ('claim','evaluate','fallback')})
"
