# band-kernel knobs re-measured on the bricked layout: accepted-list tile sort threshold, boundary-first evaluation
mkdir -p gpurun_out/r3h2
timeout -k 10 200 python -u tools/kbench.py base 128 16 >> gpurun_out/r3h2/kbench.jsonl || exit 1
for v in sort0 sort128 sort512 bfirst; do
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 200 python -u tools/kbench.py $v 128 16 >> gpurun_out/r3h2/kbench.jsonl || exit 1
done
python3 -c "
import json
for l in open('gpurun_out/r3h2/kbench.jsonl'):
    d=json.loads(l); print(d['variant'], d['128']['band_ms'], d['16']['band_ms'], d['128']['fields'], d['16']['fields'])
"
