# accepted-list tile sort threshold (AF_SORT_ACC) 256 / 512 / 768 / 1024, base twice
mkdir -p gpurun_out/r3h3
timeout -k 10 200 python -u tools/kbench.py base 128 16 >> gpurun_out/r3h3/kbench.jsonl || exit 1
for v in sort512 sort768 sort1024; do
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 200 python -u tools/kbench.py $v 128 16 >> gpurun_out/r3h3/kbench.jsonl || exit 1
done
timeout -k 10 200 python -u tools/kbench.py base2 128 16 >> gpurun_out/r3h3/kbench.jsonl || exit 1
python3 -c "
import json
for l in open('gpurun_out/r3h3/kbench.jsonl'):
    d=json.loads(l); print(d['variant'], d['128']['band_ms'], d['16']['band_ms'], d['128']['fields'], d['16']['fields'])
"
