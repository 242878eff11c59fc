# round 3 (session 2): HEAD check + init profile + band variants (threads per member, X1 polling)
bash tools/gpu_check.sh r3o tests smoke bench stats || exit $?
timeout -k 10 300 python -u tools/init_profile.py 128 > gpurun_out/r3o/init_prof.jsonl || exit 1
timeout -k 10 300 python -u tools/init_profile.py 16 >> gpurun_out/r3o/init_prof.jsonl || exit 1
for v in base t256 t512 sl0; do
  ALIFMM_LIB=$PWD/variants/$v/libalifmm.so timeout -k 10 300 python -u tools/kbench.py $v 128 16 >> gpurun_out/r3o/kbench.jsonl || exit 1
  tail -1 gpurun_out/r3o/kbench.jsonl | cut -c1-200
done
