mkdir -p gpurun_out/r3i
timeout -k 10 120 python -u tools/init_profile.py 128 > gpurun_out/r3i/init128.json || exit 1; cut -c1-400 gpurun_out/r3i/init128.json
timeout -k 10 120 python -u tools/init_profile.py 16 > gpurun_out/r3i/init16.json || exit 1
for cfg in "base:" "k8:ALIFMM_OPT_MEMBERS=8" "far1:ALIFMM_OPT_CDELTA_FAR=1.0 ALIFMM_OPT_R_FAR=1024" "far2:ALIFMM_OPT_CDELTA_FAR=1.0 ALIFMM_OPT_R_FAR=512" "sl5:ALIFMM_OPT_STRIPE_LOG=5"; do
  n=${cfg%%:*}; e=${cfg#*:}
  env $e timeout -k 10 200 python -u tools/kbench.py $n 128 16 >> gpurun_out/r3i/kbench.jsonl || exit 1
  tail -1 gpurun_out/r3i/kbench.jsonl | cut -c1-260
done
(cd /tmp && timeout -k 5 60 rocprofv3 -L > $OLDPWD/gpurun_out/r3i/counters.txt 2>&1); echo "list rc $?"
bash tools/profile.sh r3i "calib stats fetch write sq"
