mkdir -p gpurun_out/r3h
(cd /tmp && timeout -k 5 60 rocprofv3 -L > $OLDPWD/gpurun_out/r3h/counters.txt 2>&1); echo "list rc $?"
bash tools/profile.sh r3h "calib stats fetch write sq"
