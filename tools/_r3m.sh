mkdir -p gpurun_out/r3m
timeout -k 10 200 python -u tools/kbench.py midb 128 16 >> gpurun_out/r3m/kbench.jsonl || exit 1; tail -1 gpurun_out/r3m/kbench.jsonl | cut -c1-400
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r3m/tests.log 2>&1; rc=$?; tail -3 gpurun_out/r3m/tests.log; exit $rc
