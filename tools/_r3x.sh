# launch chunking (>= 2 members per source): C5 receivers, the C5 capture test, all GPU tests
mkdir -p gpurun_out/r3x
timeout -k 10 400 python -u tools/batch_bench.py 256 > gpurun_out/r3x/batch.json || exit 1
cat gpurun_out/r3x/batch.json
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3x/tests.log 2>&1; rc=$?; tail -3 gpurun_out/r3x/tests.log
cat gpurun_out/c5_capture.json | head -8
exit $rc
