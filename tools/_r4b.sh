set -o pipefail
mkdir -p gpurun_out/r4b
timeout -k 10 300 python -u bench.py --no-cpu --steps 3 > gpurun_out/r4b/bench.log 2>&1 && grep '"metric"' gpurun_out/r4b/bench.log | cut -c1-200 &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_c5.py tests/test_gpu_host_paths.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4b/tests.log 2>&1 && tail -2 gpurun_out/r4b/tests.log &&
PROG="python3 tools/c3_bench.py" timeout -k 10 600 bash tools/profile.sh r4c3 "stats fetch write sq" &&
PROG="python3 tools/fmc_bench.py" timeout -k 10 600 bash tools/profile.sh r4rays "stats sq" &&
PROG="python3 tools/weld_split.py" timeout -k 10 600 bash tools/profile.sh r4exact "stats sq"
