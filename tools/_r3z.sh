# ray kernel: 8 lanes per ray at subgrid 1 (8 rays per wavefront) vs 16
mkdir -p gpurun_out/r3z
timeout -k 10 300 python -u tools/ray_ab.py g16 64 >> gpurun_out/r3z/ray_ab.jsonl || exit 1
ALIFMM_LIB=$PWD/variants/g8/libalifmm.so timeout -k 10 300 python -u tools/ray_ab.py g8 64 >> gpurun_out/r3z/ray_ab.jsonl || exit 1
cat gpurun_out/r3z/ray_ab.jsonl
