# counters of the init kernel (instruction fetch / issue) and the available counter list
mkdir -p gpurun_out/r3s
export TMPDIR=/tmp
ROOT=$PWD
cd /tmp
timeout -s KILL 120 rocprofv3 --list-avail > $ROOT/gpurun_out/r3s/avail.txt 2>&1; echo "list-avail rc=$?"
grep -o "SQC_[A-Z_0-9]*\|SQ_IFETCH[A-Z_]*\|SQ_WAIT_INST[A-Z_]*\|SQ_INST_LEVEL[A-Z_]*" $ROOT/gpurun_out/r3s/avail.txt | sort -u | head -60
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_IFETCH --output-format csv -d $ROOT/gpurun_out/r3s/pmc_sq -o run -- python3 $ROOT/tools/init_profile.py 128 > $ROOT/gpurun_out/r3s/pmc_sq.log 2>&1; echo "sq pass rc=$?"
