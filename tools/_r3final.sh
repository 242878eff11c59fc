# final-build check: GPU tests, smoke, bench line, then the rocprofv3 passes (stats, FETCH, WRITE, SQ)
bash tools/gpu_check.sh r3f tests smoke bench || exit $?
bash tools/profile.sh r3f "stats fetch write sq" || exit $?
