# final-build check: GPU tests, smoke, bench line, then the rocprofv3 passes (stats, FETCH, WRITE, SQ)
bash tools/gpu_check.sh r3fin tests smoke bench || exit $?
bash tools/profile.sh r3fin "stats fetch write sq" || exit $?
