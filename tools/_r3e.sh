for m in 0 1 2; do timeout -k 5 30 tools/micro/residency 512 78160 384 $m || exit 1; done
timeout -k 5 30 tools/micro/residency 512 60000 384 2 || exit 1
