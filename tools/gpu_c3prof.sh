#!/bin/bash
# c3 evidence on the shipped kernel: kernel-trace stats, FETCH/WRITE passes, and
# the phase stamps (diagnostic build) of c3 alone and under load.
#   gpurun --timeout 900 -- bash tools/gpu_c3prof.sh <tag>
set -u
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
run() {
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    if [ $rc -ne 0 ]; then tail -n 20 "$OUT/$name.log"; echo "!! $name rc=$rc"; exit $rc; fi
}
run stats_c3 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/stats_c3 -o run -- python3 bench.py --config c3 --steps 2 --warmup 1 --no-cpu
find $OUT/stats_c3 -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats_c3.csv \;
run fetch_c3 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d $OUT/fetch_c3 -o run -- python3 bench.py --config c3 --steps 2 --warmup 1 --no-cpu
run write_c3 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d $OUT/write_c3 -o run -- python3 bench.py --config c3 --steps 2 --warmup 1 --no-cpu
f=$(find $OUT/fetch_c3 -name '*counter_collection.csv'); w=$(find $OUT/write_c3 -name '*counter_collection.csv')
python tools/pmc_summary.py $f $w $OUT/pmc_traffic_c3.json
run phases 300 python -u tools/gpu_prof.py 8:30:1 8:30:1024
echo "== done $(date +%T)"
