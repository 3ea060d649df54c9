#!/bin/bash
# Round-end session on the shipped library, one box: the GPU test suite, smoke(), the bench
# line of every BASELINE configuration, the closed-loop rollout throughput, and a rocprofv3
# kernel-trace summary of the default bench (c2).
#   gpurun --timeout 1200 -- bash tools/gpu_final.sh <tag>
set -u
TAG=$1
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
bash tools/gpu_round.sh $TAG || exit $?
step() {  # step <name> <seconds> cmd...
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    if [ $rc -ne 0 ]; then tail -n 20 "$OUT/$name.log"; echo "!! $name rc=$rc"; exit $rc; fi
}
step rollout 600 python tools/bench_rollout.py 1024 5 16
grep '^{' $OUT/rollout.log > $OUT/rollout.json
cat $OUT/rollout.json
step stats_c2 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/stats_c2 -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu
find $OUT/stats_c2 -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats_c2.csv \;
head -3 $OUT/kernel_stats_c2.csv
grep '^{' $OUT/stats_c2.log > $OUT/bench_under_rocprof_c2.json
echo "== done $(date +%T)"
