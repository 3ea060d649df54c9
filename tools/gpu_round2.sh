#!/bin/bash
# Round-2 measurement session: kernel-trace stats and PMC passes (each its own
# rocprofv3 run, --kernel-trace only, as MI355X_MICROARCH.md prescribes) for the
# configs given, plus the bench lines with the CPU baseline.
#   gpurun --timeout 1200 -- bash tools/gpu_round2.sh <tag> "c2 c3 c5" [bench]
set -u
TAG=$1; CFGS=${2:-"c2 c3 c5"}; BENCH=${3:-}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
python -c "import torch" 2>/dev/null
run() {  # run <name> <seconds> cmd...
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    if [ $rc -ne 0 ]; then tail -n 20 "$OUT/$name.log"; echo "!! $name rc=$rc"; exit $rc; fi
}
for c in $CFGS; do
    steps=5; [ $c = c3 ] && steps=2
    run stats_$c 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/stats_$c -o run -- python3 bench.py --config $c --steps $steps --warmup 1 --no-cpu
    find $OUT/stats_$c -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats_$c.csv \;
    grep '^{' $OUT/stats_$c.log > $OUT/bench_under_rocprof_$c.json || true
    run fetch_$c 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d $OUT/fetch_$c -o run -- python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu
    run write_$c 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d $OUT/write_$c -o run -- python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu
    f=$(find $OUT/fetch_$c -name '*counter_collection.csv'); w=$(find $OUT/write_$c -name '*counter_collection.csv')
    python tools/pmc_summary.py $f $w $OUT/pmc_traffic_$c.json > /dev/null
    if [ $c = c2 ]; then
        run sq_$c 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_BUSY_CYCLES -f csv -d $OUT/sq_$c -o run -- python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu
        python tools/pmc_table.py $(find $OUT/sq_$c -name '*counter_collection.csv') > $OUT/pmc_sq_$c.txt
        cat $OUT/pmc_sq_$c.txt
    fi
done
if [ -n "$BENCH" ]; then
    run bench_c2 400 python bench.py
    grep '^{' $OUT/bench_c2.log > $OUT/bench_c2.json
    run bench_c3 600 python bench.py --config c3 --steps 3 --warmup 1
    grep '^{' $OUT/bench_c3.log > $OUT/bench_c3.json
    run bench_c5 400 python bench.py --config c5
    grep '^{' $OUT/bench_c5.log > $OUT/bench_c5.json
    run bench_c4 400 python bench.py --config c4 --no-cpu
    grep '^{' $OUT/bench_c4.log > $OUT/bench_c4.json
fi
echo "== done $(date +%T)"
