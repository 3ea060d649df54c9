#!/bin/bash
# Round-3 measurement session on the shipped library, one box:
#   1. phase stamps and the per-problem timeline (diagnostic build libscpqp_prof.so);
#   2. per config: rocprofv3 kernel-trace stats, then PMC passes, each its own
#      rocprofv3 run with --kernel-trace only (MI355X_MICROARCH.md): an SQ pass (waves,
#      wait, VALU / LDS instructions, LDS bank conflicts), an MFMA pass (counters picked
#      from `rocprofv3 -L` by tools/pick_counters.py), FETCH_SIZE, WRITE_SIZE;
#   3. optionally the closed-loop record of main.py's own run with the RK4 restated loop.
#   gpurun --timeout 1800 -- bash tools/gpu_measure.sh <tag> "c2 c3 c5" [prof] [closed-loop]
set -u
TAG=$1; CFGS=${2:-"c2 c3 c5"}; PROF=${3:-}; CL=${4:-}
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
if [ -n "$PROF" ]; then
    run phases 300 python tools/gpu_prof.py 4:20:1 4:20:1024 8:30:1
    cat $OUT/phases.log | grep -v amdgpu.ids
    run timeline 300 python tools/gpu_timeline.py 1024
    head -20 $OUT/timeline.log
fi
timeout -s KILL 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
MFMA=$(python tools/pick_counters.py $OUT/counters_list.txt)
echo "MFMA pass counters: $MFMA"
for c in $CFGS; do
    steps=5; [ $c = c3 ] && steps=2
    run stats_$c 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/stats_$c -o run -- python3 bench.py --config $c --steps $steps --warmup 1 --no-cpu
    find $OUT/stats_$c -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats_$c.csv \;
    grep '^{' $OUT/stats_$c.log > $OUT/bench_under_rocprof_$c.json || true
    run sq_$c 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_BUSY_CYCLES -f csv -d $OUT/sq_$c -o run -- python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu
    python tools/pmc_table.py $(find $OUT/sq_$c -name '*counter_collection.csv') > $OUT/pmc_sq_$c.txt
    cat $OUT/pmc_sq_$c.txt
    if [ -n "$MFMA" ]; then
        run mfma_$c 300 rocprofv3 --kernel-trace --pmc $MFMA -f csv -d $OUT/mfma_$c -o run -- python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu
        python tools/pmc_table.py $(find $OUT/mfma_$c -name '*counter_collection.csv') > $OUT/pmc_mfma_$c.txt
        cat $OUT/pmc_mfma_$c.txt
    fi
    run fetch_$c 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d $OUT/fetch_$c -o run -- python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu
    run write_$c 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d $OUT/write_$c -o run -- python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu
    f=$(find $OUT/fetch_$c -name '*counter_collection.csv'); w=$(find $OUT/write_$c -name '*counter_collection.csv')
    python tools/pmc_summary.py $f $w $OUT/pmc_traffic_$c.json | grep -E "raw|bytes_per_launch|scratch"
done
if [ -n "$CL" ]; then
    run closed_loop_main8 900 python -u tools/closed_loop_parity.py main8 1 50 $OUT/closed_loop_main8.json
    head -40 $OUT/closed_loop_main8.log
fi
echo "== done ($(date +%T))"
