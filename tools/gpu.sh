#!/bin/bash
# One GPU box session (gpurun), as a chain of steps that stops at the first failure:
#   gpurun --timeout 1500 -- bash tools/gpu.sh <tag> <step> [<step> ...]
# Steps (each argument one step; values after ':' separated by ','):
#   tests[:k-expr]        GPU test suite (one pytest process), optionally -k filtered
#   checktests[:k-expr]   the GPU suite on the reduction-check build (SCPQP_TEST_LIB, build.py --check)
#   reducecheck:<lib>     reduction-buffer counters of a check build over the configs (records a FAIL
#                         without stopping the chain; a crash still stops it)
#   smoke                 __graft_entry__.smoke()
#   bench:<cfg>[,steps]   bench.py line of one BASELINE configuration (c2 with the CPU leg)
#   ab:<cfgs>:<libs>[:reps]  A/B of library builds, e.g. ab:c2/10,c4/3:scpqp/libscpqp.so,/tmp/x.so:2
#                         (bench.py --no-cpu, alternating; VAR=value@lib.so sets an env var)
#   phases:[VAR=v@]<lib>[:cfgs]  phase stamps of a -DSCPQP_PROF build (tools/gpu_prof.py), cfgs as 4/20/1
#   timeline:[VAR=v@]<lib>       per-problem start/end of a -DSCPQP_PROF build (c2, B = 1024)
#   stats:<cfg>           rocprofv3 --kernel-trace --stats of the bench
#   pmc:<cfg>             SQ, MFMA, FETCH_SIZE and WRITE_SIZE passes, each its own rocprofv3 run
#   rollout               closed-loop rollout throughput (tools/bench_rollout.py)
#   c5classes             c5 per-horizon-class launch times
#   bitwise:<cfg>:<a.so>,<b.so>  every output of the two builds compared exactly (tools/bitwise_ab.py)
#   closedloop            closed-loop parity record of main.py's own run (8 vehicles, 50 steps)
# Everything goes to gpurun_out/<tag>/.
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
PKG=senquential-convex-programming-for-trajectory-planning_amd
run() {  # run <name> <seconds> cmd...
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    if [ $rc -ne 0 ]; then grep -B30 "^E " "$OUT/$name.log" | tail -40; tail -n 20 "$OUT/$name.log"; echo "!! $name rc=$rc"; exit $rc; fi
}
line() {  # summary of a bench JSON line on stdin
    python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', round(d['value']), round(d['roofline']['kernel_ms'],3), 'ipm/qp', round(d['mean_ipm_iters_per_qp'],2), 'conv', d['status_converged_frac'])"
}
for st in "$@"; do
    kind=${st%%:*}; rest=""; [ "$kind" != "$st" ] && rest=${st#*:}
    case $kind in
    tests)
        ARGS=(tests -m gpu -v -x -p no:cacheprovider --timeout 170 --timeout-method thread)
        [ -n "$rest" ] && ARGS+=(-k "$rest")
        run pytest 1100 python -u -m pytest "${ARGS[@]}"
        grep -E "passed|failed" $OUT/pytest.log | tail -2 ;;
    checktests)
        ARGS=(tests -m gpu -v -x -s -p no:cacheprovider --timeout 170 --timeout-method thread)
        [ -n "$rest" ] && ARGS+=(-k "$rest")
        run checktests 1100 env SCPQP_TEST_LIB=$PWD/$PKG/scpqp/libscpqp_check.so python -u -m pytest "${ARGS[@]}"
        grep -E "passed|failed|reduction-buffer" $OUT/checktests.log | tail -3 ;;
    reducecheck)
        lib=$rest; [ "${lib:0:1}" = / ] || lib=$PWD/$lib
        name=reducecheck_$(basename $lib .so)
        echo "== $name ($(date +%T))"
        timeout -k 10 300 python tools/reduce_check.py $lib > $OUT/$name.log 2>&1; rc=$?
        tail -7 $OUT/$name.log
        if [ $rc -gt 1 ]; then echo "!! $name rc=$rc"; exit $rc; fi ;;
    smoke)
        run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
        tail -1 $OUT/smoke.log ;;
    bench)
        cfg=${rest%%,*}; steps=""; [ "$cfg" != "$rest" ] && steps="--steps ${rest#*,} --warmup 1"
        extra=""   # every config with its CPU leg and parity sample (verdict r05 item 6)
        run bench_$cfg 600 python bench.py --config $cfg $steps $extra
        grep '^{' $OUT/bench_$cfg.log > $OUT/bench_$cfg.json
        line $cfg < $OUT/bench_$cfg.json ;;
    ab)
        cfgs=${rest%%:*}; r2=${rest#*:}; libs=${r2%%:*}; reps=1; [ "$libs" != "$r2" ] && reps=${r2#*:}
        for rep in $(seq $reps); do
            for cs in ${cfgs//,/ }; do
                c=${cs%%/*}; n=${cs##*/}
                for ent in ${libs//,/ }; do
                    lib=${ent##*@}; envs=""; [ "$ent" != "$lib" ] && envs=${ent%%@*}
                    [ "${lib:0:1}" = / ] || lib=$PWD/$lib
                    run ab 300 env $envs python bench.py --lib $lib --no-cpu --config $c --steps $n --warmup 1
                    grep '^{' $OUT/ab.log | line "$c $ent" | tee -a $OUT/ab.txt
                done
            done
        done ;;
    phases)
        ent=${rest%%:*}; cfgs="4:20:1"; [ "$ent" != "$rest" ] && cfgs=$(echo ${rest#*:} | tr ',/' ' :')
        lib=${ent##*@}; envs=""; [ "$ent" != "$lib" ] && envs=${ent%%@*}
        [ "${lib:0:1}" = / ] || lib=$PWD/$lib
        name=phases_$(basename $lib .so)${envs:+_${envs%%=*}}
        run $name 300 env $envs SCPQP_PROF_LIB=$lib python tools/gpu_prof.py $cfgs
        grep -v amdgpu.ids $OUT/$name.log ;;
    timeline)
        ent=$rest; lib=${ent##*@}; envs=""; [ "$ent" != "$lib" ] && envs=${ent%%@*}
        [ "${lib:0:1}" = / ] || lib=$PWD/$lib
        name=timeline${envs:+_${envs%%=*}}
        run $name 300 env $envs SCPQP_PROF_LIB=$lib python tools/gpu_timeline.py 1024
        head -20 $OUT/$name.log ;;
    stats)
        c=$rest; steps=5; [ $c = c3 ] && steps=2; [ $c = c2 ] && steps=10
        run stats_$c 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/stats_$c -o run -- python3 bench.py --config $c --steps $steps --warmup 2 --no-cpu
        find $OUT/stats_$c -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats_$c.csv \;
        grep '^{' $OUT/stats_$c.log > $OUT/bench_under_rocprof_$c.json || true
        head -3 $OUT/kernel_stats_$c.csv ;;
    pmc)
        c=$rest
        timeout -s KILL 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
        MFMA=$(python tools/pick_counters.py $OUT/counters_list.txt)
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
        python tools/pmc_summary.py $f $w $OUT/pmc_traffic_$c.json | grep -E "raw|bytes_per_launch|scratch" ;;
    rollout)
        run rollout 600 python tools/bench_rollout.py 1024 5 16
        grep '^{' $OUT/rollout.log > $OUT/rollout.json; cat $OUT/rollout.json ;;
    c5classes)
        run c5_classes 300 python tools/c5_classes.py 3
        cat $OUT/c5_classes.log ;;
    bitwise)
        c=${rest%%:*}; r2=${rest#*:}; la=${r2%%,*}; lb=${r2#*,}
        run bitwise_$c 300 python tools/bitwise_ab.py $c $la $lb
        tail -3 $OUT/bitwise_$c.log ;;
    closedloop)
        run closed_loop_main8 1000 python -u tools/closed_loop_parity.py main8 1 50 $OUT/closed_loop_main8.json
        tail -30 $OUT/closed_loop_main8.log ;;
    *) echo "unknown step $st"; exit 2 ;;
    esac
done
echo "== done $(date +%T)"
