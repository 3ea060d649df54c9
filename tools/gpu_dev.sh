#!/bin/bash
# Development session on one GPU box: optional probes, c2 bench lines (no CPU leg), then a
# subset (or all) of the GPU tests; stops at the first failing step.
#   gpurun -- bash tools/gpu_dev.sh <tag> "<probe ...>" "<cfg:steps ...>" [pytest -k expr | all | none]
set -u
TAG=$1; PROBES=${2:-}; CFGS=${3:-}; K=${4:-none}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
step() {  # step <name> <seconds> cmd...
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    if [ $rc -ne 0 ]; then grep -B30 "^E " "$OUT/$name.log" | tail -40; tail -n 20 "$OUT/$name.log"; echo "!! $name rc=$rc"; exit $rc; fi
}
for p in $PROBES; do
    step probe_$(basename $p) 120 ./$p
    cat $OUT/probe_$(basename $p).log
done
for cs in $CFGS; do
    c=${cs%%:*}; st=${cs##*:}
    step bench_$c 300 python bench.py --no-cpu --config $c --steps $st --warmup 1
    grep '^{' $OUT/bench_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', round(d['value']), round(d['roofline']['kernel_ms'],3), 'ipm/qp', round(d['mean_ipm_iters_per_qp'],2), 'pol/qp', round(d['mean_polish_solves_per_qp'],2), 'conv', d['status_converged_frac'])"
done
if [ "$K" != "none" ]; then
    ARGS=(tests -m gpu -v -x -p no:cacheprovider --timeout 300 --timeout-method thread)
    [ "$K" != "all" ] && ARGS+=(-k "$K")
    step pytest 900 python -u -m pytest "${ARGS[@]}"
    grep -E "passed|failed" $OUT/pytest.log | tail -3
fi
echo "== done $(date +%T)"
