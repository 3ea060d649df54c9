#!/bin/bash
# One GPU box session on the shipped library: the GPU test suite, smoke(), the bench lines
# of every BASELINE configuration, then diagnostics (phase stamps of the diagnostic build
# libscpqp_prof.so at B = 1 and the c5 per-horizon-class launch times).
#   gpurun --timeout 1500 -- bash tools/gpu_round.sh <tag> [skip-tests] [diag]
set -u
TAG=$1; SKIP=${2:-}; DIAG=${3:-}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
step() {  # step <name> <seconds> cmd...
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    if [ $rc -ne 0 ]; then grep -B30 "^E " "$OUT/$name.log" | tail -40; tail -n 20 "$OUT/$name.log"; echo "!! $name rc=$rc"; exit $rc; fi
}
if [ "$SKIP" != "skip-tests" ]; then
    step pytest 900 python -u -m pytest tests -m gpu -v -x -p no:cacheprovider --timeout 300 --timeout-method thread
    grep -E "passed|failed" $OUT/pytest.log | tail -2
    step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
fi
step bench_c2 400 python bench.py
grep '^{' $OUT/bench_c2.log > $OUT/bench_c2.json
step bench_c3 600 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu
grep '^{' $OUT/bench_c3.log > $OUT/bench_c3.json
step bench_c5 400 python bench.py --config c5 --steps 5 --warmup 1 --no-cpu
grep '^{' $OUT/bench_c5.log > $OUT/bench_c5.json
step bench_c4 400 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu
grep '^{' $OUT/bench_c4.log > $OUT/bench_c4.json
for c in c2 c3 c5 c4; do python -c "import json; d=json.load(open('$OUT/bench_$c.json')); print('$c', round(d['value']), d['unit'], 'kernel_ms', round(d['roofline']['kernel_ms'], 3), 'ipm/qp', round(d['mean_ipm_iters_per_qp'], 2))"; done
if [ -n "$DIAG" ]; then
    step phases 300 python tools/gpu_prof.py 4:20:1 8:30:1
    grep -v amdgpu.ids $OUT/phases.log
    step c5_classes 300 python tools/c5_classes.py 3
    cat $OUT/c5_classes.log
fi
echo "== done $(date +%T)"
