#!/bin/bash
# End-of-round session on the shipped library: full GPU test suite, smoke(), then the
# bench lines of every BASELINE configuration (c2 with its CPU leg, c3, c5, c4 one rank).
# Counter records come from tools/gpu_measure.sh (its own session).
#   gpurun --timeout 1200 -- bash tools/gpu_final.sh <tag> [skip-tests]
set -u
TAG=${1:-final}; SKIP=${2:-}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
step() {  # step <name> <seconds> cmd...
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    if [ $rc -ne 0 ]; then grep -B30 "^E " "$OUT/$name.log" | tail -60; tail -n 20 "$OUT/$name.log"; echo "!! $name rc=$rc"; exit $rc; fi
}
if [ -z "$SKIP" ]; then
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
for c in c2 c3 c5 c4; do python -c "import json; d=json.load(open('$OUT/bench_$c.json')); print('$c', round(d['value']), d['unit'], 'kernel_ms', round(d['roofline']['kernel_ms'], 3))"; done
echo "== done $(date +%T)"
