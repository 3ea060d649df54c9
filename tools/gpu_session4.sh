#!/bin/bash
# Shipped library after the polish-tolerance change: GPU suite, polish-cap A/B on the
# new tolerance (c3, c2), bench lines c2/c3/c5 with CPU legs, timeline.
#   gpurun --timeout 1200 -- bash tools/gpu_session4.sh <tag>
set -u
TAG=${1:-s4}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "== $name"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    if [ $rc -ne 0 ]; then grep -B30 "^E " "$OUT/$name.log" | tail -60; tail -n 20 "$OUT/$name.log"; echo "!! $name rc=$rc"; exit $rc; fi
}
step pytest 900 python -u -m pytest tests -m gpu -v -x -p no:cacheprovider --timeout 300 --timeout-method thread
grep -E "passed|failed" $OUT/pytest.log | tail -1
step cap_c3 300 python -u tools/gpu_param_ab.py c3:2 polish_refine=0 polish_refine=12 polish_refine=20
step cap_c2 300 python -u tools/gpu_param_ab.py c2:10 polish_refine=0 polish_refine=40 polish_refine=8
step timeline 300 python -u tools/gpu_timeline.py
for c in c2 c3 c5; do
    extra=""; [ $c = c3 ] && extra="--steps 3 --warmup 1"
    step bench_$c 600 python bench.py --config $c $extra
    grep '^{' $OUT/bench_$c.log > $OUT/bench_$c.json
done
echo "== done"
