#!/bin/bash
# Round-end measurement of the shipped library in one box session: the full GPU test
# suite, phase stamps and timeline (diagnostic build), bench lines with CPU legs for
# c2/c3, then per-config rocprofv3 kernel stats and PMC passes (tools/gpu_round2.sh)
# with the c5 and c4 bench lines.
#   gpurun --timeout 1800 -- bash tools/gpu_final2.sh <tag>
set -u
TAG=${1:-final2}
bash tools/gpu_final.sh $TAG || exit $?
bash tools/gpu_round2.sh ${TAG}_prof "c2 c3 c5" || exit $?
OUT=gpurun_out/$TAG
for c in c5 c4; do
    echo "== bench_$c ($(date +%T))"
    extra=""; [ $c = c4 ] && extra="--no-cpu"
    timeout -k 10 400 python bench.py --config $c $extra > $OUT/bench_$c.log 2>&1 || { tail -20 $OUT/bench_$c.log; exit 1; }
    grep '^{' $OUT/bench_$c.log > $OUT/bench_$c.json
done
echo "== all done $(date +%T)"
