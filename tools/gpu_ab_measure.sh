#!/bin/bash
# Closing session of a round, one box: an A/B of a candidate build (one repetition), then the
# measurement records of the shipped library (tools/gpu_measure.sh: rocprofv3 kernel stats,
# SQ / MFMA / FETCH / WRITE passes per config, phase stamps and the c2 timeline).
#   gpurun --timeout 1200 -- bash tools/gpu_ab_measure.sh <tag> "<candidate.so ...>"
set -u
TAG=$1; CAND=${2:-}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
P=senquential-convex-programming-for-trajectory-planning_amd/scpqp
for c in c2:10 c4:3 c5:5 c3:2; do
    cfg=${c%%:*}; st=${c##*:}
    for lib in $P/libscpqp.so $CAND; do
        SCPQP_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu --config $cfg --steps $st --warmup 1 > $OUT/ab.log 2>&1 || { tail -5 $OUT/ab.log; exit 1; }
        grep '^{' $OUT/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', '$lib', round(d['value']), round(d['roofline']['kernel_ms'],3), 'ipm/qp', round(d['mean_ipm_iters_per_qp'],2))" | tee -a $OUT/ab.txt
    done
done
bash tools/gpu_measure.sh $TAG "c2 c3 c5" prof
