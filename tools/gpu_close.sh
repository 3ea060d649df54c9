#!/bin/bash
# Closing measurement session on the shipped library, one box: a run-time parameter A/B
# (tools/gpu_param_ab.py, e.g. the IPM tolerance), then the measurement records
# (tools/gpu_measure.sh: rocprofv3 kernel stats, SQ / MFMA / FETCH / WRITE passes per config,
# phase stamps and the c2 timeline of the diagnostic build libscpqp_prof.so).
#   gpurun --timeout 1200 -- bash tools/gpu_close.sh <tag> "<param set> ..."
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
if [ $# -gt 0 ]; then
    timeout -k 10 400 python tools/gpu_param_ab.py c2:10 "$@" > $OUT/pab_c2.log 2>&1 || { tail -20 $OUT/pab_c2.log; exit 1; }
    grep -v amdgpu.ids $OUT/pab_c2.log
    timeout -k 10 400 python tools/gpu_param_ab.py c4:3 "$@" > $OUT/pab_c4.log 2>&1 || { tail -20 $OUT/pab_c4.log; exit 1; }
    grep -v amdgpu.ids $OUT/pab_c4.log
fi
bash tools/gpu_measure.sh $TAG "c2 c3 c5" prof
