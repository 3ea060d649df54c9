#!/bin/bash
# A/B of library builds on one box: bench.py (no CPU leg) per SCPQP_LIB, interleaved twice.
#   gpurun -- bash tools/gpu_ab_libs.sh <tag> lib1.so lib2.so ...
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
for rep in 1 2; do
  for lib in "$@"; do
    SCPQP_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu --steps 20 ${BENCH_ARGS} > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; exit 1; }
    grep '^{' $OUT/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', round(d['value']), round(d['roofline']['kernel_ms'],3))"
  done
done
