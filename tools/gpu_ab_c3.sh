#!/bin/bash
# c3 A/B of library builds plus the c3 parity tests on the first library.
#   gpurun -- bash tools/gpu_ab_c3.sh <tag> lib1.so lib2.so ...
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
BENCH_ARGS="--config c3 --steps 3 --warmup 1" timeout -k 10 600 bash tools/gpu_ab_libs.sh "$@" || exit 1
SCPQP_LIB=$PWD/$2 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "c3" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && { grep -B40 "^E " $OUT/pytest.log | tail -60; exit $rc; }
exit 0
