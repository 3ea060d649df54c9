#!/bin/bash
# c2/c4 A/B of c2-only diagnostic builds plus c2-shaped parity tests on one of them.
#   gpurun -- bash tools/gpu_c2_ab.sh <tag> "<lib.so ...>" <lib for the tests>
TAG=$1; LIBS=$2; TLIB=$3; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
bash tools/gpu_session.sh $TAG "c2:5 c4:3" "$LIBS" none || exit 1
SCPQP_LIB=$PWD/$TLIB timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "c2_full or c4_rank" > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && { grep -B5 -A30 "^E " $OUT/pytest.log | head -80; exit $rc; }
exit 0
