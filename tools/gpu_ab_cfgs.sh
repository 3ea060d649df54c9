#!/bin/bash
# A/B of library builds on several configs (bench.py, no CPU leg), then the gpu
# tests selected by -k on the first library.
#   gpurun -- bash tools/gpu_ab_cfgs.sh <tag> "<cfg:steps ...>" "<pytest -k>" lib1.so lib2.so ...
TAG=$1; CFGS=$2; K=$3; shift 3
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for cs in $CFGS; do
    c=${cs%%:*}; st=${cs##*:}
    for lib in "$@"; do
      SCPQP_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu --config $c --steps $st --warmup 1 > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; exit 1; }
      grep '^{' $OUT/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', '$lib', round(d['value']), round(d['roofline']['kernel_ms'],3))"
    done
  done
done
if [ -n "$K" ]; then
  SCPQP_LIB=$PWD/$1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "$K" > $OUT/pytest.log 2>&1
  rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && { grep -B40 "^E " $OUT/pytest.log | tail -60; exit $rc; }
fi
exit 0
