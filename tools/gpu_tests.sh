#!/bin/bash
# GPU parity tests (one pytest process) and optional closed-loop parity records.
#   gpurun -- bash tools/gpu_tests.sh <tag> [pytest -k expr] [closed-loop cases...]
TAG=${1:-t}; K=${2:-}; shift 2 || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS=(tests -m gpu -v -x -p no:cacheprovider --timeout 300 --timeout-method thread)
[ -n "$K" ] && ARGS+=(-k "$K")
timeout -k 10 900 python -u -m pytest "${ARGS[@]}" > $OUT/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/pytest.log | tail -70
[ $rc -ne 0 ] && { grep -B30 "^E " $OUT/pytest.log | tail -80; exit $rc; }
for c in "$@"; do
  set -- $(echo $c | tr ':' ' ')
  timeout -k 10 600 python -u tools/closed_loop_parity.py $1 $2 $3 $OUT/closed_loop_$1.json > $OUT/cl_$1.log 2>&1 || { tail -30 $OUT/cl_$1.log; exit 1; }
  head -30 $OUT/cl_$1.log
done
