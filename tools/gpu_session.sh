#!/bin/bash
# One GPU box session: A/B bench of library builds (bench.py, no CPU leg, two
# alternating repetitions), then the GPU test suite on the shipped library.
#   gpurun -- bash tools/gpu_session.sh <tag> "<cfg:steps ...>" "<lib.so ...>" [pytest -k expr | all | none]
# Libraries built with -DSCPQP_DIAG_C2ONLY serve c2-shaped problems only (c2, c4).  A library
# entry of the form VAR=value@lib.so runs that library with the environment variable set
# (e.g. SCPQP_SHAPE=0@ab/lib_diag.so: the runtime-shape instantiation of a -DSCPQP_DIAG build).
TAG=$1; CFGS=$2; LIBS=$3; K=${4:-none}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for cs in $CFGS; do
    c=${cs%%:*}; st=${cs##*:}
    for ent in $LIBS; do
      lib=${ent##*@}; envs=""; [ "$ent" != "$lib" ] && envs=${ent%%@*}
      env $envs SCPQP_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu --config $c --steps $st --warmup 1 > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; exit 1; }
      grep '^{' $OUT/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', '$ent', round(d['value']), round(d['roofline']['kernel_ms'],3), 'ipm/qp', round(d['mean_ipm_iters_per_qp'],2), 'conv', d['status_converged_frac'])" | tee -a $OUT/ab.txt
    done
  done
done
if [ "$K" != "none" ]; then
  ARGS=(tests -m gpu -v -x -p no:cacheprovider --timeout 300 --timeout-method thread)
  [ "$K" != "all" ] && ARGS+=(-k "$K")
  timeout -k 10 900 python -u -m pytest "${ARGS[@]}" > $OUT/pytest.log 2>&1
  rc=$?
  grep -E "passed|failed" $OUT/pytest.log | tail -3
  [ $rc -ne 0 ] && { grep -E "FAILED|ERROR" $OUT/pytest.log | head; grep -B30 "^E " $OUT/pytest.log | tail -60; exit $rc; }
fi
exit 0
