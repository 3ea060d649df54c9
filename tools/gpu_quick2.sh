#!/bin/bash
# Parity subset + bench (no CPU leg): gpurun -- bash tools/gpu_quick2.sh <tag> [pytest -k expr]
TAG=${1:-q}; K=${2:-"parity or trace or known"}
OUT=gpurun_out/$TAG; mkdir -p $OUT
ls -la --time-style=+%T senquential-convex-programming-for-trajectory-planning_amd/scpqp/libscpqp.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "$K" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && { grep -B40 "^E " $OUT/pytest.log | tail -60; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('value', round(d['value']), 'kernel_ms', round(r['kernel_ms'],3), 'ipm/qp', round(d['mean_ipm_iters_per_qp'],3), 'scp', d['mean_scp_iters'])"
