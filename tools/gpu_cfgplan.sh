#!/bin/bash
# GPU tests, then bench.py (no CPU leg) on c3 and c5 under each memory plan.
OUT=gpurun_out/${1:-cfgplan}
mkdir -p $OUT
python -c "import torch" 2>/dev/null
timeout -k 10 400 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $OUT/pytest.txt 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for c in c5 c3; do
for p in ${PLANS:-default 1 2}; do
  if [ "$p" = default ]; then unset SCPQP_PLAN; else export SCPQP_PLAN=$p; fi
  timeout -k 10 300 python bench.py --config $c --no-cpu --steps 3 --warmup 1 > $OUT/$c.p$p.log 2>&1 || { echo "$c plan $p failed"; tail -5 $OUT/$c.p$p.log; continue; }
  grep '^{' $OUT/$c.p$p.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c plan $p', round(d['value']), 'solves/s', round(d['roofline']['kernel_ms'],2), 'ms conv', d['status_converged_frac'], d['config'].get('resources', ''))"
done
done
