#!/bin/bash
# bench.py (no CPU leg) under each forced memory plan: SCPQP_PLAN=0 (all LDS), 1 (vectors in workspace)
OUT=gpurun_out/${1:-planab}
mkdir -p $OUT
python -c "import torch" 2>/dev/null
for b in ${BATCHES:-1024 4096}; do
for p in ${PLANS:-0 1}; do
  SCPQP_PLAN=$p timeout -k 10 200 python bench.py --no-cpu --steps 5 --warmup 1 --batch $b > $OUT/p$p.b$b.log 2>&1 || { echo "plan $p failed"; tail -20 $OUT/p$p.b$b.log; exit 1; }
  grep '^{' $OUT/p$p.b$b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('plan $p B $b', round(d['value']), 'solves/s', round(d['roofline']['kernel_ms'],2), 'ms conv', d['status_converged_frac'])"
done
done
