#!/bin/bash
# HBM traffic (FETCH_SIZE / WRITE_SIZE passes, rocprofv3 --kernel-trace --pmc) of the
# c2 bench kernel under each forced memory plan.
OUT=gpurun_out/${1:-pmcplan}
mkdir -p $OUT
export TMPDIR=/tmp
python -c "import torch" 2>/dev/null
for p in ${PLANS:-0 1}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    SCPQP_PLAN=$p timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c -f csv -d $OUT/p$p$c -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > $OUT/p$p$c.log 2>&1 || { echo "plan $p $c failed"; tail -5 $OUT/p$p$c.log; exit 1; }
    find $OUT/p$p$c -name '*counter_collection.csv' -exec cp {} $OUT/p$p.$c.csv \;
  done
  python tools/pmc_summary.py $OUT/p$p.FETCH_SIZE.csv $OUT/p$p.WRITE_SIZE.csv $OUT/p$p.json | grep -E '"kernel"|hbm_bytes|hbm_read|hbm_write|scratch'
  grep '^{' $OUT/p${p}WRITE_SIZE.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('plan $p', round(d['value']), 'solves/s')"
done
