#!/bin/bash
# bench.py on the BASELINE configs c2 (the metric's workload), c3 and c5.
OUT=gpurun_out/${1:-cfg}
mkdir -p $OUT
python -c "import torch" 2>/dev/null
for c in c2 c3 c5; do
  timeout -k 10 400 python bench.py --config $c --steps 5 --warmup 1 ${CPU:---no-cpu} > $OUT/$c.log 2>&1 || { echo "$c failed"; tail -20 $OUT/$c.log; exit 1; }
  grep '^{' $OUT/$c.log > $OUT/$c.json
  python -c "import json; d=json.load(open('$OUT/$c.json')); print('$c', round(d['value']), 'solves/s', round(d['roofline']['kernel_ms'],2), 'ms', 'frac', round(d['roofline']['frac'],4), 'conv', d['status_converged_frac'], 'warm', round(d['warm_certified_qp_frac'],2), d.get('cpu_baseline',{}).get('value'), d.get('traj_linf_err'))"
done
