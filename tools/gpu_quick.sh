#!/bin/bash
# Quick GPU iteration: parity tests, phase stamps (diagnostic build), bench without CPU leg.
TAG=${1:-quick}
OUT=gpurun_out/$TAG
mkdir -p $OUT
python -c "import torch" 2>/dev/null
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && { echo "pytest rc=$rc"; tail -40 $OUT/pytest.log; exit $rc; }
timeout -k 10 120 python tools/gpu_prof.py > $OUT/phases.txt 2>&1 || { echo "prof failed"; cat $OUT/phases.txt; exit 1; }
cat $OUT/phases.txt
timeout -k 10 300 python bench.py --no-cpu > $OUT/bench.log 2>&1 || { echo "bench failed"; cat $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'kernel_ms', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])"
if [ -n "$PMC" ]; then
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d $OUT/pmcw -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > $OUT/pmcw.log 2>&1 && python tools/pmc_table.py $(find $OUT/pmcw -name '*counter_collection.csv')
fi
