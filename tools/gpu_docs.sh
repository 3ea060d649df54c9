#!/bin/bash
# Diagnostics quoted in DESIGN.md: phase stamps, batch scaling, per-problem timeline, c3/c5 bench lines.
OUT=gpurun_out/${1:-docs}
mkdir -p $OUT
python -c "import torch" 2>/dev/null
timeout -k 10 200 python tools/gpu_prof.py > $OUT/phases.txt 2>&1 || { echo "prof failed"; tail $OUT/phases.txt; exit 1; }
timeout -k 10 200 python tools/gpu_scale.py 4 20 > $OUT/scaling.txt 2>&1 || { echo "scale failed"; tail $OUT/scaling.txt; exit 1; }
timeout -k 10 200 python tools/gpu_timeline.py 1024 > $OUT/timeline.txt 2>&1 || { echo "timeline failed"; tail $OUT/timeline.txt; exit 1; }
for c in c3 c5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu --steps 3 --warmup 1 > $OUT/$c.log 2>&1 || { echo "$c failed"; tail -5 $OUT/$c.log; exit 1; }
  grep '^{' $OUT/$c.log > $OUT/$c.json
done
cat $OUT/scaling.txt; head -3 $OUT/timeline.txt
