#!/bin/bash
# PMC counter passes on the bench kernel (each pass its own rocprofv3 run, --kernel-trace only).
TAG=${1:-pmc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
python -c "import torch" 2>/dev/null
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $line -f csv -d $OUT/p$i -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu ${BENCH_ARGS} > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -20 $OUT/p$i.log; exit 1; }
  find $OUT/p$i -name '*counter_collection.csv' -exec cp {} $OUT/pass$i.csv \;
done <<'PASSES'
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVES SQ_INSTS_VMEM
SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
PASSES
python tools/pmc_table.py $OUT/pass*.csv | tee $OUT/summary.txt
