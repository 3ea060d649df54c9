#!/bin/bash
# Run-time polish-penalty A/B on the shipped kernel (tools/gpu_param_ab.py, interleaved).
#   gpurun --timeout 1200 -- bash tools/gpu_pab_polish.sh
set -u
OUT=gpurun_out/r03_pab_polish; mkdir -p $OUT
export TMPDIR=/tmp
for c in c2:10 c4:3 c5:5; do
    timeout -k 10 400 python tools/gpu_param_ab.py $c "polish_delta=3e-7" "polish_delta=2e-7" "polish_delta=5e-7" > $OUT/${c%%:*}.log 2>&1 || { tail -20 $OUT/${c%%:*}.log; exit 1; }
    grep -v amdgpu $OUT/${c%%:*}.log
done
