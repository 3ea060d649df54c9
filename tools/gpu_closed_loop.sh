#!/bin/bash
# Closed-loop parity record of main.py's own run (8 vehicles, 50 MPC steps) on the shipped library.
#   gpurun --timeout 1200 -- bash tools/gpu_closed_loop.sh <tag>
TAG=${1:-cl}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u tools/closed_loop_parity.py main8 1 50 $OUT/closed_loop_main8.json > $OUT/cl.log 2>&1
rc=$?
tail -30 $OUT/cl.log
exit $rc
