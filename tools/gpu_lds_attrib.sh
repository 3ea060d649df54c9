#!/bin/bash
# LDS bank-conflict attribution from counters (round 4): one SQ pass per build and config.
# The diagnostic builds repeat one phase result-neutrally (-DSCPQP_DIAG_X2_TRAIL: the
# trailing update's loads and stores a second time with the entries unchanged; _SOLVE: every
# triangular solve twice; _ASM: the assembly tiles twice), so the conflict count of that phase
# is the build's count minus the shipped library's.
#   gpurun -- bash tools/gpu_lds_attrib.sh <tag> "c2 c5"
set -u
TAG=$1; CFGS=${2:-"c2 c5"}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
for c in $CFGS; do
  for lib in senquential-convex-programming-for-trajectory-planning_amd/scpqp/libscpqp.so ab/lib_x2_trail.so ab/lib_x2_solve.so ab/lib_x2_asm.so; do
    b=$(basename $lib .so)
    SCPQP_LIB=$PWD/$lib timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_BUSY_CYCLES -f csv -d $OUT/lds_${c}_$b -o run -- python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu > $OUT/lds_${c}_$b.log 2>&1 || { tail -5 $OUT/lds_${c}_$b.log; exit 1; }
    echo "== $c $b"
    python tools/pmc_table.py $(find $OUT/lds_${c}_$b -name '*counter_collection.csv') | tee $OUT/lds_${c}_$b.txt
  done
done
