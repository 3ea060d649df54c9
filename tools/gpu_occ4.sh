#!/bin/bash
# A/B of the OCC=4 diagnostic build (plan 2, 4 workgroups per CU) against the shipped
# library on c2.  Swaps libscpqp.so for libscpqp_occ4.so on the box copy only.
OUT=gpurun_out/${1:-occ4}
mkdir -p $OUT
L=senquential-convex-programming-for-trajectory-planning_amd/scpqp
show() { grep '^{' $1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', round(d['value']), 'solves/s', round(d['roofline']['kernel_ms'],2), 'ms grid', d['roofline']['workgroups'], 'plan', d['roofline']['memory_plan'], 'conv', d['status_converged_frac'])"; }
for b in ${BATCHES:-1024}; do
  timeout -k 10 200 python bench.py --no-cpu --steps 5 --warmup 1 --batch $b > $OUT/base.b$b.log 2>&1 || { echo "base failed"; tail -20 $OUT/base.b$b.log; exit 1; }
  show $OUT/base.b$b.log "base B $b"
  SCPQP_PLAN=2 timeout -k 10 200 python bench.py --no-cpu --steps 5 --warmup 1 --batch $b > $OUT/p2.b$b.log 2>&1 || { echo "p2 failed"; tail -20 $OUT/p2.b$b.log; exit 1; }
  show $OUT/p2.b$b.log "plan2 occ3 B $b"
done
cp $L/libscpqp_occ4.so $L/libscpqp.so
for b in ${BATCHES:-1024}; do
  SCPQP_PLAN=2 SCPQP_OCC4=1 timeout -k 10 200 python bench.py --no-cpu --steps 5 --warmup 1 --batch $b > $OUT/occ4.b$b.log 2>&1 || { echo "occ4 failed"; tail -20 $OUT/occ4.b$b.log; exit 1; }
  show $OUT/occ4.b$b.log "plan2 occ4 B $b"
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- python3 bench.py --no-cpu --steps 3 --warmup 1 > $OUT/prof.log 2>&1 || true
