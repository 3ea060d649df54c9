#!/bin/bash
# One GPU-box session: parity tests, the bench line, the rocprofv3 kernel-trace
# summary and the HBM PMC passes (separate runs, as MI355X_MICROARCH.md asks).
#   gpurun --timeout 1200 -- bash tools/gpu_round.sh [tag] [steps...]
# steps: tests bench prof pmc (default: all)
set -u
TAG=${1:-r01}
shift || true
STEPS=${*:-tests bench prof pmc}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
has() { [[ " $STEPS " == *" $1 "* ]]; }
run() {  # run <name> <seconds> cmd...  ; stops the script on any failure
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    tail -n 25 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then echo "!! $name failed rc=$rc"; exit $rc; fi
}
ls -la senquential-convex-programming-for-trajectory-planning_amd/scpqp/*.so
if has tests; then
    run pytest_gpu 700 python -m pytest tests -m gpu -q --maxfail=10 -p no:cacheprovider
fi
if has bench; then
    run bench 400 python bench.py
    grep '^{' "$OUT/bench.log" > "$OUT/bench.json"
fi
if has prof; then
    run rocprof_stats 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o run -- \
        python3 bench.py --steps 10 --warmup 2 --no-cpu
    find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
    grep '^{' "$OUT/rocprof_stats.log" > "$OUT/bench_under_rocprof.json" || true
fi
if has pmc; then
    run pmc_fetch 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d "$OUT/pmc_fetch" -o run -- \
        python3 bench.py --steps 3 --warmup 1 --no-cpu
    run pmc_write 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d "$OUT/pmc_write" -o run -- \
        python3 bench.py --steps 3 --warmup 1 --no-cpu
    find "$OUT/pmc_fetch" -name '*counter_collection.csv' -exec cp {} "$OUT/pmc_fetch.csv" \;
    find "$OUT/pmc_write" -name '*counter_collection.csv' -exec cp {} "$OUT/pmc_write.csv" \;
fi
echo "== done $(date +%T)"
