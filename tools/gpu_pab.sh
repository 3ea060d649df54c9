set -u
OUT=gpurun_out/r03_pab; mkdir -p $OUT
timeout -k 10 400 python tools/gpu_param_ab.py c2:10 "ipm_tol=1e-9" "ipm_tol=3e-9" "ipm_tol=1e-8" "polish_delta=6e-7" > $OUT/c2.log 2>&1 || { tail -20 $OUT/c2.log; exit 1; }
cat $OUT/c2.log
timeout -k 10 400 python tools/gpu_param_ab.py c4:3 "ipm_tol=1e-9" "ipm_tol=3e-9" "ipm_tol=1e-8" > $OUT/c4.log 2>&1 || { tail -20 $OUT/c4.log; exit 1; }
cat $OUT/c4.log
