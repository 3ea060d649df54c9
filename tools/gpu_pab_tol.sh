set -u
OUT=gpurun_out/r03_pab3; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python tools/gpu_param_ab.py c3:2 "ipm_tol=1e-9" "ipm_tol=3e-9" > $OUT/c3.log 2>&1 || { tail -20 $OUT/c3.log; exit 1; }
grep -v amdgpu $OUT/c3.log
timeout -k 10 400 python tools/gpu_param_ab.py c2:10 "ipm_tol=1e-9" "ipm_tol=3e-9" > $OUT/c2.log 2>&1 || { tail -20 $OUT/c2.log; exit 1; }
grep -v amdgpu $OUT/c2.log
timeout -k 10 400 python tools/gpu_param_ab.py c5:5 "ipm_tol=1e-9" "ipm_tol=3e-9" > $OUT/c5.log 2>&1 || { tail -20 $OUT/c5.log; exit 1; }
grep -v amdgpu $OUT/c5.log
