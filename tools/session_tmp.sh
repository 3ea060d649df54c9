set -e
mkdir -p gpurun_out/r06d
timeout -k 10 100 python tools/solve_time.py senquential-convex-programming-for-trajectory-planning_amd/scpqp/libscpqp.so c4 2 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06d/prod_c4.log
timeout -k 10 200 python tools/solve_time.py senquential-convex-programming-for-trajectory-planning_amd/scpqp/libscpqp_check.so c4 2 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06d/check_c4.log
