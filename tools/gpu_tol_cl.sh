#!/bin/bash
# IPM-tolerance A/B with the polish cap, then refreshed 50-step closed-loop parity records.
mkdir -p gpurun_out/pab gpurun_out/cl
timeout -k 10 300 python -u tools/gpu_param_ab.py c2:10 ipm_tol=1e-9 ipm_tol=3e-9 ipm_tol=1e-8 > gpurun_out/pab/tol_c2.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/gpu_param_ab.py c4:3 ipm_tol=1e-9 ipm_tol=3e-9 ipm_tol=1e-8 > gpurun_out/pab/tol_c4.txt 2>&1 || exit 1
timeout -k 10 400 python -u tools/closed_loop_parity.py main8 1 50 gpurun_out/cl/closed_loop_main8.json > gpurun_out/cl/main8.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/closed_loop_parity.py c2 16 50 gpurun_out/cl/closed_loop_c2x16.json > gpurun_out/cl/c2x16.log 2>&1 || exit 1
