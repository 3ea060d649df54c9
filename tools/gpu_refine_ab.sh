#!/bin/bash
# A/B of the cold-polish solve cap (polish_refine) on c2/c4/c5/c3 (tools/gpu_param_ab.py).
mkdir -p gpurun_out/pab
timeout -k 10 300 python -u tools/gpu_param_ab.py c2:10 polish_refine=40 polish_refine=16 polish_refine=12 polish_refine=10 polish_refine=8 > gpurun_out/pab/ref2_c2.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/gpu_param_ab.py c3:2 polish_refine=40 polish_refine=12 polish_refine=8 > gpurun_out/pab/ref2_c3.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/gpu_param_ab.py c4:3 polish_refine=40 polish_refine=12 polish_refine=8 > gpurun_out/pab/ref2_c4.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/gpu_param_ab.py c5:5 polish_refine=40 polish_refine=12 polish_refine=8 > gpurun_out/pab/ref2_c5.txt 2>&1 || exit 1
