#!/bin/bash
# Polish stopping-tolerance variants (ab/pt*.so) against the shipped library, with
# |du| measured against the shipped library's answers (SAVE/CMP in tools/gpu_param_ab.py).
mkdir -p gpurun_out/pt
for c in c3:2 c2:10 c5:5; do
    cfg=${c%%:*}
    SAVE=gpurun_out/pt/$cfg.npz timeout -k 10 300 python -u tools/gpu_param_ab.py $c polish_refine=0 > gpurun_out/pt/ship_$cfg.txt 2>&1 || exit 1
    for v in pt9 pt3; do
        SCPQP_LIB=$PWD/ab/$v.so CMP=gpurun_out/pt/$cfg.npz timeout -k 10 300 python -u tools/gpu_param_ab.py $c polish_refine=0 > gpurun_out/pt/${v}_$cfg.txt 2>&1 || exit 1
    done
done
rm -f gpurun_out/pt/*.npz
