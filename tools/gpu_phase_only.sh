#!/bin/bash
mkdir -p gpurun_out/${1:-ph}
python -c "import torch" 2>/dev/null
timeout -k 10 120 python tools/gpu_prof.py > gpurun_out/${1:-ph}/phases.txt 2>&1; rc=$?
cat gpurun_out/${1:-ph}/phases.txt; exit $rc
