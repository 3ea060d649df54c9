mkdir -p gpurun_out/scale
python -c "import torch" 2>/dev/null
timeout -k 10 300 python tools/gpu_scale.py 4 20 > gpurun_out/scale/c2.txt 2>&1; rc=$?; cat gpurun_out/scale/c2.txt; exit $rc
