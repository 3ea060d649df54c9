mkdir -p gpurun_out/c3
python -c "import torch" 2>/dev/null
timeout -k 10 700 python tools/c3_probe.py 8 30 32 > gpurun_out/c3/probe.txt 2>&1; rc=$?; cat gpurun_out/c3/probe.txt; exit $rc
