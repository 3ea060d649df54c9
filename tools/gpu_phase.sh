mkdir -p gpurun_out/r01d
python -c "import torch" 
timeout -k 10 120 python tools/gpu_prof.py > gpurun_out/r01d/phases.txt 2>&1; echo "rc=$?" >> gpurun_out/r01d/phases.txt
cat gpurun_out/r01d/phases.txt
bash tools/gpu_round.sh r01d prof pmc
