mkdir -p gpurun_out/edge
rm -f gpurun_out/edge/log.txt
python -c "import torch, numpy, scipy" >> gpurun_out/edge/log.txt 2>&1
for c in ${CASES:-hp20 zero1 zero2 big2 badhp hp1 hp64}; do
  timeout -k 5 45 python tools/edge_probe.py $c >> gpurun_out/edge/log.txt 2>&1 || { echo "FAILED $c rc=$?" >> gpurun_out/edge/log.txt; break; }
done
cat gpurun_out/edge/log.txt
