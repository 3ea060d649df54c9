mkdir -p gpurun_out/pab
for c in c2:20 c4:3 c5:10 c3:2; do
  SCPQP_LIB=$PWD/ab/ws03.so timeout -k 10 300 python -u tools/gpu_param_ab.py $c polish_delta=1e-6 > gpurun_out/pab/ws03_${c%%:*}.txt 2>&1 || exit 1
  SCPQP_LIB=$PWD/ab/ws1.so timeout -k 10 300 python -u tools/gpu_param_ab.py $c polish_delta=3e-7 > gpurun_out/pab/ws1_${c%%:*}.txt 2>&1 || exit 1
done
