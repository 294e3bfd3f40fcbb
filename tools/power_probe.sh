#!/bin/bash
# Dev (GPU box): power and clocks while the headline kernel runs (rocm-smi
# samples during a long bench run; read-only queries).
set -o pipefail
mkdir -p gpurun_out/pw
timeout -k 10 150 python3 -u bench.py --steps 5000 --warmup 5 --no-cpu --no-check > gpurun_out/pw/bench.log 2>&1 &
BP=$!
sleep 5
for i in 1 2 3 4 5 6 7 8 9 10 11 12; do
  timeout 20 rocm-smi --showpower --showclocks --showtemp 2>/dev/null | grep -E "^0|GPU\[0\]|Power|sclk|mclk|fclk|Temp" | head -12 >> gpurun_out/pw/smi.txt
  echo ---- >> gpurun_out/pw/smi.txt
  sleep 1
done
wait $BP; rc=$?
grep '^{' gpurun_out/pw/bench.log | cut -c1-300
grep -E "sclk|Power \\(W\\)|junction" gpurun_out/pw/smi.txt | head -48
exit $rc
