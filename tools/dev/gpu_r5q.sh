#!/bin/bash
# Round 5, box pass q: stereo s16 / planar mixes of 1-3 tracks on the 8-row
# fused kernels (phantom rows) against the generic kernel (XM_FAST_IO_MINTR
# 1 vs the default 4), same box, every line bit-checked; the s16 / planar /
# conversion GPU tests with the knob at 1.
set -o pipefail
mkdir -p gpurun_out/r5q
export TMPDIR=/tmp
XM_FAST_IO_MINTR=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_convert.py tests/test_gpu_fast_convert.py tests/test_gpu_parity.py tests/test_gpu_fast_layouts.py tests/test_gpu_fast_small.py tests/test_gpu_fast_multisp.py > gpurun_out/r5q/pytest.txt 2>&1 || { tail -30 gpurun_out/r5q/pytest.txt; exit 1; }
tail -2 gpurun_out/r5q/pytest.txt
for i in 1 2; do
  for K in 4 1; do
    XM_FAST_IO_MINTR=$K timeout -k 10 300 python3 tools/bench_configs.py s16rs1 s16rs2 s16rs3 planar2 conv2 --steps 20 --warmup 3 --no-box > gpurun_out/r5q/ab_$K.txt 2>&1 || { tail -5 gpurun_out/r5q/ab_$K.txt; exit 1; }
    grep '^{' gpurun_out/r5q/ab_$K.txt | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('mintr=$K', d['config'], d.get('kernel'), d['ms_per_step'], d['roofline']['frac'], d.get('parity_check'))" | tee -a gpurun_out/r5q/ab.txt
  done
done
