#!/bin/bash
# Round 5, box pass g: the 320/147 fused kernel (tests, the UP kernel it shares
# its tables' generator with, bench lines).
set -o pipefail
mkdir -p gpurun_out/r5g
timeout -k 10 900 python -u -m pytest tests/test_gpu_fast_u2.py tests/test_gpu_fast_up.py tests/test_gpu_fast_small.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5g/pytest.txt 2>&1 || { tail -30 gpurun_out/r5g/pytest.txt; exit 1; }
tail -2 gpurun_out/r5g/pytest.txt
timeout -k 10 600 python3 tools/bench_configs.py r44to96 r22to48 up --steps 10 --warmup 3 > gpurun_out/r5g/configs.jsonl 2>&1 || { tail -5 gpurun_out/r5g/configs.jsonl; exit 1; }
grep '^{' gpurun_out/r5g/configs.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['config'], d['ms_per_step'], d['roofline']['frac'], d.get('kernel'), d.get('parity_check'))"
